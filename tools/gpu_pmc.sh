#!/bin/bash
# PMC passes for the render kernel, each counter group in its own rocprofv3 run
# (--pmc is never combined with trace domains; MI355X_MICROARCH.md §rocprofv3 PMC slots).
cd "$GRAFT_REPO_ROOT"; R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/pmc"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
ARGS=${PMC_ARGS:-"--chunk 1024 --launches 2"}
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- \
      python3 "$R/tools/pmc_run.py" $ARGS > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
run fetch FETCH_SIZE && \
run write WRITE_SIZE && \
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU && \
run sq2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_TRANS_F32 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH GRBM_GUI_ACTIVE
echo "pmc done"
[ -n "$PMC_MIX" ] && run sq3 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS
echo "mix done"
