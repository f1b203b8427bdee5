#!/bin/bash
# PMC passes for the render launch of one bench configuration (PMC_CONFIG, default C2; PMC_WORLD
# for rank 0's share at N GPUs), each counter group in its own rocprofv3 run (--pmc is never
# combined with trace domains; MI355X_MICROARCH.md §rocprofv3 PMC slots: <= 8 SQ, 4 TCC, 4 TCP,
# 2 TA, 2 TD, 2 GRBM per run).  Output: gpurun_out/pmc/<config>[_wN]/<pass>/.
cd "$GRAFT_REPO_ROOT"; R="$GRAFT_REPO_ROOT"
CFG=${PMC_CONFIG:-C2}; WORLD=${PMC_WORLD:-1}
NAME=$CFG; [ "$WORLD" != 1 ] && NAME=${CFG}_w$WORLD
OUT="$R/gpurun_out/pmc/$NAME"; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
ARGS="--config $CFG --world $WORLD --launches ${PMC_LAUNCHES:-2} $PMC_EXTRA"
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- \
      python3 "$R/tools/pmc_run.py" $ARGS > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$NAME $name rc=$rc"; return $rc
}
run fetch FETCH_SIZE && \
run write WRITE_SIZE && \
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU && \
run sq2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_TRANS_F32 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH GRBM_GUI_ACTIVE && \
run mem TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TA_TA_BUSY_sum GRBM_GUI_ACTIVE && \
run l2 TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE || exit 1
echo "pmc $NAME done"
