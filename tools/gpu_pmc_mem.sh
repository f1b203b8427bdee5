#!/bin/bash
# PMC passes on the vector-memory pipeline (TA / TD / TCP, UTCL1) for a global-memory scene
# (default the C3 stand-in), each counter group in its own rocprofv3 run.
cd "$GRAFT_REPO_ROOT"; R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${PMCM_DIR:-pmcm}"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
ARGS=${PMC_ARGS:-"--scene bunny --chunk 64 --launches 1"}
run() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- \
      python3 "$R/tools/pmc_run.py" $ARGS > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
run m1 TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum GRBM_GUI_ACTIVE && \
run m2 TD_TD_BUSY_sum TD_TC_STALL_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_UTCL1_STALL_MULTI_MISS_sum GRBM_GUI_ACTIVE && \
run m3 SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE && \
run m4 TCC_HIT_sum TCC_MISS_sum SQ_WAVES SQ_INSTS_SALU SQ_THREAD_CYCLES_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE
