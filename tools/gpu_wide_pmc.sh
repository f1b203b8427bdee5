#!/bin/bash
# Vector-memory and L2 PMC profile of the global-memory walk (C3 stand-in, 64 frames): the wide
# walk (default) and the binary walk (tuning key 16 = 1), same build.
cd "$GRAFT_REPO_ROOT"; R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/wide_pmc"; mkdir -p "$O"
export TMPDIR=/tmp PMC_SEGMENTS=1
PMCM_DIR=wide_pmc/wide PMC_ARGS="--scene bunny --chunk 64 --launches 1" bash tools/gpu_pmc_mem.sh || exit 1
PMCM_DIR=wide_pmc/bin PMC_ARGS="--scene bunny --chunk 64 --launches 1 --key 16=1" bash tools/gpu_pmc_mem.sh || exit 1
for v in wide:0 bin:1; do
  n=${v%%:*}; k=${v#*:}
  (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE \
     --output-format csv -d "$O/$n/l2" -o run -- python3 "$R/tools/pmc_run.py" --scene bunny --chunk 64 --launches 1 \
     --key 16=$k > "$O/$n/l2.log" 2>&1) || exit $?
done
python3 tools/pmc_mem_reduce.py "$O/wide" "$O/bin" > "$O/pmc_mem.json"
grep -h segments "$O/wide/m1.log" "$O/bin/m1.log"
