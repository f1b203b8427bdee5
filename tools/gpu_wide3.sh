#!/bin/bash
# Wide walk: parity suite, unroll / stack-depth A/B (branchy visit), and the vector-memory PMC
# profile of the C3 stand-in with the wide walk and with the binary walk (key 16 = 1).
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/wide3"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1; rc=$?
tail -2 "$O/tests.log"; [ $rc -eq 0 ] || exit $rc
for s in bunny sponza; do
  timeout -k 10 400 python tools/ab_inproc.py --libs cur,u1,u3,u4,k3,cur:16=1 --scene $s --spp 64 --chunk 64 --rounds 3 > "$O/ab_$s.log" 2>&1 || exit $?
  echo "== $s builds"; grep -E "median|differ" "$O/ab_$s.log"
done
export PMC_SEGMENTS=1
PMCM_DIR=wide3/pmcm_wide PMC_ARGS="--scene bunny --chunk 64 --launches 1" bash tools/gpu_pmc_mem.sh || exit 1
PMCM_DIR=wide3/pmcm_bin PMC_ARGS="--scene bunny --chunk 64 --launches 1 --key 16=1" bash tools/gpu_pmc_mem.sh || exit 1
python3 tools/pmc_mem_reduce.py gpurun_out/wide3/pmcm_wide gpurun_out/wide3/pmcm_bin > "$O/pmc_mem.json"
grep -h segments gpurun_out/wide3/pmcm_wide/m1.log gpurun_out/wide3/pmcm_bin/m1.log
