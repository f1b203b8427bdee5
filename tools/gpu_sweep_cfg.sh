#!/bin/bash
# 2,000-case seeded random-scene sweep (HIP vs oracle, variants 0 and 3: the wide walk on every
# global-memory case), then the C3 / C4 / C5 bench lines and the per-GPU-share probes.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$O"
timeout -k 10 600 python -u tools/fuzz_sweep.py --cases ${SWEEP_CASES:-2000} --first ${SWEEP_FIRST:-300000} --scale 4 \
    > "$O/sweep.txt" 2>&1; rc=$?
tail -2 "$O/sweep.txt"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_configs.sh
