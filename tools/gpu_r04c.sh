#!/bin/bash
# One call for a changed default of the short-launch path: its lifecycle / viewer tests, a
# per-build loop A/B against build/libptrace_s2.so, then the full round measurement (r04c) and
# the C3 / C4 / C5 / per-GPU-share lines of the same build.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lifecycle.py \
    tests/test_viewer.py > "$O/s3_tests.log" 2>&1 || { tail -30 "$O/s3_tests.log"; exit 1; }
tail -1 "$O/s3_tests.log"
LIBS=s2,cur ROUNDS=2 ROWS=none,rgba8_present_1,rgba8_present_2 bash tools/gpu_ifps_libs.sh || exit 1
IFPS_ARGS="--scene bunny" LIBS=s2,cur ROUNDS=1 ROWS=none FRAMES=100 bash tools/gpu_ifps_libs.sh || exit 1
ROUND_TAG=r04c bash tools/gpu_final.sh || exit 1
bash tools/gpu_configs.sh
