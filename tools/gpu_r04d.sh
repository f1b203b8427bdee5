#!/bin/bash
# Scratch-ring build: its lifecycle / viewer tests, a per-build loop A/B against
# build/libptrace_ring1.so (the previous one-entry-per-stream ring) and ring3, then the full
# round measurement (r04d) and the configs lines of the same build.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lifecycle.py \
    tests/test_viewer.py > "$O/ring_tests.log" 2>&1 || { tail -30 "$O/ring_tests.log"; exit 1; }
tail -1 "$O/ring_tests.log"
LIBS=ring1,cur,ring3 ROUNDS=2 ROWS=none,rgba8_present_2 bash tools/gpu_ifps_libs.sh || exit 1
IFPS_ARGS="--scene bunny" LIBS=ring1,cur ROUNDS=1 ROWS=none FRAMES=100 bash tools/gpu_ifps_libs.sh || exit 1
ROUND_TAG=r04d bash tools/gpu_final.sh || exit 1
bash tools/gpu_configs.sh
