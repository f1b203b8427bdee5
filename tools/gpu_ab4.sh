#!/bin/bash
# Per-GPU share A/B (rank 0 of a world-8 row split, C2 shape) of prebuilt libraries, then the
# GPU tests of the working tree's library and its C3 / C4 A/B.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$O"
TAG=${ROUND_TAG:-ab}
if [ -n "$W_LIBS" ]; then
  timeout -k 10 300 python -u tools/ab_inproc.py --libs $W_LIBS --rounds 3 --spp 1024 --chunk 1024 --world 8 > "$O/${TAG}_w8.log" 2>&1 || exit $?
  echo "w8:"; grep median "$O/${TAG}_w8.log"
fi
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > "$O/${TAG}_tests.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 "$O/${TAG}_tests.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/ab_inproc.py --libs ${C3_LIBS:-d2b,cur} --rounds 3 --scene bunny --spp 64 --chunk 64 > "$O/${TAG}_c3.log" 2>&1 || exit $?
echo "C3:"; grep median "$O/${TAG}_c3.log"
timeout -k 10 400 python -u tools/ab_inproc.py --libs ${C3_LIBS:-d2b,cur} --rounds 3 --scene sponza --spp 32 --chunk 32 > "$O/${TAG}_c4.log" 2>&1 || exit $?
echo "C4:"; grep median "$O/${TAG}_c4.log"
