#!/bin/bash
# Same-process A/B of prebuilt libraries (tools/ab_build.sh) on C2 (1024-frame launch, the
# bench's shape) and optionally C3, then the interactive loop of the working tree's library.
#   AB_LIBS=base,head,cur AB_C3=1 AB_IFPS=1 bash tools/gpu_ab3.sh
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$O"
TAG=${ROUND_TAG:-ab}
if [ -n "$AB_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > "$O/${TAG}_tests.log" 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -2 "$O/${TAG}_tests.log"
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$AB_LIBS" ]; then
  timeout -k 10 400 python -u tools/ab_inproc.py --libs $AB_LIBS --rounds ${AB_ROUNDS:-5} --spp ${AB_SPP:-1024} --chunk ${AB_SPP:-1024} > "$O/${TAG}_c2.log" 2>&1 || exit $?
  echo "C2:"; grep median "$O/${TAG}_c2.log"
fi
if [ -n "$AB_C3" ]; then
  timeout -k 10 400 python -u tools/ab_inproc.py --libs ${AB_LIBS:-base,cur} --rounds 3 --scene bunny --spp 64 --chunk 64 > "$O/${TAG}_c3.log" 2>&1 || exit $?
  echo "C3:"; grep median "$O/${TAG}_c3.log"
fi
if [ -n "$AB_IFPS" ]; then
  timeout -k 10 300 python tools/interactive_fps.py --frames 400 --rows none --combos "${IFPS_COMBOS:-9=0;9=1}" > "$O/${TAG}_ifps.json" 2> "$O/${TAG}_ifps.err" || exit $?
  cat "$O/${TAG}_ifps.json"
fi
