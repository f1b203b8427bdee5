#!/bin/bash
# Wide global walk: GPU parity suite, then same-process A/B of the wide walk
# against the binary global walk (tuning key 16 = 1) on the C3 / C4 stand-ins.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/wide"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1; rc=$?
tail -5 "$O/tests.log"; [ $rc -eq 0 ] || exit $rc
for s in bunny sponza; do
  timeout -k 10 300 python tools/ab_inproc.py --libs cur,cur:16=1 --scene $s --spp 64 --chunk 64 --rounds 3 > "$O/ab_$s.log" 2>&1 || exit $?
  grep -E "median|differ" "$O/ab_$s.log"
done
