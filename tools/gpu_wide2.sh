#!/bin/bash
# Wide walk tuning: parity suite, then same-process A/B of unroll / stack-depth builds and a
# threshold sweep (tuning keys 0 leaf, 1 shade, 6 walk floor) on the C3 / C4 stand-ins.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/wide2"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1; rc=$?
tail -2 "$O/tests.log"; [ $rc -eq 0 ] || exit $rc
for s in bunny sponza; do
  timeout -k 10 400 python tools/ab_inproc.py --libs cur,u1,u3,k1,k3,cur:16=1 --scene $s --spp 64 --chunk 64 --rounds 3 > "$O/ab_$s.log" 2>&1 || exit $?
  echo "== $s builds"; grep -E "median|differ" "$O/ab_$s.log"
  timeout -k 10 400 python tools/ab_inproc.py --libs cur,cur:0=14,cur:0=28,cur:1=16,cur:1=32,cur:6=3,cur:6=10 --scene $s --spp 64 --chunk 64 --rounds 3 > "$O/keys_$s.log" 2>&1 || exit $?
  echo "== $s keys"; grep -E "median|differ" "$O/keys_$s.log"
done
