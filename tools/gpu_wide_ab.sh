#!/bin/bash
# Same-process A/B of wide-walk builds / tuning keys on the C3 and C4 stand-ins (1080p, 64 spp).
#   LIBS="cur,u3,cur:17=768" bash tools/gpu_wide_ab.sh   (runs the GPU parity suite first
#   unless NOTEST=1)
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/wide_ab"; mkdir -p "$O"
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1; rc=$?
  tail -2 "$O/tests.log"; [ $rc -eq 0 ] || exit $rc
fi
for s in ${SCENES:-bunny sponza}; do
  timeout -k 10 500 python tools/ab_inproc.py --libs ${LIBS:-cur} --scene $s --spp ${SPP:-64} --chunk ${SPP:-64} --rounds ${ROUNDS:-3} > "$O/ab_$s.log" 2>&1 || exit $?
  echo "== $s"; grep -E "median|differ" "$O/ab_$s.log"
done
