#!/bin/bash
# Full GPU parity suite, then same-process key sweeps: one-frame dispatch loop and C2 launches.
#   SWEEP1="...;..." SWEEP2="...;..." bash tools/gpu_check_sweep.sh
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$O"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$O/cs_tests.log" 2>&1; rc=$?
  echo "tests rc=$rc"; tail -4 "$O/cs_tests.log"
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 python tools/keysweep.py --spp 256 --chunk 1 --rounds 3 --configs "${SWEEP1}" > "$O/cs_one.log" 2>&1 || exit $?
echo "== one-frame loop"; grep median "$O/cs_one.log"
[ -n "$SWEEP2" ] || exit 0
timeout -k 10 400 python tools/keysweep.py --spp 256 --chunk 256 --rounds 3 --configs "${SWEEP2}" > "$O/cs_long.log" 2>&1 || exit $?
echo "== 256-frame launches"; grep median "$O/cs_long.log"
