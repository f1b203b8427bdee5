#!/bin/bash
# Parity tests of the working tree's library, then a same-process A/B (tools/ab_inproc.py)
# of build/libptrace_<tag>.so against it: C2 (Cornell, LDS walk) and, with AB_C3=1, the C3
# stand-in (global-memory walk).
#   AB_LIBS=base,cur AB_C3=1 bash tools/gpu_ab.sh
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 300 > "$O/ab_tests.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 "$O/ab_tests.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/ab_inproc.py --libs ${AB_LIBS:-base,cur} --rounds ${AB_ROUNDS:-5} > "$O/ab_c2.log" 2>&1 || exit $?
echo "C2:"; grep -v amdgpu.ids "$O/ab_c2.log" | grep median
if [ -n "$AB_C3" ]; then
  timeout -k 10 400 python -u tools/ab_inproc.py --libs ${AB_LIBS:-base,cur} --rounds 3 --scene bunny --spp 64 --chunk 64 > "$O/ab_c3.log" 2>&1 || exit $?
  echo "C3:"; grep -v amdgpu.ids "$O/ab_c3.log" | grep median
fi
