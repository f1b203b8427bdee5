#!/bin/bash
# The one-dispatch-per-frame loop: lifecycle/viewer parity tests, then tools/interactive_fps.py
# (overlap on / off) and its rocprofv3 kernel-trace summary.
cd "$GRAFT_REPO_ROOT"; R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out"; mkdir -p "$O"
export TMPDIR=/tmp
TAG=${ROUND_TAG:-r03}
timeout -k 10 600 python -u -m pytest tests/test_gpu_lifecycle.py tests/test_viewer.py tests/test_gpu_parity.py -x -q \
    --timeout 200 --timeout-method thread > "$O/${TAG}_ifps_tests.log" 2>&1; rc=$?
echo "tests rc=$rc"; tail -4 "$O/${TAG}_ifps_tests.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/interactive_fps.py --frames ${IFPS_FRAMES:-400} > "$O/${TAG}_ifps.json" 2> "$O/${TAG}_ifps.err"; rc=$?
echo "ifps rc=$rc"; cat "$O/${TAG}_ifps.json"
[ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/${TAG}_ifps_kt" -o run -- \
    python3 "$R/tools/interactive_fps.py" --frames 200 --rows none > "$O/${TAG}_ifps_kt.json" 2> "$O/${TAG}_ifps_kt.err"; rc=$?
echo "kt rc=$rc"; cat "$O/${TAG}_ifps_kt.json"
exit $rc
