#!/bin/bash
# Full measurement pass: parity tests, the PMC passes (reduced on the box so the bench line
# carries this build's traffic / VALU figures), the default bench line, and the rocprofv3
# kernel-trace summary of the same bench command.  Each GPU step has its own time limit
# and the chain stops at the first failure that is not a plain test failure.
cd "$GRAFT_REPO_ROOT"; R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out"; mkdir -p "$O"
export TMPDIR=/tmp
TAG=${ROUND_TAG:-latest}
timeout -k 10 900 python -m pytest tests -q -m gpu > "$O/round_tests.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 "$O/round_tests.log"
[ $rc -le 1 ] || exit $rc
bash tools/gpu_pmc.sh || exit 1
python3 tools/pmc_traffic.py "$O/pmc" "$TAG" > "$O/pmc_summary.json" || exit 1
timeout -k 10 600 python bench.py > "$O/round_bench.json" 2> "$O/round_bench.err"; rc=$?
echo "bench rc=$rc"; cat "$O/round_bench.json"
[ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/round_kt" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline > "$O/round_kt_bench.json" 2> "$O/round_kt.err"; rc=$?
echo "rocprof kt rc=$rc"; cat "$O/round_kt_bench.json"
exit $rc
