#!/bin/bash
# Round-3 measurement pass: GPU parity tests, PMC passes (reduced so the bench line carries this
# build's VALU / traffic figures), the default bench line, and the rocprofv3 kernel-trace summary
# of the same bench command.  Each GPU step has its own time limit; the chain stops at the first
# step that did not finish cleanly (a plain test failure, rc 1, still lets the measurement run).
cd "$GRAFT_REPO_ROOT"; R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out"; mkdir -p "$O"
export TMPDIR=/tmp
TAG=${ROUND_TAG:-r03}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread ${PYTEST_ARGS} \
      > "$O/${TAG}_tests.log" 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -5 "$O/${TAG}_tests.log"
  [ $rc -le 1 ] || exit $rc
fi
[ -n "$TESTS_ONLY" ] && exit 0
PMC_ARGS="--chunk 1024 --launches 2" bash tools/gpu_pmc.sh || exit 1
python3 tools/pmc_traffic.py "$O/pmc" "$TAG" > "$O/${TAG}_pmc_summary.json" || exit 1
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > "$O/${TAG}_bench.json" 2> "$O/${TAG}_bench.err"; rc=$?
echo "bench rc=$rc"; cat "$O/${TAG}_bench.json"
[ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/${TAG}_kt" -o run -- \
    python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-cold > "$O/${TAG}_kt_bench.json" 2> "$O/${TAG}_kt.err"; rc=$?
echo "rocprof kt rc=$rc"; cat "$O/${TAG}_kt_bench.json"
exit $rc
