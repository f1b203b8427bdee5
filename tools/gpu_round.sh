#!/bin/bash
# Full measurement pass on one GPU box: parity tests, the PMC passes of every config the bench
# line reports (reduced on the box, so the bench line carries this build's rooflines), the
# default bench line (C2 + secondary C3/C4), and the rocprofv3 kernel-trace summary of the same
# bench command.  Each GPU step has its own time limit and the chain stops at the first
# failure that is not a plain test failure.  The profiles written on the box are copied into
# gpurun_out/profiles/ (gpurun merges only gpurun_out/ back).
#   ROUND_TAG=r05c [SKIP_TESTS=1] [PMC_CONFIGS="C2 C3 C4"] [PMC_WORLDS="8"] bash tools/gpu_round.sh
cd "$GRAFT_REPO_ROOT"; R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out"; mkdir -p "$O/profiles/pmc"
export TMPDIR=/tmp
TAG=${ROUND_TAG:-latest}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > "$O/round_tests.log" 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -3 "$O/round_tests.log"
  [ $rc -le 1 ] || exit $rc
fi
for c in ${PMC_CONFIGS:-C2 C3 C4}; do
  PMC_CONFIG=$c bash tools/gpu_pmc.sh || exit 1
  python3 tools/pmc_traffic.py "$O/pmc/$c" "$TAG" "$c" > "$O/pmc_summary_$c.json" || exit 1
done
for w in $PMC_WORLDS; do
  PMC_CONFIG=C2 PMC_WORLD=$w bash tools/gpu_pmc.sh || exit 1
  python3 tools/pmc_traffic.py "$O/pmc/C2_w$w" "$TAG" C2 world=$w > "$O/pmc_summary_C2_w$w.json" || exit 1
done
cp profiles/pmc/*.json "$O/profiles/pmc/"; cp profiles/${TAG}_pmc_*.json "$O/profiles/" 2>/dev/null
timeout -k 10 900 python bench.py > "$O/round_bench.json" 2> "$O/round_bench.err"; rc=$?
echo "bench rc=$rc"; cat "$O/round_bench.json"
[ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/round_kt" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline > "$O/round_kt_bench.json" 2> "$O/round_kt.err"; rc=$?
echo "rocprof kt rc=$rc"; cat "$O/round_kt_bench.json"
exit $rc
