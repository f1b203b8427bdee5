#!/bin/bash
# End-of-round measurement, in stages that each fit one gpurun call (ROUND_TAG names the set):
#   STAGE=round   tools/gpu_round.sh: PMC passes of C2 / C3 / C4 and C2's per-rank share at
#                 N = 8, the default bench line (C2 + secondary C3 / C4) and its kernel trace
#   STAGE=configs tools/gpu_configs.sh (C2..C5 lines, share proxies) + tools/gpu_interactive.sh
#   STAGE=checks  GPU parity suite, a 4x-size random-scene sweep, and the wide-vs-binary
#                 memory-pipe counters of the C3 / C4 stand-ins (tools/gpu_pmc_mem.sh)
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$O"
export ROUND_TAG=${ROUND_TAG:-latest}
case "${STAGE:-round}" in
round)
  SKIP_TESTS=1 PMC_WORLDS=${PMC_WORLDS:-8} bash tools/gpu_round.sh ;;
configs)
  bash tools/gpu_configs.sh || exit $?
  bash tools/gpu_interactive.sh || exit $?
  # render blocks per CU of the overlapped one-frame launches (tuning key 18), render only
  timeout -k 10 300 python tools/interactive_fps.py --rows none --frames 400 \
      --combos "${IFPS_COMBOS:-9=0;18=2;18=3;18=4;18=6}" > "$O/${ROUND_TAG}_ifps_key18.json" 2>&1
  echo "key18 rc=$?"; cat "$O/${ROUND_TAG}_ifps_key18.json" ;;
checks)
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 400 --timeout-method thread > "$O/${ROUND_TAG}_gpu_tests.log" 2>&1; rc=$?
  tail -3 "$O/${ROUND_TAG}_gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 600 python -u tools/fuzz_sweep.py --cases ${SWEEP_CASES:-600} --first 300000 --scale 4 > "$O/${ROUND_TAG}_fuzz_sweep_4x.txt" 2>&1; rc=$?
  tail -2 "$O/${ROUND_TAG}_fuzz_sweep_4x.txt"; [ $rc -eq 0 ] || exit $rc
  for s in bunny sponza; do
    PMCM_DIR=pmcm_$s/wide PMC_ARGS="--scene $s --chunk 64 --launches 1" bash tools/gpu_pmc_mem.sh || exit 1
    PMCM_DIR=pmcm_$s/binary PMC_ARGS="--scene $s --chunk 64 --launches 1 --key 16=1" bash tools/gpu_pmc_mem.sh || exit 1
  done
  python3 tools/pmc_mem_reduce.py "$O/pmcm_bunny/wide" "$O/pmcm_bunny/binary" "$O/pmcm_sponza/wide" \
      "$O/pmcm_sponza/binary" > "$O/${ROUND_TAG}_pmc_mem_wide_vs_binary.json" ;;
esac
