#!/bin/bash
# The rest of a measurement pass after gpu_r03.sh has refreshed profiles/traffic_latest.json:
# the default bench line (now carrying this build's PMC figures), the C3/C4/C5 lines and the
# per-GPU shares (gpu_configs.sh), the interactive-loop rows and their rocprof kernel trace.
cd "$GRAFT_REPO_ROOT"; R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out"; mkdir -p "$O"
export TMPDIR=/tmp
TAG=${ROUND_TAG:-r03}
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > "$O/${TAG}_bench.json" 2> "$O/${TAG}_bench.err" || exit $?
echo "bench: $(cut -c1-160 "$O/${TAG}_bench.json")"
bash tools/gpu_configs.sh || exit $?
timeout -k 10 600 python -u tools/interactive_fps.py --frames 400 > "$O/${TAG}_interactive.json" 2> "$O/${TAG}_interactive.err" || exit $?
cat "$O/${TAG}_interactive.json"
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/${TAG}_ikt" -o run -- \
    python3 "$R/tools/interactive_fps.py" --frames 400 --rows none --combos "9=0" > "$O/${TAG}_ikt.json" 2> "$O/${TAG}_ikt.err" || exit $?
echo "interactive kt: $(cat "$O/${TAG}_ikt.json")"
