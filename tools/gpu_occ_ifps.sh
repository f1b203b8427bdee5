cd "$GRAFT_REPO_ROOT"
NOTEST=1 LIBS=cur,cur:3=5,cur:3=7 bash tools/gpu_wide_ab.sh || exit $?
O="$GRAFT_REPO_ROOT/gpurun_out/ifps_bunny"; mkdir -p "$O"
timeout -k 10 300 python tools/interactive_fps.py --scene bunny --frames 200 --rows none --combos "18=0;18=8;18=4" > "$O/ifps.json" 2> "$O/ifps.err" || exit $?
python3 -c "import json;d=json.load(open('$O/ifps.json'));[print(k, v) for k, v in d.items() if isinstance(v, dict)]"
