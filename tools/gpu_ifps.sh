#!/bin/bash
# One-dispatch-per-frame loop: tools/interactive_fps.py over tuning combos,
# then a rocprofv3 kernel-trace summary of one combo.
#   IFPS_COMBOS="18=6;18=7" IFPS_KT="18=6" bash tools/gpu_ifps.sh
cd "$GRAFT_REPO_ROOT"; R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/ifps"; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 300 python tools/interactive_fps.py --frames ${IFPS_FRAMES:-400} --rows ${IFPS_ROWS:-none,rgba8_present_2} \
   --combos "${IFPS_COMBOS:-9=0}" > "$O/ifps.json" 2> "$O/ifps.err" || exit $?
python3 -c "import json;d=json.load(open('$O/ifps.json'));[print(k, v) for k, v in d.items() if isinstance(v, dict)]"
if [ -n "$IFPS_KT" ]; then
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o run -- \
      python3 "$R/tools/interactive_fps.py" --frames 300 --rows none --combos "$IFPS_KT" > "$O/kt.json" 2> "$O/kt.err" || exit $?
  cat "$O/kt.json"; cut -d, -f1-8 "$O/kt/run_kernel_stats.csv" | head -8
fi
