#!/bin/bash
# The one-dispatch-per-frame loop (tools/interactive_fps.py, render only) of several builds,
# one process per build (overlapped launches of two builds in one process share hardware
# queues), ROUNDS times in alternation.   LIBS=cur,ce1 ROUNDS=2 bash tools/gpu_ifps_libs.sh
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/ifps_libs"; mkdir -p "$O"
B="$GRAFT_REPO_ROOT/opengl-path-tracing_amd/build"
for r in $(seq 1 ${ROUNDS:-2}); do
  for l in ${LIBS//,/ }; do
    lib="$B/libptrace_$l.so"; [ "$l" = cur ] && lib="$B/libptrace.so"
    PT_LIB="$lib" timeout -k 10 200 python -u tools/interactive_fps.py --rows ${ROWS:-none} --frames ${FRAMES:-600} \
        --combos "${COMBOS:-9=0}" ${IFPS_ARGS} > "$O/$l.$r.json" 2>&1 || { tail -20 "$O/$l.$r.json"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], {k: v['ms_per_frame'] for k, v in d.items() if isinstance(v, dict)})" "$O/$l.$r.json" "$l.$r"
  done
done
