#!/bin/bash
# Round-4 measurement batch: wide-walk build / workgroup A/B (C3, C4 stand-ins), the phase
# clock of the wide walk (experiment build libptrace_phase.so), and the one-dispatch-per-frame
# loop with the overlapped renders' grid capped per CU (tuning key 18).
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/batch"; mkdir -p "$O"
LIBS=${LIBS:-cur,cur:17=512,cur:17=768,u3,k3,s3,all3,all3:17=768} bash tools/gpu_wide_ab.sh || exit $?
PT_LIB="$GRAFT_REPO_ROOT/opengl-path-tracing_amd/build/libptrace_phase.so" timeout -k 10 300 \
   python tools/probe.py --scene bunny --spp 64 --variants 0 --chunks 64 --rounds 1 > "$O/phase_bunny.log" 2>&1 || exit $?
echo "== phase bunny"; grep -v amdgpu.ids "$O/phase_bunny.log" | tail -3
timeout -k 10 300 python tools/interactive_fps.py --frames 400 --rows none,rgba8_present_2 \
   --combos "9=0;18=6;18=5;18=4" > "$O/ifps.json" 2> "$O/ifps.err" || exit $?
python3 -c "import json;d=json.load(open('$O/ifps.json'));[print(k, v) for k, v in d.items() if isinstance(v, dict)]"
