#!/bin/bash
# Phase-clock breakdown (experiment builds with -DPT_PHASE_CLOCK) of build/libptrace_<tag>.so.
#   PC_LIBS=pcbase,pccur bash tools/gpu_phase.sh
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$O"
for l in ${PC_LIBS//,/ }; do
  PT_LIB="$GRAFT_REPO_ROOT/opengl-path-tracing_amd/build/libptrace_$l.so" timeout -k 10 300 \
     python tools/probe.py --spp 128 --variants 0 --chunks 128 --rounds 1 ${PC_ARGS} > "$O/pc_$l.log" 2>&1 || exit $?
  echo "== $l"; grep -v amdgpu.ids "$O/pc_$l.log" | tail -4
done
