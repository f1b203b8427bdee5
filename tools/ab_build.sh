#!/bin/bash
# Builds the library of git revision REV as opengl-path-tracing_amd/build/libptrace_TAG.so
# (in-tree, so it travels to the GPU box) for same-box A/B timing with tools/ab.py.
#   tools/ab_build.sh HEAD~1 base
#   PT_EXTRA="-DFOO=1" tools/ab_build.sh . foo    (REV "." = the working tree)
set -e
REV=$1; TAG=$2
R=$(cd "$(dirname "$0")/.." && pwd)
W=$(mktemp -d /tmp/ab_XXXX)
if [ "$REV" = "." ]; then
  mkdir -p "$W/opengl-path-tracing_amd"
  cp -r "$R/include" "$W/"; cp -r "$R/opengl-path-tracing_amd/csrc" "$R/opengl-path-tracing_amd/Makefile" "$W/opengl-path-tracing_amd/"
else
  git -C "$R" archive "$REV" opengl-path-tracing_amd include | tar -x -C "$W"
fi
make -s -C "$W/opengl-path-tracing_amd" -j8 build/libptrace.so PT_EXTRA="$PT_EXTRA"
cp "$W/opengl-path-tracing_amd/build/libptrace.so" "$R/opengl-path-tracing_amd/build/libptrace_$TAG.so"
rm -rf "$W"
echo "built $REV -> build/libptrace_$TAG.so"
