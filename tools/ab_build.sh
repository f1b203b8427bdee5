#!/bin/bash
# Builds the library of git revision REV as opengl-path-tracing_amd/build/libptrace_TAG.so
# (in-tree, so it travels to the GPU box) for same-box A/B timing with tools/ab.py.
#   tools/ab_build.sh HEAD~1 base
set -e
REV=$1; TAG=$2
R=$(cd "$(dirname "$0")/.." && pwd)
W=$(mktemp -d /tmp/ab_XXXX)
git -C "$R" archive "$REV" opengl-path-tracing_amd include | tar -x -C "$W"
make -s -C "$W/opengl-path-tracing_amd" -j8 build/libptrace.so
cp "$W/opengl-path-tracing_amd/build/libptrace.so" "$R/opengl-path-tracing_amd/build/libptrace_$TAG.so"
rm -rf "$W"
echo "built $REV -> build/libptrace_$TAG.so"
