cd "$GRAFT_REPO_ROOT"; export PT_LIB=$GRAFT_REPO_ROOT/opengl-path-tracing_amd/build/libptrace_wt.so
for fr in 1 2 4 16 64; do echo "frames=$fr"; timeout -k 10 120 python tools/wave_trace.py --frames $fr --reps 10 || exit $?; done
