#!/bin/bash
# WRITE_SIZE / FETCH_SIZE per C2 launch (1024 frames) for the working tree's library and a
# prebuilt comparison build (PT_LIB), each pass its own rocprofv3 run.
cd "$GRAFT_REPO_ROOT"; R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/wamp"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for lib in cur ${WAMP_LIBS}; do
  for c in WRITE_SIZE FETCH_SIZE; do
    if [ "$lib" = cur ]; then unset PT_LIB; else export PT_LIB="$R/opengl-path-tracing_amd/build/libptrace_$lib.so"; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$OUT/${lib}_$c" -o run -- \
        python3 "$R/tools/pmc_run.py" --chunk 1024 --launches 1 > "$OUT/${lib}_$c.log" 2>&1 || exit $?
    echo "$lib $c done"
  done
done
