cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/acc"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1; rc=$?
tail -2 "$O/tests.log"; [ $rc -eq 0 ] || exit $rc
for lib in acc1 cur; do
  L="$GRAFT_REPO_ROOT/opengl-path-tracing_amd/build/libptrace.so"; [ $lib = cur ] || L="$GRAFT_REPO_ROOT/opengl-path-tracing_amd/build/libptrace_$lib.so"
  PT_LIB=$L PT_LIB_PARTIAL=1 timeout -k 10 300 python tools/interactive_fps.py --frames 400 --rows none,rgba8_present_2 --combos "9=0;18=6;18=6,9=3" > "$O/ifps_$lib.json" 2> "$O/ifps_$lib.err" || exit $?
  echo "== $lib"; python3 -c "import json;d=json.load(open('$O/ifps_$lib.json'));[print(k, v) for k, v in d.items() if isinstance(v, dict)]"
done
