cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/opengl-path-tracing_amd/build/libptrace_lean.so
PT_LIB=$L timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x --timeout 300 > gpurun_out/exp_tests.log 2>&1; rc=$?
echo "pytest(lean) rc=$rc"; tail -2 gpurun_out/exp_tests.log; [ $rc -eq 0 ] || exit $rc
for lib in cur lean; do
 LL=$GRAFT_REPO_ROOT/opengl-path-tracing_amd/build/libptrace.so; [ $lib = lean ] && LL=$L
 PT_LIB=$LL timeout -k 10 600 python tools/probe.py --spp 1024 --variants 0 --chunks 1024 --rounds 2 --tunings 0:0:1:7,0:0:1:8 > gpurun_out/sweep_$lib.log 2>&1; echo "$lib rc=$?"; grep "^round 1" gpurun_out/sweep_$lib.log | cut -c1-80
done
