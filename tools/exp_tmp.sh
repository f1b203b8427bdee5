cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fastmath.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/ab.py --libs base,cur --rounds 3 -- --spp 128 --variants 0 --chunks 128 --rounds 1 > gpurun_out/ab.log 2>&1; echo "ab rc=$?"; cat gpurun_out/ab.log
