cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "v3 or large_scene or c3 or -3]" > gpurun_out/t_lay.log 2>&1; rc=$?; tail -3 gpurun_out/t_lay.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/ab_inproc.py --libs base,cur --rounds 3 --scene bunny --spp 64 --chunk 64 > gpurun_out/ab_c3.log 2>&1 || exit $?
echo C3; grep median gpurun_out/ab_c3.log
timeout -k 10 400 python tools/ab_inproc.py --libs base,cur --rounds 3 --scene sponza --spp 64 --chunk 64 > gpurun_out/ab_c4.log 2>&1 || exit $?
echo C4; grep median gpurun_out/ab_c4.log
