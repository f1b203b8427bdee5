cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python tools/ab_inproc.py --libs cur,u2,u6,u8 --rounds 3 --scene bunny --spp 64 --chunk 64 > gpurun_out/ab_c3.log 2>&1 || exit $?
echo "C3:"; grep median gpurun_out/ab_c3.log
timeout -k 10 600 python tools/ab_inproc.py --libs cur,u2,u6,u8 --rounds 3 --scene sponza --spp 32 --chunk 32 > gpurun_out/ab_c4.log 2>&1 || exit $?
echo "C4:"; grep median gpurun_out/ab_c4.log
