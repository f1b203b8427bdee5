cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/keysweep.py --scene bunny --spp 64 --configs "3=6;3=7;3=8;3=5" --rounds 2 > gpurun_out/ks_c3w.log 2>&1 || exit $?
grep median gpurun_out/ks_c3w.log
timeout -k 10 300 python -u tools/keysweep.py --scene sponza --spp 64 --configs "3=6;3=7;3=8" --rounds 2 > gpurun_out/ks_c4w.log 2>&1 || exit $?
grep median gpurun_out/ks_c4w.log
