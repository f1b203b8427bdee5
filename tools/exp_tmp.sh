cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/keysweep.py --variant 4 --scene bunny --spp 64 --configs "11=40;11=48;11=56;11=60" --rounds 2 > gpurun_out/ks_wfg.log 2>&1 || exit $?
grep median gpurun_out/ks_wfg.log
