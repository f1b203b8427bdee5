cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/keysweep.py --variant 5 --spp 64 --configs "1=44;1=16;1=16,12=32;1=8,12=16,11=8;1=30,12=48" --rounds 2 > gpurun_out/ks_v5.log 2>&1 || exit $?
grep median gpurun_out/ks_v5.log
