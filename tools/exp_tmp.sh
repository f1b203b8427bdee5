cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/keysweep.py --variant 4 --spp 64 --configs "11=40;11=16;11=24;11=32;11=52;12=48,13=48;10=1024" --rounds 2 > gpurun_out/ks_a.log 2>&1 || exit $?
grep median gpurun_out/ks_a.log
