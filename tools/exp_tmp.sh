cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python tools/ab_inproc.py --libs cur,${EXP_LIBS} --rounds 4 > gpurun_out/ab_c2.log 2>&1 || exit $?
echo "C2:"; grep median gpurun_out/ab_c2.log
