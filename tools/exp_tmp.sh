cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python tools/probe.py --spp 128 --variants 0 --chunks 128 --rounds 3 --tunings 48:44,48:40,52:40,52:44,56:40,56:44,48:36,60:40 > gpurun_out/sweep.log 2>&1; echo "rc=$?"; grep round gpurun_out/sweep.log
