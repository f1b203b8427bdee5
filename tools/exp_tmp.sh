cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python tools/probe.py --spp 1024 --variants 0 --chunks 1024 --rounds 2 --tunings 52:44,48:44,44:44,56:44,48:40,52:48 > gpurun_out/sweep.log 2>&1; echo "rc=$?"; grep "^round 1" gpurun_out/sweep.log | cut -c1-80
