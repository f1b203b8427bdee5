cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python tools/probe.py --spp 128 --variants 0 --chunks 128 --rounds 2 --tunings 0:0:1:0:0:0:63,0:0:1:0:0:0:56,0:0:1:0:0:0:48,0:0:1:0:0:0:40,0:0:1:0:0:0:0 > gpurun_out/sweep.log 2>&1; echo "rc=$?"; grep "^round 1" gpurun_out/sweep.log | cut -c1-80
timeout -k 10 900 python tools/probe.py --scene bunny --spp 64 --variants 0 --chunks 64 --rounds 2 --tunings 0:0:1:0:0:0:63,0:0:1:0:0:0:48,0:0:1:0:0:0:32,0:0:1:0:0:0:0 > gpurun_out/sweep3.log 2>&1; echo "rc=$?"; grep "^round 1" gpurun_out/sweep3.log | cut -c1-80
