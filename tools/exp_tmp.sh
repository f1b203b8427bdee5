cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python tools/probe.py --spp 128 --variants 0 --chunks 128 --rounds 2 --tunings 52:44:1:7:0:8,56:44:1:7:0:8,60:44:1:7:0:8,56:48:1:7:0:8,56:40:1:7:0:8,52:44:1:7:0:12,56:44:1:7:0:12,60:48:1:7:0:12,48:40:1:7:0:8 > gpurun_out/sweep.log 2>&1; echo "rc=$?"; grep "^round 1" gpurun_out/sweep.log | cut -c1-80
