cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=16:24:1:6:0:6,16:24:1:7:0:6,16:24:1:8:0:6
timeout -k 10 900 python tools/probe.py --scene bunny --spp 64 --variants 0 --chunks 64 --rounds 2 --tunings $T > gpurun_out/sweep3.log 2>&1; echo "rc=$?"; grep "^round 1" gpurun_out/sweep3.log | cut -c1-80
timeout -k 10 900 python tools/probe.py --scene sponza --spp 32 --variants 0 --chunks 32 --rounds 2 --tunings $T > gpurun_out/sweep4.log 2>&1; echo "rc=$?"; grep "^round 1" gpurun_out/sweep4.log | cut -c1-80
