#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -k "large_scene or rays_per" > gpurun_out/ts.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/ts.log
[ $rc -le 1 ] || exit $rc
for s in bunny sponza; do
  timeout -k 10 600 python tools/probe.py --scene $s --spp 32 --variants 0,3 --chunks 32 --rounds 1 > gpurun_out/probe_$s.log 2>&1; echo "probe $s rc=$?"; grep -v amdgpu gpurun_out/probe_$s.log
done
