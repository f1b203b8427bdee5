#!/bin/bash
# One GPU iteration: parity tests (all variants) then the variant/launch-shape probe.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/t.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/t.log
if [ $rc -le 1 ]; then
  timeout -k 10 600 python tools/probe.py ${PROBE_ARGS:---spp 64 --variants 0,3 --chunks 16,64} > gpurun_out/probe.log 2>&1; rc=$?
  echo "probe rc=$rc"; cat gpurun_out/probe.log | grep -v amdgpu.ids
fi
