#!/bin/bash
# usage: SWEEP_SCENES="bunny sponza" SWEEP_TUNE="..." bash tools/gpu_sweep.sh
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for s in ${SWEEP_SCENES:-bunny}; do
  timeout -k 10 900 python tools/probe.py --scene $s --spp ${SWEEP_SPP:-32} --variants ${SWEEP_VARIANTS:-0} --chunks ${SWEEP_CHUNK:-32} --rounds 1 --tunings ${SWEEP_TUNE:-32:48} > gpurun_out/sweep_$s.log 2>&1; rc=$?; echo "sweep $s rc=$rc"; grep round gpurun_out/sweep_$s.log
  [ $rc -eq 0 ] || exit $rc
done
