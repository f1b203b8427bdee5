#!/bin/bash
# Graph replay tests + a 2-rank rehearsal of the N>1 bench path on the single GPU of the
# box (gloo collective, both ranks on device 0) + C5-shaped graph bench at reduced spp.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$O"
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -k "progressive or rays_per" > "$O/tg.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 "$O/tg.log"
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
   bench.py --gpus 2 --steps 2 --warmup 1 --spp 64 --dist-backend gloo > "$O/multi2.json" 2> "$O/multi2.err"; rc=$?
echo "2-rank gloo rc=$rc"; cat "$O/multi2.json"; [ $rc -eq 0 ] || { tail -20 "$O/multi2.err"; exit $rc; }
timeout -k 10 600 python bench.py --config C5 --spp 1024 --steps 2 --warmup 1 --no-cpu-baseline > "$O/c5.json" 2> "$O/c5.err"; rc=$?
echo "C5 rc=$rc"; cat "$O/c5.json"
