cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu > gpurun_out/t1.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/t1.log
if [ $rc -le 1 ]; then
  timeout -k 10 600 python bench.py --spp 64 --chunk 16 --steps 2 --warmup 1 > gpurun_out/b1.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/b1.log
fi
