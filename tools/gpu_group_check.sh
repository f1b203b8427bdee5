cd "$GRAFT_REPO_ROOT"; O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_group.py tests/test_gpu_cli.py tests/test_gpu_lifecycle.py -x -v --timeout 200 --timeout-method thread > $O/g2_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -25 $O/g2_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --dist-backend gloo > $O/g2_bench2.json 2> $O/g2_bench2.err; rc=$?
echo "bench2 rc=$rc"; cat $O/g2_bench2.json; tail -5 $O/g2_bench2.err
exit $rc
