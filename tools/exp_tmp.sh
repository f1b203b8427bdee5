cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for c in 64 128 256 512; do
  timeout -k 10 300 python bench.py --config C5 --chunk $c --no-cpu-baseline --steps 2 > gpurun_out/c5_$c.json 2> gpurun_out/c5_$c.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/c5_$c.json'));print($c, d['value'], d['ms_per_frame'], d['config']['workload'][-30:])"
done
