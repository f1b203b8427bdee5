#!/bin/bash
# Secondary measurements: the bench line for C3/C4/C5 and the C2 per-GPU share at N=2/4/8
# (rank 0 of the row split rendered alone on one GPU).  Each GPU step has its own limit.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/cfg"; mkdir -p "$O"
for c in C3 C4 C5; do
  timeout -k 10 600 python bench.py --config $c --no-cpu-baseline > "$O/$c.json" 2> "$O/$c.err" || exit $?
  echo "$c $(python3 -c "import json;d=json.load(open('$O/$c.json'));print(d['value'],d['ms_per_frame'])")"
done
for w in 2 4 8; do
  timeout -k 10 600 python tools/probe.py --world $w --spp 1024 --variants 0 --chunks 1024 --rounds 2 > "$O/w$w.log" 2>&1 || exit $?
  echo "world $w: $(grep '^round 1' "$O/w$w.log" | cut -c1-90)"
done
