#!/bin/bash
# Secondary measurements on one GPU: the bench line of C3/C4/C5 and the per-GPU share proxy of
# the configs BASELINE sends to several GPUs -- rank 0 of an N-way row split rendered alone
# (bench.py --share-of N, its own launch shape and code path, no collective): C2 at N = 2/4/8,
# C4 and C5 at N = 8.  Each GPU step has its own limit; tools/configs_summary.py collects
# the lines into gpurun_out/cfg/configs.json.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/cfg"; mkdir -p "$O"
run() {  # name args...
  local name=$1; shift
  timeout -k 10 600 python bench.py --no-cpu-baseline --no-cold --secondary none "$@" > "$O/$name.json" 2> "$O/$name.err" || return $?
  echo "$name $(python3 -c "import json;d=json.load(open('$O/$name.json'));print(d['value'],d['ms_per_frame'])")"
}
for c in ${CONFIGS:-C2 C3 C4 C5}; do run $c --config $c || exit $?; done
for s in ${SHARES:-C2:2 C2:4 C2:8 C4:8 C5:8}; do
  c=${s%%:*}; w=${s##*:}
  run ${c}_share$w --config $c --share-of $w --steps ${SHARE_STEPS:-3} || exit $?
done
python3 tools/configs_summary.py "$O" > "$O/configs.json"
