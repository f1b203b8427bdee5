#!/bin/bash
# L2 (TCC) hit rate of the global-memory walk (C3 stand-in, 64 frames), wide and binary walk,
# and a threshold re-sweep of the wide walk (keys 0 leaf, 1 shade, 6 walk floor).
cd "$GRAFT_REPO_ROOT"; R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/l2"; mkdir -p "$O"
export TMPDIR=/tmp
for v in wide:0 bin:1; do
  n=${v%%:*}; k=${v#*:}
  (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE \
     --output-format csv -d "$O/$n" -o run -- python3 "$R/tools/pmc_run.py" --scene bunny --chunk 64 --launches 1 --key 16=$k \
     > "$O/$n.log" 2>&1) || exit $?
done
python3 tools/pmc_mem_reduce.py "$O/wide" "$O/bin" > "$O/l2.json"
python3 -c "
import json; d=json.load(open('$O/l2.json'))
for k,v in d.items():
    c=v['counters']; print(k, 'TCC hit %.3f' % (c['TCC_HIT_sum']/(c['TCC_HIT_sum']+c['TCC_MISS_sum'])), 'TCC req %.3g' % (c['TCC_HIT_sum']+c['TCC_MISS_sum']), 'TCP->TCC %.3g' % c['TCP_TCC_READ_REQ_sum'])"
NOTEST=1 LIBS=cur,cur:0=16,cur:0=24,cur:1=20,cur:1=28,cur:6=4,cur:6=8 bash tools/gpu_wide_ab.sh
