#!/bin/bash
# Per-GPU share of the global-memory configs: rank 0 of a WORLD-way row split rendered alone
# on one GPU (tools/probe.py --world), for the C3 / C4 stand-ins at 256 spp in one launch.
#   SHARE_SCENES="bunny sponza" SHARE_WORLDS="1 8" bash tools/gpu_share.sh
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/share"; mkdir -p "$O"
for s in ${SHARE_SCENES:-bunny sponza}; do
  for w in ${SHARE_WORLDS:-1 8}; do
    timeout -k 10 300 python tools/probe.py --scene $s --world $w --spp 256 --variants 0 --chunks 256 --rounds 2 \
        > "$O/$s.w$w.log" 2>&1 || exit $?
    echo "$s world $w: $(grep '^round 1' "$O/$s.w$w.log" | cut -c1-100)"
    grep '^variant' "$O/$s.w$w.log" | cut -c1-300
  done
done
