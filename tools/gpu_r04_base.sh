#!/bin/bash
# Round-4 baseline on the current build: counting stats + rates of the global-memory walk
# (C3 / C4 stand-ins) and C2, same box.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/base"; mkdir -p "$O"
for s in bunny sponza; do
  timeout -k 10 300 python tools/probe.py --scene $s --spp 64 --chunks 64 --rounds 2 > "$O/$s.log" 2>&1 || exit $?
  grep -E "nodes/seg|^round" "$O/$s.log"
done
timeout -k 10 300 python tools/probe.py --scene cornell --spp 128 --chunks 128 --rounds 2 > "$O/cornell.log" 2>&1 || exit $?
grep -E "nodes/seg|^round" "$O/cornell.log"
