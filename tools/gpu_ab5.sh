#!/bin/bash
# Same-process A/B of base vs the working tree's library over launch shapes (C2, C3, C4, short
# launches, the world-8 share, 4K), each case its own ab_inproc run.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/ab5"; mkdir -p "$O"
LIBS=${AB_LIBS:-base,cur}
run() { name=$1; shift; timeout -k 10 300 python -u tools/ab_inproc.py --libs $LIBS --rounds 3 "$@" > "$O/$name.log" 2>&1 || exit $?; echo "$name:"; grep median "$O/$name.log"; }
run c2 --spp 1024 --chunk 1024
run c3 --scene bunny --spp 256 --chunk 256
run c4 --scene sponza --spp 256 --chunk 256
run c3_f1 --scene bunny --spp 16 --chunk 1
run c3_f16 --scene bunny --spp 32 --chunk 16
run c2_w8 --spp 1024 --chunk 1024 --world 8
run c2_4k --spp 256 --chunk 256 --width 3840 --height 2160
run c2_f4 --spp 64 --chunk 4
