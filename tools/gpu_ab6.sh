#!/bin/bash
# Short-launch A/B with the library order reversed, and each library alone in its process.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/ab6"; mkdir -p "$O"
run() { name=$1; libs=$2; shift 2; timeout -k 10 300 python -u tools/ab_inproc.py --libs $libs --rounds 3 "$@" > "$O/$name.log" 2>&1 || exit $?; echo "$name:"; grep median "$O/$name.log"; }
run c2_f4_rev cur,base --spp 64 --chunk 4
run c3_f1_rev cur,base --scene bunny --spp 16 --chunk 1
run c2_f4_base base --spp 64 --chunk 4
run c2_f4_cur cur --spp 64 --chunk 4
run c3_f1_base base --scene bunny --spp 16 --chunk 1
run c3_f1_cur cur --scene bunny --spp 16 --chunk 1
run c3_f16_base base --scene bunny --spp 32 --chunk 16
run c3_f16_cur cur --scene bunny --spp 32 --chunk 16
