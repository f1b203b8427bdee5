#!/bin/bash
# Where the one-dispatch-per-frame loop loses against long launches: 1-frame
# work items inside long launches (tuning key 5), and the one-frame loop with the overlap knobs.
cd "$GRAFT_REPO_ROOT"; O="$GRAFT_REPO_ROOT/gpurun_out/decomp"; mkdir -p "$O"
timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_cli.py \
    tests/test_gpu_group.py > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
timeout -k 10 300 python -u tools/ab_inproc.py --libs cur,cur:5=1,cur:5=2,cur:5=4 --spp 256 --chunk 256 --rounds 3 \
    > "$O/items.txt" 2>&1 || { tail -20 "$O/items.txt"; exit 1; }
tail -4 "$O/items.txt"
timeout -k 10 300 python -u tools/interactive_fps.py --rows none --frames 400 \
    --combos "9=0;9=1;18=7;4=512;4=128" > "$O/ifps.json" 2>&1 || { tail -20 "$O/ifps.json"; exit 1; }
tail -30 "$O/ifps.json"
