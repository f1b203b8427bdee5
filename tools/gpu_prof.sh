#!/bin/bash
# rocprofv3: kernel-trace stats of a short bench + counter list (separate runs, no --pmc mixing).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/prof
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 -L > "$R/gpurun_out/prof/counters_list.txt" 2>&1; echo "list rc=$?"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof/kt" -o run -- python3 "$R/bench.py" --spp 256 --chunk 64 --steps 2 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/prof/kt_bench.log" 2>&1; echo "kt rc=$?"
tail -3 "$R/gpurun_out/prof/kt_bench.log"
find "$R/gpurun_out/prof/kt" -name "*stats*" | head
