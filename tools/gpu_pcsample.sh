#!/bin/bash
# PC sampling of the C2 render kernel (rocprofv3 beta): which instructions the waves sit on.
# Stochastic (hardware) sampling when the device offers it, else host-trap sampling.
cd "$GRAFT_REPO_ROOT"; R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/pcs"; mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 60 rocprofv3 -L > "$O/list.txt" 2>&1; echo "list rc=$?"
grep -i -B2 -A12 "pc.sampl" "$O/list.txt" | head -60
ARGS=${PCS_ARGS:-"--chunk 64 --launches 1"}
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles \
    --pc-sampling-interval ${PCS_INTERVAL:-1048576} --output-format csv -d "$O/st" -o run -- \
    python3 "$R/tools/pmc_run.py" $ARGS > "$O/st.log" 2>&1; rc=$?
echo "stochastic rc=$rc"; tail -5 "$O/st.log"
if [ $rc -eq 1 ] || [ $rc -eq 255 ]; then
  timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
      --pc-sampling-interval ${PCS_TIME_US:-10} --output-format csv -d "$O/ht" -o run -- \
      python3 "$R/tools/pmc_run.py" $ARGS > "$O/ht.log" 2>&1; rc=$?
  echo "host_trap rc=$rc"; tail -5 "$O/ht.log"
fi
find "$O" -name "*.csv" | head; exit $rc
