#!/bin/bash
# PMC comparison of library builds (A/B): for each build in $LIBS (cur = build/libptrace.so,
# other = build/libptrace_<name>.so) one rocprofv3 --pmc pass per counter group over
# tools/pmc_run.py.  Reduce with: python3 tools/pmc_ab.py gpurun_out/pmcab
cd "$GRAFT_REPO_ROOT"; R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/pmcab"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
B="$R/opengl-path-tracing_amd/build"
G1=${PMC_G1:-"SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_IFETCH GRBM_GUI_ACTIVE"}
G2=${PMC_G2:-"SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_LDS_IDX_ACTIVE"}
for l in ${LIBS:-base cur}; do
  lib="$B/libptrace_$l.so"; [ "$l" = cur ] && lib="$B/libptrace.so"
  for g in 1 2; do
    eval cs=\$G$g
    PT_LIB="$lib" timeout -k 10 300 rocprofv3 --kernel-trace --pmc $cs --output-format csv -d "$OUT/${l}_g$g" -o run -- \
        python3 "$R/tools/pmc_run.py" ${PMC_ARGS:---chunk 128 --launches 2} > "$OUT/${l}_g$g.log" 2>&1
    rc=$?; echo "$l g$g rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
