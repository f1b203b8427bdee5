#!/bin/bash
# LDS bank-conflict attribution: one PMC pass of C2's 1024-frame launch per
# diagnostic build -- cur, triangles from HBM (dtri: -DPT_DIAG_TRIS_GLOBAL), materials + spheres
# from HBM (dshade: -DPT_DIAG_SHADE_GLOBAL), both (dboth) -- built beforehand with
# PT_EXTRA=... bash tools/ab_build.sh . <name>.  Summary: python3 tools/lds_attr.py.
cd "$GRAFT_REPO_ROOT"; R="$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; cd /tmp
for L in cur dtri dshade dboth; do
  if [ $L = cur ]; then export PT_LIB=$R/opengl-path-tracing_amd/build/libptrace.so PT_LIB_PARTIAL=0
  else export PT_LIB=$R/opengl-path-tracing_amd/build/libptrace_$L.so PT_LIB_PARTIAL=1; fi
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d $R/gpurun_out/ldsattr/$L -o run -- python3 $R/tools/pmc_run.py --config C2 --launches 1 > $R/gpurun_out/ldsattr_$L.log 2>&1 || exit $?
  echo "$L done"
done
