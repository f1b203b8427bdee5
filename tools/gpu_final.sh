#!/bin/bash
# Round measurement: tools/gpu_round.sh (GPU parity suite, C2 PMC passes, default bench line,
# rocprofv3 kernel-trace summary of the same command), then tools/gpu_interactive.sh.
cd "$GRAFT_REPO_ROOT"
export ROUND_TAG=${ROUND_TAG:-r04}
bash tools/gpu_round.sh || exit $?
bash tools/gpu_interactive.sh
