#!/bin/bash
# Round-4 session W: the full measurement session (tools/round_profile.sh: -m gpu suite, PMC passes,
# default bench line, rocprofv3 kernel statistics) and smoke on the round's tree.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/r04w} bash tools/round_profile.sh || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > ${OUT:-gpurun_out/r04w}/smoke.log 2>&1; echo "smoke rc=$?"
tail -1 ${OUT:-gpurun_out/r04w}/smoke.log
