#!/bin/bash
# Round-4 session B: the batch sweep (tools/bsweep.sh, B = 1 .. 16384) and the FETCH_SIZE
# calibration probe; results under gpurun_out/ (copied to profiles/r04_bsweep, profiles/r04_fcal).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/fetch_calib.sh || exit 1
bash tools/bsweep.sh 20 1 8 64 512 4096 16384 || exit 1
