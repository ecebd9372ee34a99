#!/bin/bash
# Round-4 session G1: FETCH_SIZE calibration, the batch sweep, the LSD measurements.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/r04_b.sh || exit 1
bash tools/r04_lsd.sh || exit 1
