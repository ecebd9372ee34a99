#!/bin/bash
# Round-4 session K: pose GN compaction — pose / outlier parity tests, A/B at B = 16384.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04k
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v -m gpu -k "pose or outlier or bench_config or stress or euroc" --timeout 500 --timeout-method thread > $O/pytest.log 2>&1; echo "pytest rc=$?"
grep -E "passed|failed" $O/pytest.log | tail -2
bash tools/ab_bench.sh $O/ab 8 build/prev default || exit 1
