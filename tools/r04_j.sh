#!/bin/bash
# Round-4 session J: cut-search step rewrite — line-cut parity tests, A/B at B = 16384 and B = 1.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04j
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v -m gpu -k "cut or bench_config or proven or kitti or outlier" --timeout 500 --timeout-method thread > $O/pytest.log 2>&1; echo "pytest rc=$?"
grep -E "passed|failed" $O/pytest.log | tail -2
bash tools/ab_bench.sh $O/ab 8 build/prev default || exit 1
for d in build/prev default; do
  tag=$(basename $d)
  if [ "$d" = default ]; then unset GFPL_LIB_DIR; else export GFPL_LIB_DIR=$(realpath $d); fi
  timeout -k 10 300 python bench.py --batch 1 --steps 40 --warmup 5 --no-cpu --no-detect --no-host-fed --no-b1 --parity-seqs 1 > $O/b1_$tag.log 2>&1 || { tail -5 $O/b1_$tag.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/b1_$tag.log').read().strip().splitlines()[-1]); print('B=1 $tag', round(d['ms_per_step'],3), d['kernel_ms'], d['parity_sampled']['mismatches'])"
done
