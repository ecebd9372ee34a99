#!/bin/bash
# One GPU-box measurement session, parameterised (replaces the per-session tools/r04_*.sh):
#   bash tools/session.sh NAME STEP [STEP ...]
# Every step runs under its own time limit; the steps are chained and the session stops at
# the first failure (no GPU step after a fault, abort or timeout).  Output: gpurun_out/NAME/.
# Steps:
#   tests[:A,B,...]     pytest -m gpu (optionally -k "A or B or ...")
#   smoke               __graft_entry__.smoke()
#   bench[:ARGS]        bench.py --steps 20 --warmup 5 ARGS (ARGS: comma-separated, e.g. bench:--cut-proof,--no-cpu)
#   quick[:ARGS]        bench.py --steps 5 --warmup 2, tracking only (no CPU / detection / host-fed / B=1 legs)
#   ab:DIR1+DIR2+...    tools/ab_bench.sh over library dirs (built with tools/variant.sh; "default" = in-tree)
#   bsweep:B1+B2+...    tools/bsweep.sh 20 B1 B2 ...
#   cfg                 tools/cfg_lines.sh (cfg3 / cfg4 / cfg5 lines and LSD)
#   profile[:ARGS]      tools/round_profile.sh (PMC passes, bench line, rocprofv3 statistics), SKIP_TESTS=1
#   rocprof[:ARGS]      rocprofv3 --kernel-trace --stats of a tracking-only bench
#   dump:LIBDIR         a short tracking-only bench on a diagnostic build (tools/build_variant.sh) with
#                       --dump-records: step records + clock slots in $O/dump_<tag>[_clk].npy
#   fullparity[:ARGS]   bench.py --parity-seqs -1 (every sequence replayed on the oracle), short window
set -o pipefail
name=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$name
mkdir -p $O
args() { echo "$1" | tr ',' ' '; }
summary() {   # bench log -> one line
  tail -1 "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']), round(d['ms_per_step'],3), d['stage_ms'], d['kernel_ms'], d['cut_search'].get('mode'), d['cut_search'].get('exact_frac'), 'parity', d['parity_sampled']['frames'], d['parity_sampled']['mismatches'], 'b1', d.get('latency_b1_ms'))"
}
for step in "$@"; do
  kind=${step%%:*}; arg=""; [ "$kind" != "$step" ] && arg=${step#*:}
  echo "== $step"
  case $kind in
    tests)
      kexpr=$(echo "$arg" | sed "s/,/ or /g")
      timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu ${kexpr:+-k "$kexpr"} --timeout 300 --timeout-method thread \
          > $O/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error|passed|failed" $O/pytest_gpu.log | tail -15; exit 1; }
      tail -1 $O/pytest_gpu.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
      tail -1 $O/smoke.log ;;
    bench)
      timeout -k 10 900 python bench.py --steps 20 --warmup 5 $(args "$arg") > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
      summary $O/bench.log ;;
    quick)
      tag=$(echo "$arg" | tr -c 'a-zA-Z0-9_\n' '_')
      timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu --no-detect --no-host-fed --no-b1 $(args "$arg") \
          > $O/quick$tag.log 2>&1 || { tail -5 $O/quick$tag.log; exit 1; }
      summary $O/quick$tag.log ;;
    ab)
      bash tools/ab_bench.sh $O 20 $(echo "$arg" | tr '+' ' ') || exit 1 ;;
    bsweep)
      bash tools/bsweep.sh 20 $(echo "$arg" | tr '+' ' ') || exit 1
      mv gpurun_out/bsweep* $O/ ;;
    cfg)
      OUT=$O bash tools/cfg_lines.sh || exit 1 ;;
    profile)
      SKIP_TESTS=1 OUT=$O/profile bash tools/round_profile.sh $(args "$arg") || exit 1 ;;
    rocprof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o prof -f csv -- python3 bench.py --steps 5 --warmup 2 \
          --no-cpu --no-detect --no-host-fed --no-b1 --parity-seqs 0 $(args "$arg") > $O/rocprof.log 2>&1 \
          || { tail -5 $O/rocprof.log; exit 1; }
      find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
      cut -d, -f1-4 $O/kernel_stats.csv | head -14 ;;
    dump)
      tag=$(basename $arg)
      GFPL_LIB_DIR=$(realpath $arg) timeout -k 10 400 python bench.py --steps 3 --warmup 2 --batch 16384 --distinct 16384 --no-cpu \
          --no-detect --no-host-fed --no-b1 --proven-steps 0 --parity-seqs 0 --dump-records $O/dump_$tag.npy \
          > $O/dump_$tag.log 2>&1 || { tail -5 $O/dump_$tag.log; exit 1; }
      summary $O/dump_$tag.log
      python3 tools/cut_phases.py $O/dump_${tag}_clk.npy || true
      python3 tools/sp_phases.py $O/dump_${tag}_clk.npy || true ;;
    fullparity)
      tag=$(echo "$arg" | tr -c 'a-zA-Z0-9_\n' '_')
      timeout -k 10 900 python -u bench.py --steps 3 --warmup 2 --parity-seqs -1 --no-cpu --no-detect --no-host-fed \
          --no-b1 --proven-steps 0 $(args "$arg") > $O/fullparity$tag.log 2>&1 || { tail -5 $O/fullparity$tag.log; exit 1; }
      summary $O/fullparity$tag.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
