export GFPL_LIB_DIR=${LIBV:-build/cutprof}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --batch 16384 --steps 1 --warmup 0 --no-cpu > gpurun_out/cutprof.log 2>&1; rc=$?
grep -E "cutprof|cutstats|spprof" gpurun_out/cutprof.log | tail -24; exit $rc
