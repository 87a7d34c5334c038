#!/bin/bash
# Perf-only session: fp32 vs x3 bench lines + rocprofv3 kernel stats of the x3 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -25 $OUT/pytest_gpu.log; [ $rc -le 1 ] || { echo "pytest crashed rc=$rc"; exit $rc; }
for p in x3 fp32; do
  timeout -k 10 400 python bench.py --steps 5 --warmup 2 --precision $p --no-cpu-baseline > $OUT/bench_$p.log 2>&1
  rc=$?; tail -1 $OUT/bench_$p.log; [ $rc -eq 0 ] || { echo "bench $p failed rc=$rc"; exit $rc; }
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_x3 -o bench -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/prof_x3.log 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "rocprof failed rc=$rc"; tail -5 $OUT/prof_x3.log; exit $rc; }
head -4 $OUT/prof_x3/bench_kernel_stats.csv | cut -c1-200
