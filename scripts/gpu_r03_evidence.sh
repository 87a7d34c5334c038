#!/bin/bash
# Round-3 evidence at HEAD: the whole -m gpu suite, smoke(), the default bench line, rocprofv3 kernel stats of
# the bench command, and the train.py-step benches (default.conf, default_mv.conf) with a kernel split of the
# default_mv step. Every step under its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r03d}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
rc=$?; tail -1 $OUT/smoke.log; [ $rc -eq 0 ] || { echo "smoke rc=$rc"; exit $rc; }
timeout -k 10 600 python -u bench.py > $OUT/bench.log 2> $OUT/bench.err
rc=$?; tail -c 1500 $OUT/bench.log; echo; [ $rc -eq 0 ] || { echo "bench rc=$rc"; exit $rc; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o bench -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-legs --no-pmc > $OUT/prof.log 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "rocprof rc=$rc"; tail -5 $OUT/prof.log; exit $rc; }
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/bench_kernel_stats.csv
head -4 $OUT/bench_kernel_stats.csv | cut -c1-160
for c in default default_mv; do
  timeout -k 10 300 python -u bench.py --mode train --conf $c --steps 20 --warmup 5 > $OUT/bench_train_$c.log 2>&1
  rc=$?; tail -1 $OUT/bench_train_$c.log | cut -c1-300; echo; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/tprof -o train -- python bench.py --mode train --conf default_mv --train-modes hip --steps 10 --warmup 3 > $OUT/tprof.log 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "train rocprof rc=$rc"; exit $rc; }
find $OUT/tprof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/train_mv_kernel_stats.csv
head -6 $OUT/train_mv_kernel_stats.csv | cut -c1-160
