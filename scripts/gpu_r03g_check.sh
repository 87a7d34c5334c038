#!/bin/bash
# Round-3 training-glue changes: the weight-gradient and table tests, every field parity test (x3 tables
# feed them), then the train.py-step benches. Every step under its own time limit; the first failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03g}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_parity.py -x -v --timeout 180 \
  --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest.log | head -20; exit $rc; }
for c in default default_mv; do
  timeout -k 10 300 python -u bench.py --mode train --conf $c --steps 20 --warmup 5 > $OUT/bench_train_$c.log 2>&1
  rc=$?; tail -1 $OUT/bench_train_$c.log | cut -c1-300; echo; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/tprof -o train -- python bench.py --mode train --conf default_mv --train-modes hip --steps 10 --warmup 3 > $OUT/tprof.log 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "train rocprof rc=$rc"; exit $rc; }
find $OUT/tprof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/train_mv_kernel_stats.csv
head -8 $OUT/train_mv_kernel_stats.csv | cut -c1-150
