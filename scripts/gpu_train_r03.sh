#!/bin/bash
# Training evidence: the gradient tests, train.py-step benches (default.conf and default_mv.conf) and a
# rocprofv3 kernel split of the default_mv step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-train}; mkdir -p $OUT
if [ -z "${NOTEST:-}" ]; then
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_train.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
for c in default default_mv; do
  timeout -k 10 300 python -u bench.py --mode train --conf $c --steps 20 --warmup 5 > $OUT/bench_train_$c.log 2>&1
  rc=$?; echo "bench $c rc=$rc"; tail -1 $OUT/bench_train_$c.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o train -- python bench.py --mode train --conf default_mv --train-modes hip --steps 10 --warmup 3 > $OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/train_mv_kernel_stats.csv
head -12 $OUT/train_mv_kernel_stats.csv | cut -c1-200
