#!/bin/bash
# Quick training-kernel check: gradient tests, then the training-forward timing diag and the default_mv step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-tq}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_train.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/pytest.log | head -20; exit $rc; }
timeout -k 10 120 python -u scripts/train_fwd_ab.py > $OUT/train_fwd.log 2>&1; rc=$?; grep "^\[" $OUT/train_fwd.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --mode train --conf default_mv --steps 20 --warmup 5 > $OUT/bench_train_mv.log 2>&1
rc=$?; tail -1 $OUT/bench_train_mv.log | cut -c1-400; exit $rc
