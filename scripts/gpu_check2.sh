#!/bin/bash
# GPU suite (per-test timeout, verbose) then the default bench line (with the CPU baseline).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; grep -E "FAIL|ERROR|passed|failed" $OUT/pytest_gpu.log | tail -15; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1
rc=$?; tail -1 $OUT/bench.log; exit $rc
