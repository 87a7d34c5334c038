#!/bin/bash
# Dev loop on the GPU box: selected GPU tests (PYTEST_K filter) then a short bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest_dev.log 2>&1
rc=$?; tail -15 $OUT/pytest_dev.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 2 ${BENCH_ARGS:-} > $OUT/bench_dev.log 2>&1
rc=$?; tail -1 $OUT/bench_dev.log; [ $rc -eq 0 ] || { echo "bench rc=$rc"; tail -20 $OUT/bench_dev.log; exit $rc; }
