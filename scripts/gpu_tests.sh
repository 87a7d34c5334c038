#!/bin/bash
# The whole -m gpu suite in one process (per-test timeout), log under gpurun_out/$TAG.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-tests}; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/ ${EXTRA:-} > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest_gpu.log; exit $rc
