#!/bin/bash
# Selected GPU tests: TESTS="tests/x.py tests/y.py" K="expr" bash scripts/gpu_tests.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu ${K:+-k "$K"} -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_sel.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed|max rel" $OUT/pytest_sel.log | tail -40; exit $rc
