#!/bin/bash
# Round-3 GPU session: the named test files, then the default bench line.
# usage: scripts/gpu_r03.sh TAG [pytest files...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python -u bench.py > $OUT/bench.log 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 3000 $OUT/bench.log
exit $rc
