#!/bin/bash
# sample_fine: the sampling parity tests, then the isolated timing (scripts/fine_bench.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-fine}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_philox.py tests/test_gpu_scale.py -k "fine or sample or merge or philox or c3 or Philox" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/pytest.log | head -20; exit $rc; }
for i in 1 2 3; do timeout -k 10 120 python scripts/fine_bench.py 2>&1 | tail -1; done
