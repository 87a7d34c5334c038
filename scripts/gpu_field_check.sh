#!/bin/bash
# Field kernel change check: the field / training / scale parity tests, then a same-box A/B of the C3 fine
# pass against build/diag_base (the previous commit's library): VARIANTS as in gpu_field_ab.sh.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-fcheck}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_train.py tests/test_gpu_scale.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $OUT/pytest.log | head -20; exit $rc; }
VARIANTS="${VARIANTS:-base:adaptive-volume-rendering_amd/build/diag_base/libavr_hip.so:- tree:-:-}" ROUNDS=${ROUNDS:-3} bash scripts/gpu_field_ab.sh
