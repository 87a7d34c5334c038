#!/bin/bash
# Dev loop on the GPU box: the GPU tests named in TESTS (files or node ids, default all) with a per-test timeout,
# then the commands of CMDS (";"-separated, each under its own time limit); the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-dev}; mkdir -p $OUT
export AVR_TEST_REPORT=$OUT/philox_c3_flip_rates.jsonl
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TLIMIT:-600} python -u -m pytest $TESTS -m gpu -x -v -s --timeout 240 --timeout-method thread \
    -p no:cacheprovider ${PYTEST_ARGS:-} > $OUT/pytest.log 2>&1
  rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "Error|assert|FAILED" $OUT/pytest.log | head -20; exit $rc; }
fi
i=0
IFS=';' read -ra C <<< "${CMDS:-}"
for c in "${C[@]}"; do
  [ -z "${c// }" ] && continue
  i=$((i+1))
  timeout -k 10 ${CLIMIT:-300} bash -c "$c" > $OUT/cmd$i.log 2>&1
  rc=$?; tail -c 1200 $OUT/cmd$i.log; echo; [ $rc -eq 0 ] || { echo "cmd $i rc=$rc: $c"; exit $rc; }
done
exit 0
