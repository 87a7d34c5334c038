#!/bin/bash
# Quick GPU iteration: field + renderer parity tests, then the x3 bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -15 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --precision ${PREC:-x3} --no-cpu-baseline > $OUT/bench.log 2>&1
rc=$?; tail -1 $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('VALUE', d['value'], 'ms/step', d['ms_per_step'], 'field TF', d['roofline']['achieved'], 'frac', d['roofline']['frac'], 'launch ms', d['roofline']['avg_launch_ms'])"
exit $rc
