#!/bin/bash
# A/B of the x3 field layouts (4 waves x 8 tiles vs 8 waves x 4 tiles): field
# parity tests under the 8-wave layout, then the bench in both.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
AVR_X3_WAVES=8 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread -k "field or render or smoke or march or adaptive" > $OUT/pytest_w8.log 2>&1
rc=$?; tail -5 $OUT/pytest_w8.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
for w in 4 8 4 8; do
  AVR_X3_WAVES=$w timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_w$w.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "bench w$w rc=$rc"; tail -20 $OUT/bench_w$w.log; exit $rc; }
  python -c "import json,sys; d=json.loads([l for l in open('$OUT/bench_w$w.log') if l.startswith('{')][-1]); print('waves $w', d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
done
