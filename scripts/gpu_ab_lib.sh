#!/bin/bash
# Same-box A/B of the default build and an alternative library ($ALT, via AVR_LIB_PATH), alternated ROUNDS times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/ablib; mkdir -p $OUT
for r in $(seq ${ROUNDS:-2}); do
  for v in base alt; do
    if [ $v = alt ]; then export AVR_LIB_PATH=$PWD/$ALT; else unset AVR_LIB_PATH; fi
    timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/r$r.$v.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "[$v] rc=$rc"; tail -5 $OUT/r$r.$v.log; exit $rc; }
    python -c "import json; d=json.loads([l for l in open('$OUT/r$r.$v.log') if l.startswith('{')][-1]); print('[$v]', d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
  done
done
