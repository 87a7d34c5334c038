#!/bin/bash
# Same-box A/B of two source trees' bench lines: the current tree and $OLD (a git worktree built in place),
# alternated ROUNDS times. Diagnostics only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/abtrees; mkdir -p $OUT
for r in $(seq ${ROUNDS:-2}); do
  for t in . ${OLD:-abold}; do
    (cd $t && timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-}) > $OUT/r$r.$(basename $t).log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "[$t] rc=$rc"; tail -5 $OUT/r$r.$(basename $t).log; exit $rc; }
    python -c "import json; d=json.loads([l for l in open('$OUT/r$r.$(basename $t).log') if l.startswith('{')][-1]); print('[$t]', d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
  done
done
