#!/bin/bash
# Bench sweep over field-kernel variants: each entry of VARIANTS is "ENV=VAL ..." for one bench run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/sweep; mkdir -p $OUT
i=0
while IFS= read -r v; do
  [ -z "$v" ] && continue
  i=$((i+1))
  env $v timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline > $OUT/b$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "[$v] rc=$rc"; tail -5 $OUT/b$i.log; exit $rc; }
  python -c "import json; d=json.loads([l for l in open('$OUT/b$i.log') if l.startswith('{')][-1]); print('[$v]', d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
done <<< "$VARIANTS"
