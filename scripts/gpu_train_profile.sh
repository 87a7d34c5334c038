#!/bin/bash
# Kernel-time breakdown of the training step (bench.py --mode train, HIP path only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/train; mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o train -- python bench.py --mode train --steps 5 --warmup 2 --train-modes hip > $OUT/prof.log 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/prof.log; exit $rc; }
tail -1 $OUT/prof.log
python - $OUT/prof/train_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel ms {tot / 1e6:.2f} over 7 steps")
for r in rows[:22]:
    print(f'{float(r["TotalDurationNs"]) / 1e6:9.2f} ms {int(r["Calls"]):5d} {float(r["Percentage"]):6.2f}%  {r["Name"][:100]}')
PY
