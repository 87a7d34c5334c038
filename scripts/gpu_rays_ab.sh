#!/bin/bash
# rays_coarse_kernel: rays per workgroup sweep (AVR_RPB), kernel durations from rocprofv3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-rays}; mkdir -p $OUT
for rpb in ${RPBS:-64 32 16 8}; do
  AVR_RPB=$rpb RAYS_REPS=20 timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $OUT/r$rpb -o p -- python scripts/rays_bench.py > $OUT/r$rpb.log 2>&1 || { tail -5 $OUT/r$rpb.log; exit 1; }
  f=$(find $OUT/r$rpb -name "*kernel_stats.csv" | head -1)
  python - "$f" $rpb <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "coarse" in r["Name"]:
        print(f"rpb {sys.argv[2]:>3s} {r['Name'][:60]:60s} calls {r['Calls']:>4s} avg {float(r['AverageNs'])/1e3:7.2f} us min {float(r['MinNs'])/1e3:7.2f}")
PY
done
