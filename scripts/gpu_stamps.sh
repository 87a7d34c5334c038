#!/bin/bash
# Phase stamps of the x3 field kernel, then one PMC pass (instruction cache) over the same script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/stamps; mkdir -p $OUT
timeout -k 10 300 python scripts/phase_stamps.py | tee $OUT/stamps.txt || exit 1
if [ -n "${PMC:-}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $PMC -f csv -d $OUT/pmc -o pmc -- python scripts/phase_stamps.py > $OUT/pmc.log 2>&1 || exit 1
  python - <<'PY'
import csv, glob, collections
rows = list(csv.DictReader(open(glob.glob("gpurun_out/stamps/pmc/**/pmc_counter_collection.csv", recursive=True)[0])))
agg = collections.defaultdict(float)
for r in rows:
    if "field_x3" in r["Kernel_Name"]:
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(agg.items()):
    print(f"{k:32s} {v:.4g}")
PY
fi
