#!/bin/bash
# weight_grad_kernel: isolated timing, kernel trace, and SQ / TCC counters.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/wgrad; mkdir -p $OUT
timeout -k 10 300 python scripts/wgrad_bench.py > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o wg -- python scripts/wgrad_bench.py > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
grep -h weight_grad $OUT/trace/*kernel_stats.csv | cut -c1-200
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  WG_REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -f csv -d $OUT/pmc$i -o pmc -- python scripts/wgrad_bench.py > $OUT/pmc$i.log 2>&1 || { echo "pmc $i failed"; tail -3 $OUT/pmc$i.log; continue; }
done
python - $OUT <<'PY'
import csv, glob, sys, collections
vals = collections.defaultdict(list)
for p in sorted(glob.glob(sys.argv[1] + "/pmc*/**/pmc_counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(p)):
        if "weight_grad" in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(vals.items()):
    print(f"{k:24s} mean over {len(v)} dispatches: {sum(v) / len(v):.4g}")
PY
