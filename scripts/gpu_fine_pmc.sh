#!/bin/bash
# sample_fine_kernel: isolated timing and SQ counters (dynamic instruction mix, waits).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/fine; mkdir -p $OUT
timeout -k 10 120 python scripts/fine_bench.py > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
[ "${PMC:-1}" = 1 ] || exit 0
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  FINE_REPS=2 timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp -f csv -d $OUT/pmc$i -o pmc -- python scripts/fine_bench.py > $OUT/pmc$i.log 2>&1 || { echo "pmc $i failed"; tail -3 $OUT/pmc$i.log; exit 1; }
done
python - $OUT <<'PY'
import csv, glob, sys, collections
vals = collections.defaultdict(list)
for p in sorted(glob.glob(sys.argv[1] + "/pmc*/**/pmc_counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(p)):
        if "sample_fine" in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in vals.items()}
for k, v in sorted(m.items()):
    print(f"{k:24s} {v:.4g}" + (f"   per wave {v / m['SQ_WAVES']:.1f}" if "SQ_WAVES" in m and k != "SQ_WAVES" else ""))
PY
