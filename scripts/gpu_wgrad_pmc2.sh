#!/bin/bash
# weight-gradient kernels (AVR_WGRAD_WAVES in WAVES, AVR_WGRAD_PIPE in PIPES): SQ counters per dispatch of scripts/wgrad_bench.py
# (LDS waits / bank conflicts, MFMA busy, instruction mix), one rocprofv3 --pmc pass per group.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-wgpmc}; mkdir -p $OUT
for w0 in ${WAVES:-8 4}; do
for pp in ${PIPES:-0}; do
  export AVR_WGRAD_WAVES=$w0 AVR_WGRAD_PIPE=$pp
  w=$w0.p$pp
  i=0
  for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_WAVES" \
             "FETCH_SIZE"; do
    i=$((i+1))
    WG_REPS=1 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -f csv -d $OUT/w$w.p$i -o pmc -- python scripts/wgrad_bench.py > $OUT/w$w.p$i.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "pmc w$w pass $i rc=$rc"; tail -3 $OUT/w$w.p$i.log; exit $rc; }
  done
  python - $OUT $w <<'PY'
import csv, glob, sys, collections
vals = collections.defaultdict(list)
durs = []
for p in sorted(glob.glob(f"{sys.argv[1]}/w{sys.argv[2]}.p*/**/pmc_counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(p)):
        if "weight_grad" in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE" and "End_Timestamp" in r:
                durs.append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
m = {k: sum(v) / len(v) for k, v in vals.items()}
print(f"== AVR_WGRAD_WAVES / PIPE = {sys.argv[2]}")
for k, v in sorted(m.items()):
    print(f"  {k:26s} {v:.4g}")
if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
    print(f"  MFMA busy / (GUI_ACTIVE / 8 XCDs x 1024 SIMDs): {m['SQ_VALU_MFMA_BUSY_CYCLES'] / (m['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f}")
if durs:
    d = sum(durs) / len(durs)
    print(f"  dispatch {d / 1e6:.3f} ms; GRBM_GUI_ACTIVE / 8 XCDs / duration = {m['GRBM_GUI_ACTIVE'] / 8 / d:.3f} GHz")
PY
done
done
