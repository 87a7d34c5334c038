#!/bin/bash
# Round-end evidence for profiles/: full GPU test suite, the default bench line
# (with cpu_baseline), rocprofv3 kernel stats of the same bench command, and
# separate PMC passes (FETCH_SIZE / WRITE_SIZE / L2 hit) for the field kernel's
# HBM traffic per launch (gfx950: FETCH_SIZE x 2, MI355X_MICROARCH.md HBM section).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r02}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
rc=$?; tail -1 $OUT/smoke.log; [ $rc -eq 0 ] || { echo "smoke rc=$rc"; exit $rc; }
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1
rc=$?; tail -1 $OUT/bench.log; [ $rc -eq 0 ] || { echo "bench rc=$rc"; exit $rc; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o bench -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/prof.log 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "rocprof rc=$rc"; tail -5 $OUT/prof.log; exit $rc; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -f csv -d $OUT/pmc$i -o pmc -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/pmc$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "pmc pass $i rc=$rc"; tail -5 $OUT/pmc$i.log; exit $rc; }
done
python - "$OUT" <<'PY'
import csv, glob, json, sys, collections
out = sys.argv[1]
vals = collections.defaultdict(list)
for path in sorted(glob.glob(f"{out}/pmc*/**/pmc_counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(path)):
        if "field_x3_kernel" in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {k: sum(v) / len(v) for k, v in vals.items()}
fetch = res.get("FETCH_SIZE")   # KB per dispatch
write = res.get("WRITE_SIZE")
hit, miss = res.get("TCC_HIT_sum"), res.get("TCC_MISS_sum")
j = {"kernel": "field_x3_kernel<4,8> (8 waves)", "source": f"rocprofv3 --pmc over bench.py --steps 1 --warmup 1 ({out})",
     "dispatches_averaged": len(vals.get("FETCH_SIZE", [])),
     "fetch_size_kb_per_launch_raw": fetch, "write_size_kb_per_launch": write,
     "hbm_bytes_per_launch": None if fetch is None else int(2 * fetch * 1024 + (write or 0) * 1024),
     "note": "FETCH_SIZE doubled (gfx950 reports half of 16-B-per-lane reads); includes Infinity-Cache hits",
     "l2_hit_rate": None if not hit else hit / (hit + miss)}
json.dump(j, open(f"{out}/field_pmc.json", "w"), indent=1)
print(json.dumps(j))
PY
# per-kernel summary of every pass: HBM GB/s from FETCH/WRITE, MFMA busy, L2 hit rate
python scripts/pmc_summary.py $OUT/pmc_kernels.json $OUT/pmc1 $OUT/pmc2 $OUT/pmc3 $OUT/pmc4
