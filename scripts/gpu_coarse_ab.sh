#!/bin/bash
# Same-box A/B of rays_coarse_kernel / sample_coarse_kernel across library builds (LIBS: "name=path ...",
# "prod" = the in-tree library), kernel durations from rocprofv3 over scripts/rays_bench.py, ROUNDS times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-coarse_ab}; mkdir -p $OUT
for r in $(seq ${ROUNDS:-2}); do
  for spec in ${LIBS:-prod}; do
    name=${spec%%=*}; path=${spec#*=}
    if [ "$name" = prod ]; then unset AVR_LIB_PATH; else export AVR_LIB_PATH=$PWD/$path; fi
    d=$OUT/$name.$r
    RAYS_REPS=40 timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $d -o p -- python scripts/rays_bench.py > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
    f=$(find $d -name "*kernel_stats.csv" | head -1)
    python - "$f" $name <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "coarse" in r["Name"] or "fill" in r["Name"]:
        print(f"{sys.argv[2]:>6s} {r['Name'][:48]:48s} calls {r['Calls']:>4s} avg {float(r['AverageNs'])/1e3:7.2f} us min {float(r['MinNs'])/1e3:7.2f}")
PY
  done
done
