#!/bin/bash
# weight_grad_kernel A/B: scripts/wgrad_bench.py for the in-tree build and each diag library in LIBS
# (build/diag_<name>/libavr_hip.so), each AVR_WGRAD_WAVES value in WAVES (8 or 4) and each AVR_WGRAD_PIPE
# value in PIPES (0 or 1),
# kernel durations from rocprofv3 --stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-wg}; mkdir -p $OUT
for r in $(seq ${ROUNDS:-1}); do
for lib in ${LIBS:--}; do
for w in ${WAVES:-8}; do
for pp in ${PIPES:-0}; do
  export AVR_WGRAD_WAVES=$w AVR_WGRAD_PIPE=$pp
  if [ "$lib" = "-" ]; then unset AVR_LIB_PATH; n=tree$w.p$pp; else export AVR_LIB_PATH=$PWD/adaptive-volume-rendering_amd/build/diag_$lib/libavr_hip.so; n=$lib$w.p$pp; fi
  WG_REPS=${WG_REPS:-5} timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $OUT/$n.$r -o p -- python scripts/wgrad_bench.py > $OUT/$n.$r.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -20 $OUT/$n.$r.log; exit $rc; }
  f=$(find $OUT/$n.$r -name "*kernel_stats.csv" | head -1)
  python - "$f" $n <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "weight_grad" in r["Name"]:
        print(f"{sys.argv[2]:>8s} {r['Name'][:40]:40s} calls {r['Calls']:>3s} avg {float(r['AverageNs'])/1e6:7.3f} ms min {float(r['MinNs'])/1e6:7.3f}")
PY
done
done
done
done
