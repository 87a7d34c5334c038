#!/bin/bash
# Kernel-level A/B of the training kernels: scripts/train_fwd_ab.py under rocprofv3 --kernel-trace --stats for
# each library in LIBS ("-" = in-tree build, else build/diag_<name>/libavr_hip.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-tprof}; mkdir -p $OUT
for lib in ${LIBS:--}; do
  if [ "$lib" = "-" ]; then unset AVR_LIB_PATH; n=tree; else export AVR_LIB_PATH=$PWD/adaptive-volume-rendering_amd/build/diag_$lib/libavr_hip.so; n=$lib; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $OUT/$n -o p -- python scripts/train_fwd_ab.py > $OUT/$n.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -20 $OUT/$n.log; exit $rc; }
  echo "== $n"; grep "^\[" $OUT/$n.log
  f=$(find $OUT/$n -name "*kernel_stats.csv" | head -1)
  python - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "avr::" in n and float(r["TotalDurationNs"]) > 1e6:
        print(f"  {n[:46]:46s} calls {r['Calls']:>4s} avg {float(r['AverageNs'])/1e3:9.1f} us  min {float(r['MinNs'])/1e3:9.1f}")
PY
done
