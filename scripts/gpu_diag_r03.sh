#!/bin/bash
# Round-3 diagnostics: training forward vs inference forward under diagnostic builds (LIBS).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/diag; mkdir -p $OUT
for lib in ${LIBS:--}; do
  if [ "$lib" = "-" ]; then unset AVR_LIB_PATH; else export AVR_LIB_PATH=$PWD/adaptive-volume-rendering_amd/build/diag_$lib/libavr_hip.so; fi
  echo "lib $lib" >> $OUT/train_fwd.log
  timeout -k 10 180 python -u scripts/train_fwd_ab.py >> $OUT/train_fwd.log 2>&1 || { tail -20 $OUT/train_fwd.log; exit 1; }
done
grep "^\[\|^lib" $OUT/train_fwd.log
