#!/bin/bash
# Same-box A/B of field kernel variants: each VARIANT is "tag:libpath:debugflags" (libpath "-" = default build),
# alternated ROUNDS times, one process per measurement (scripts/field_ab.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/fieldab; mkdir -p $OUT
for r in $(seq ${ROUNDS:-3}); do
  for v in $VARIANTS; do
    IFS=: read tag lib dbg <<< "$v"
    if [ "$lib" = "-" ]; then unset AVR_LIB_PATH; else export AVR_LIB_PATH=$PWD/$lib; fi
    if [ "$dbg" = "-" ]; then unset AVR_DEBUG; else export AVR_DEBUG=$dbg; fi
    TAG=$tag timeout -k 10 120 python scripts/field_ab.py >> $OUT/ab.log 2>> $OUT/ab.err
    rc=$?; [ $rc -eq 0 ] || { echo "[$tag] rc=$rc"; tail -5 $OUT/ab.err; exit $rc; }
    tail -1 $OUT/ab.log
  done
done
