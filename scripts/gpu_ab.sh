#!/bin/bash
# A/B the phase stamps of several stamps builds: STAMPS_LIBS="a.so b.so ..."
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for lib in $STAMPS_LIBS; do
  echo "=== $lib"
  STAMPS_LIB=$PWD/$lib timeout -k 10 300 python scripts/phase_stamps.py > gpurun_out/ab/$(basename $lib).txt 2>&1 || exit 1
  grep -E "${AB_GREP:-kernel|total}" gpurun_out/ab/$(basename $lib).txt
done
