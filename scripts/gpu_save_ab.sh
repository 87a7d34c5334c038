#!/bin/bash
# Training forward (SAVE) cost split: scripts/train_fwd_ab.py "train" (and "infer8") for the in-tree build and
# each diag library in LIBS (build/diag_<name>/libavr_hip.so), ROUNDS rounds, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for r in $(seq ${ROUNDS:-2}); do
for lib in - ${LIBS:-}; do
  if [ "$lib" = "-" ]; then unset AVR_LIB_PATH; n=tree; else export AVR_LIB_PATH=$PWD/adaptive-volume-rendering_amd/build/diag_$lib/libavr_hip.so; n=$lib; fi
  CONF=${CONF:-default_mv} VARIANTS=${VARIANTS:-infer8,train} timeout -k 10 120 python -u scripts/train_fwd_ab.py 2>&1 | grep "^\[" | sed "s/^/$n r$r /" || exit 1
done
done
