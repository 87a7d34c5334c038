#!/bin/bash
# Clock and MFMA busy of the training kernels: one rocprofv3 --pmc pass (GRBM_GUI_ACTIVE, SQ_VALU_MFMA_BUSY_CYCLES)
# over bench.py --mode train (default_mv, HIP path), summarised per kernel and pass by scripts/train_clock.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-tclock}; mkdir -p $OUT
timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES -f csv -d $OUT/pmc -o pmc -- python bench.py --mode train --conf ${CONF:-default_mv} --train-modes hip --steps 3 --warmup 2 > $OUT/pmc.log 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "pmc rc=$rc"; tail -5 $OUT/pmc.log; exit $rc; }
f=$(find $OUT/pmc -name "*counter_collection.csv" | head -1)
python scripts/train_clock.py "$f"
