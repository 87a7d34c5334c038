#!/bin/bash
# PMC passes over one command (CMD, default a 1-step bench line): each counter group of GROUPS (";"-separated) is
# its own `rocprofv3 --kernel-trace --pmc` pass (no sys / runtime trace domains; at most 8 SQ, 4 TCC, 2 GRBM
# counters per pass), then scripts/pmc_summary.py averages every counter per kernel and derives clock (GRBM_GUI_ACTIVE / 8 XCDs / dispatch time), MFMA busy and HBM bytes (2 x FETCH_SIZE, gfx950).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc}; mkdir -p $OUT
CMD=${CMD:-python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-legs --no-pmc}
GROUPS=${GROUPS:-"FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU;SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_LDS;SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"}
i=0
IFS=';' read -ra G <<< "$GROUPS"
for grp in "${G[@]}"; do
  i=$((i+1))
  timeout -s KILL ${LIMIT:-180} rocprofv3 --kernel-trace --pmc $grp -f csv -d $OUT/p$i -o pmc -- $CMD > $OUT/p$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "pass $i [$grp] rc=$rc"; tail -3 $OUT/p$i.log; exit $rc; }
done
python scripts/pmc_summary.py $OUT/summary.json $OUT/p* | tee $OUT/summary.txt
