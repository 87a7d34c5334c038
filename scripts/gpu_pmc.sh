#!/bin/bash
# PMC passes over a short bench (1 timed step): L2 hit/miss, HBM bytes, MFMA
# and wait counters. Each counter group is its own rocprofv3 pass
# (--kernel-trace + --pmc only, no sys/runtime trace domains).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc; mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
grep -oE "(TCC|SQ|TCP|GRBM)_[A-Z0-9_]+(\[[0-9]+\])?" $OUT/avail.txt | sort -u > $OUT/counters.txt || true
wc -l $OUT/counters.txt
CMD="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --precision ${PREC:-x3}"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" "SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "SQ_INST_CYCLES_VMEM SQ_VALU_MFMA_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -f csv -d $OUT/p$i -o pmc -- $CMD > $OUT/p$i.log 2>&1
  echo "pass $i [$grp] rc=$?"
done
ls $OUT/p*/ | head
