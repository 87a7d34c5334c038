#!/bin/bash
# Board power and clocks sampled once a second while the C3 bench (or $CMD) runs: is the kernel power-capped?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/power; mkdir -p $OUT
# CMD: the workload to sample (default: the C3 bench)
timeout -k 10 300 ${CMD:-python bench.py --steps ${STEPS:-30} --warmup 2 --no-cpu-baseline} > $OUT/bench.log 2>&1 &
pid=$!
for i in $(seq 240); do
  echo "== t=$i" >> $OUT/smi.log
  timeout 10 amd-smi metric -g 0 -p -c -t >> $OUT/smi.log 2>&1 || timeout 10 rocm-smi --showpower --showclocks --showtemp >> $OUT/smi.log 2>&1
  kill -0 $pid 2>/dev/null || break
  sleep 1
done
wait $pid; rc=$?
tail -1 $OUT/bench.log
exit $rc
