#!/bin/bash
# One GPU-box session: parity tests, smoke, a short bench and a rocprofv3
# kernel-trace summary. Each GPU step has its own time limit; the chain stops
# at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
echo "== host: $(nproc) cpus; $(python -c 'import torch;print(torch.__version__)')"
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -15 $OUT/pytest_gpu.log
# test failures (rc 1) still let smoke/bench run; a crash, abort or timeout stops here
[ $rc -le 1 ] || { echo "pytest gpu crashed rc=$rc"; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; cat $OUT/smoke.log | tail -3; [ $rc -eq 0 ] || { echo "smoke failed rc=$rc"; exit $rc; }
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > $OUT/bench.log 2>&1
rc=$?; tail -2 $OUT/bench.log; [ $rc -eq 0 ] || { echo "bench failed rc=$rc"; exit $rc; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o bench -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/prof.log 2>&1
rc=$?; tail -2 $OUT/prof.log; [ $rc -eq 0 ] || { echo "rocprof failed rc=$rc"; exit $rc; }
find $OUT/prof -name "*stats*" | head
