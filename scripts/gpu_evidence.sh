#!/bin/bash
# Evidence at HEAD on the GPU box (profiles/<TAG>_*): the steps named in STEPS, in this order, each under its own
# time limit; the first failure ends the script.
#   tests  the whole -m gpu suite in one process (per-test timeout)       -> $OUT/pytest_gpu.log
#   smoke  __graft_entry__.smoke()                                        -> $OUT/smoke.log
#   bench  the default bench line (legs, PMC traffic, CPU baseline)        -> $OUT/bench.log
#   prof   rocprofv3 --kernel-trace --stats of a short bench command        -> $OUT/bench_kernel_stats.csv
#   train  bench.py --mode train for each conf in CONFS (+ TRAIN_ARGS)      -> $OUT/bench_train_<conf>.log
#   tprof  rocprofv3 kernel stats of the HIP train step (CONFS' last conf)  -> $OUT/train_kernel_stats.csv
#   trainx the --bn, AdaptiveVolumeRenderer, NS 2 and spade + NS 2 train steps (default_mv)
#          -> $OUT/bench_train_{bn,adaptive,views2,spade_views2}_mv.log
#   bprof  rocprofv3 kernel stats of the --bn HIP train step (default_mv)   -> $OUT/train_bn_kernel_stats.csv
# env: TAG (default r04), STEPS (default all), PYTEST_ARGS (extra pytest args, e.g. "-k philox"), CONFS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r04}
OUT=gpurun_out/$TAG; mkdir -p $OUT
STEPS=${STEPS:-tests smoke bench prof train tprof trainx bprof}
CONFS=${CONFS:-default default_mv}
export AVR_TEST_REPORT=$OUT/philox_c3_flip_rates.jsonl
has() { [[ " $STEPS " == *" $1 "* ]]; }
if has tests; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "FAILED|Error" $OUT/pytest_gpu.log | head; exit $rc; }
fi
if has smoke; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
  rc=$?; tail -1 $OUT/smoke.log; [ $rc -eq 0 ] || { echo "smoke rc=$rc"; exit $rc; }
fi
if has bench; then
  timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2> $OUT/bench.err
  rc=$?; tail -c 600 $OUT/bench.log; echo; [ $rc -eq 0 ] || { echo "bench rc=$rc"; tail -5 $OUT/bench.err; exit $rc; }
fi
if has prof; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o bench -- python bench.py --steps 3 --warmup 1 \
    --no-cpu-baseline --no-legs --no-pmc > $OUT/prof.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "rocprof rc=$rc"; tail -5 $OUT/prof.log; exit $rc; }
  cp "$(find $OUT/prof -name '*kernel_stats.csv' | head -1)" $OUT/bench_kernel_stats.csv
  head -4 $OUT/bench_kernel_stats.csv | cut -c1-160
fi
if has train; then
  for c in $CONFS; do
    timeout -k 10 300 python -u bench.py --mode train --conf $c --steps 20 --warmup 5 ${TRAIN_ARGS:-} > $OUT/bench_train_$c.log 2>&1
    rc=$?; tail -1 $OUT/bench_train_$c.log | cut -c1-300; echo; [ $rc -eq 0 ] || { echo "train $c rc=$rc"; exit $rc; }
  done
fi
if has tprof; then
  c=${CONFS##* }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/tprof -o train -- python bench.py --mode train \
    --conf $c --train-modes hip --steps 10 --warmup 3 ${TRAIN_ARGS:-} > $OUT/tprof.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "train rocprof rc=$rc"; tail -5 $OUT/tprof.log; exit $rc; }
  cp "$(find $OUT/tprof -name '*kernel_stats.csv' | head -1)" $OUT/train_kernel_stats.csv
  head -6 $OUT/train_kernel_stats.csv | cut -c1-160
fi
if has trainx; then
  for x in "bn:--bn" "adaptive:--renderer adaptive --train-modes hip,hip_graph,torch" "views2:--views 2" "spade_views2:--spade --views 2"; do
    timeout -k 10 300 python -u bench.py --mode train --conf default_mv ${x#*:} --steps 20 --warmup 5 > $OUT/bench_train_${x%%:*}_mv.log 2>&1
    rc=$?; tail -1 $OUT/bench_train_${x%%:*}_mv.log | cut -c1-300; echo; [ $rc -eq 0 ] || { echo "train ${x%%:*} rc=$rc"; exit $rc; }
  done
fi
if has bprof; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/bprof -o train -- python bench.py --mode train \
    --conf default_mv --bn --train-modes hip --steps 10 --warmup 3 > $OUT/bprof.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "bn train rocprof rc=$rc"; tail -5 $OUT/bprof.log; exit $rc; }
  cp "$(find $OUT/bprof -name '*kernel_stats.csv' | head -1)" $OUT/train_bn_kernel_stats.csv
  head -4 $OUT/train_bn_kernel_stats.csv | cut -c1-160
fi
# the traces stay on the box (gpurun copies back at most 64 MiB)
find $OUT -name '*kernel_trace.csv' -delete; find $OUT -name '*_results.db' -delete
exit 0
