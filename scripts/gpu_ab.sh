#!/bin/bash
# Same-box A/B (boxes differ by +-5 %, so kernel changes are decided on one box), alternated ROUNDS times, one
# process per measurement. Each entry of VARIANTS (space separated) is "tag:where:ENV=VAL,ENV=VAL", where is
#   -               the in-tree build,
#   path/to/lib.so  a library loaded through AVR_LIB_PATH (e.g. build/diag_x/libavr_hip.so from `make diag`),
#   DIR             another source tree (a directory: a git worktree built on the CPU side, sent with the snapshot).
# CMD is the measurement, run from the variant's tree (default: a short bench line, summarised):
#   CMD="python scripts/field_ab.py"  (field launch alone)   CMD="python scripts/wgrad_bench.py"
#   CMD="python scripts/fine_bench.py"  CMD="python scripts/rays_bench.py"  CMD="python scripts/train_fwd_ab.py train"
# PROF=1 runs CMD under rocprofv3 --kernel-trace --stats and keeps each kernel_stats.csv.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab}; mkdir -p $OUT
CMD=${CMD:-python bench.py --steps ${BSTEPS:-5} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-}}
for r in $(seq ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    IFS=: read -r tag where envs <<< "$v"
    dir=$ROOT
    unset AVR_LIB_PATH
    if [ "$where" = "-" ] || [ -z "$where" ]; then :
    elif [ -d "$ROOT/$where" ]; then dir=$ROOT/$where
    else export AVR_LIB_PATH=$ROOT/$where
    fi
    log=$OUT/r$r.$tag.log
    ( cd "$dir" && IFS=, && for e in $envs; do [ -n "$e" ] && export "$e"; done && IFS=' ' &&
      if [ "${PROF:-0}" = 1 ]; then
        timeout -k 10 ${LIMIT:-300} rocprofv3 --kernel-trace --stats -f csv -d $ROOT/$OUT/prof_r$r.$tag -o ab -- $CMD
      else
        TAG=$tag timeout -k 10 ${LIMIT:-300} $CMD
      fi ) > $log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "[$tag] rc=$rc"; tail -5 $log; exit $rc; }
    if grep -q '^{' $log; then
      python -c "import json; d=json.loads([l for l in open('$log') if l.startswith('{')][-1]); r=d.get('roofline',{}); print('[$tag]', d['value'], d.get('ms_per_step'), r.get('frac'), r.get('avg_launch_ms'))"
    else
      echo "[$tag] $(tail -1 $log)"
    fi
  done
done
exit 0
