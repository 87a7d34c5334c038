set -u
export TMPDIR=/tmp
OUT=gpurun_out/r04e; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/tprof -o train -- python bench.py --mode train --conf default_mv --bn --train-modes hip --steps 10 --warmup 3 > $OUT/tprof.log 2>&1 || exit $?
cp "$(find $OUT/tprof -name '*kernel_stats.csv' | head -1)" $OUT/train_bn_kernel_stats.csv
head -25 $OUT/train_bn_kernel_stats.csv | cut -c1-200
BN=1 CONF=default_mv timeout -k 10 300 python -u scripts/train_profile.py > $OUT/train_profile_bn.log 2>&1 || exit $?
head -60 $OUT/train_profile_bn.log | cut -c1-250
