set -u
export TMPDIR=/tmp
TAG=r04f TESTS="tests/test_gpu_train_bn.py" CMDS="python -u bench.py --mode train --conf default_mv --bn --steps 10 --warmup 3" bash scripts/gpu_dev.sh || exit $?
OUT=gpurun_out/r04f
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/tprof -o train -- python bench.py --mode train --conf default_mv --bn --train-modes hip --steps 10 --warmup 3 > $OUT/tprof.log 2>&1 || exit $?
cp "$(find $OUT/tprof -name '*kernel_stats.csv' | head -1)" $OUT/train_bn_kernel_stats.csv
head -14 $OUT/train_bn_kernel_stats.csv | cut -c1-180
