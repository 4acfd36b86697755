# round-3 call: every pooled-input layer's dX as its own direct launch (MT_DCONV_BWD=2) vs the product
set -u
OUT=gpurun_out/c10; mkdir -p $OUT
export TMPDIR=/tmp
MANETTE_HIP_LIB=$PWD/manette_amd/libmanette_hip_bwd2.so timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -k "test_loss_backward_parity and PWYX or test_lstm_loss_backward_parity" > $OUT/tests_bwd2.log 2>&1 || exit $?
for v in bwd2 product; do
  L=$PWD/manette_amd/libmanette_hip_$v.so; [ $v = product ] && L=$PWD/manette_amd/libmanette_hip.so
  for c in breakout-pwyx-figar-rgb mspacman-lstm-figar; do
    MANETTE_HIP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/bwd_${v}_$c -o run -- python3 tools/bwd_only.py --config $c --reps 10 > $OUT/bwd_${v}_$c.log 2>&1 || exit $?
  done
done
timeout -k 10 300 python bench.py --config breakout-pwyx-figar-rgb --steps 20 --warmup 5 --no_cpu_baseline --trunk_sweep '' > $OUT/bench_pwyx.log 2>&1 || exit $?
