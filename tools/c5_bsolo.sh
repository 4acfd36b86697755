# round-3 call: direct dX as its own launch ahead of the weight-gradient group (MT_DCONV_BWD=2)
set -u
OUT=gpurun_out/c5; mkdir -p $OUT
export TMPDIR=/tmp
MANETTE_HIP_LIB=$PWD/manette_amd/libmanette_hip_bsolo.so timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -k "test_loss_backward_parity and PWYX or test_lstm_loss_backward_parity" > $OUT/tests_bsolo.log 2>&1 || exit $?
for v in bsolo product; do
  L=$PWD/manette_amd/libmanette_hip_$v.so; [ $v = product ] && L=$PWD/manette_amd/libmanette_hip.so
  for c in breakout-pwyx-figar-rgb mspacman-lstm-figar; do
    MANETTE_HIP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/bwd_${v}_$c -o run -- python3 tools/bwd_only.py --config $c --reps 10 > $OUT/bwd_${v}_$c.log 2>&1 || exit $?
  done
done
