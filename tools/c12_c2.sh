# round-3 call: conv2 forward tilings (8 waves / 5-tap weight chunks) vs the product
set -u
OUT=gpurun_out/c12; mkdir -p $OUT
export TMPDIR=/tmp
MANETTE_HIP_LIB=$PWD/manette_amd/libmanette_hip_c2w8.so timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -k "test_forward_parity and PWYX" > $OUT/tests_c2w8.log 2>&1 || exit $?
MANETTE_HIP_LIB=$PWD/manette_amd/libmanette_hip_c2w8k.so timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -k "test_forward_parity and PWYX" > $OUT/tests_c2w8k.log 2>&1 || exit $?
for v in product c2w8 c2w8k c2k; do
  L=$PWD/manette_amd/libmanette_hip_$v.so; [ $v = product ] && L=$PWD/manette_amd/libmanette_hip.so
  for c in breakout-pwyx-figar-rgb mspacman-lstm-figar; do
    MANETTE_HIP_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/sweep_${v}_$c -o run -- python3 tools/sweep_only.py --config $c --envs 32 --reps 20 > $OUT/sweep_${v}_$c.log 2>&1 || exit $?
  done
done
