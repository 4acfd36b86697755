# round-3 call: conv2 8-wave forward adopted (tests + benches); conv1 8-wave variant A/B
set -u
OUT=gpurun_out/c13; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -k "PWYX or pwyx or lstm or LSTM" > $OUT/tests.log 2>&1 || exit $?
MANETTE_HIP_LIB=$PWD/manette_amd/libmanette_hip_c1w8.so timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -k "test_forward_parity and PWYX" > $OUT/tests_c1w8.log 2>&1 || exit $?
for v in product c1w8; do
  L=$PWD/manette_amd/libmanette_hip_$v.so; [ $v = product ] && L=$PWD/manette_amd/libmanette_hip.so
  for c in breakout-pwyx-figar-rgb mspacman-lstm-figar; do
    MANETTE_HIP_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/sweep_${v}_$c -o run -- python3 tools/sweep_only.py --config $c --envs 32 --reps 20 > $OUT/sweep_${v}_$c.log 2>&1 || exit $?
  done
done
for c in breakout-pwyx-figar-rgb mspacman-lstm-figar; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no_cpu_baseline > $OUT/bench_$c.log 2>&1 || exit $?
done
