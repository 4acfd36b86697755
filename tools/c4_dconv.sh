# round-3 call: direct-conv forward variants + direct dX in the backward
set -u
OUT=gpurun_out/c4; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -k "PWYX or pwyx or lstm or LSTM" > $OUT/tests.log 2>&1 || exit $?
for c in breakout-pwyx-figar-rgb mspacman-lstm-figar; do
  for v in product nobwd w4 t14; do
    L=$PWD/manette_amd/libmanette_hip_$v.so; [ $v = product ] && L=$PWD/manette_amd/libmanette_hip.so
    MANETTE_HIP_LIB=$L timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 5 --no_cpu_baseline --trunk_sweep '' > $OUT/bench_${c}_$v.log 2>&1 || exit $?
  done
done
for v in product w4 t14; do
  L=$PWD/manette_amd/libmanette_hip_$v.so; [ $v = product ] && L=$PWD/manette_amd/libmanette_hip.so
  MANETTE_HIP_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/sweep_$v -o run -- python3 tools/sweep_only.py --config breakout-pwyx-figar-rgb --envs 32 --reps 20 > $OUT/sweep_$v.log 2>&1 || exit $?
done
for v in product nobwd; do
  L=$PWD/manette_amd/libmanette_hip_$v.so; [ $v = product ] && L=$PWD/manette_amd/libmanette_hip.so
  for c in breakout-pwyx-figar-rgb mspacman-lstm-figar; do
    MANETTE_HIP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/bwd_${v}_$c -o run -- python3 tools/bwd_only.py --config $c --reps 10 > $OUT/bwd_${v}_$c.log 2>&1 || exit $?
  done
done
