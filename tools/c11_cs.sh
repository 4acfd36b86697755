# round-3 call: LDS pixel stride / row padding table (dconv_cs) vs the CI + 4 rule
set -u
OUT=gpurun_out/c11; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -k "PWYX or pwyx or lstm or LSTM" > $OUT/tests.log 2>&1 || exit $?
for v in product oldcs; do
  L=$PWD/manette_amd/libmanette_hip_$v.so; [ $v = product ] && L=$PWD/manette_amd/libmanette_hip.so
  for c in breakout-pwyx-figar-rgb mspacman-lstm-figar; do
    MANETTE_HIP_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/sweep_${v}_$c -o run -- python3 tools/sweep_only.py --config $c --envs 32 --reps 20 > $OUT/sweep_${v}_$c.log 2>&1 || exit $?
    MANETTE_HIP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/bwd_${v}_$c -o run -- python3 tools/bwd_only.py --config $c --reps 10 > $OUT/bwd_${v}_$c.log 2>&1 || exit $?
  done
done
