# round-3 call: direct weight gradient of the strided VALID layers (NATURE, NIPS RGB conv2) vs generic
set -u
OUT=gpurun_out/c15; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -k "NATURE or nature or NIPS or nips or pong" > $OUT/tests.log 2>&1 || exit $?
for v in product nowgs; do
  L=$PWD/manette_amd/libmanette_hip_$v.so; [ $v = product ] && L=$PWD/manette_amd/libmanette_hip.so
  for c in breakout-nature-figar seaquest-nature; do
    MANETTE_HIP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/bwd_${v}_$c -o run -- python3 tools/bwd_only.py --config $c --reps 10 > $OUT/bwd_${v}_$c.log 2>&1 || exit $?
  done
done
