# round-3 call: direct forward for the NATURE strided VALID convs (MT_DCONV_STRIDED) vs the generic GEMM
set -u
OUT=gpurun_out/c14; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -k "NATURE or nature" > $OUT/tests.log 2>&1 || exit $?
for v in product nostr; do
  L=$PWD/manette_amd/libmanette_hip_$v.so; [ $v = product ] && L=$PWD/manette_amd/libmanette_hip.so
  for c in breakout-nature-figar seaquest-nature; do
    MANETTE_HIP_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/sweep_${v}_$c -o run -- python3 tools/sweep_only.py --config $c --envs 64 --reps 20 > $OUT/sweep_${v}_$c.log 2>&1 || exit $?
    MANETTE_HIP_LIB=$L timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no_cpu_baseline --trunk_sweep '' > $OUT/bench_${c}_$v.log 2>&1 || exit $?
  done
done
