# round-3 call: direct weight gradient (DWgradJob) + conv2 direct dX: PWYX/LSTM tests, bwd traces, benches
set -u
OUT=gpurun_out/c6; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -k "PWYX or pwyx or lstm or LSTM" > $OUT/tests.log 2>&1 || exit $?
for v in product nodw; do
  L=$PWD/manette_amd/libmanette_hip_$v.so; [ $v = product ] && L=$PWD/manette_amd/libmanette_hip.so
  for c in breakout-pwyx-figar-rgb mspacman-lstm-figar; do
    MANETTE_HIP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/bwd_${v}_$c -o run -- python3 tools/bwd_only.py --config $c --reps 10 > $OUT/bwd_${v}_$c.log 2>&1 || exit $?
    MANETTE_HIP_LIB=$L timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 5 --no_cpu_baseline --trunk_sweep '' > $OUT/bench_${c}_$v.log 2>&1 || exit $?
  done
done
MANETTE_HIP_LIB=$PWD/manette_amd/libmanette_hip_probe.so timeout -k 10 200 python tools/probe.py > $OUT/probe_fwd.log 2>&1 || exit $?
MANETTE_HIP_LIB=$PWD/manette_amd/libmanette_hip_probe.so timeout -k 10 200 python tools/probe_bwd.py > $OUT/probe_bwd.log 2>&1 || exit $?
