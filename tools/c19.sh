# round-3 call: the whole GPU suite at HEAD (loss kernel's bootstrap slabs ahead of the PCIe loads,
# gray conv1 dW on 4 M-tiles per wave), LSTM / Pong benches + traces, and the strided dW split experiment
set -u
OUT=gpurun_out/c19; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
echo "tests rc=$rc" > $OUT/suite.log
case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no_cpu_baseline --trunk_sweep '' > $OUT/bench_pong.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config mspacman-lstm-figar --steps 20 --warmup 5 --no_cpu_baseline > $OUT/bench_lstm.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/bwd_lstm -o run -- python3 tools/bwd_only.py --config mspacman-lstm-figar --reps 10 > $OUT/bwd_lstm.log 2>&1 || exit $?
MANETTE_HIP_LIB=$PWD/manette_amd/libmanette_hip_wsplit.so timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -k "NATURE or nature" > $OUT/tests_wsplit.log 2>&1 || exit $?
for v in wsplit product; do
  L=$PWD/manette_amd/libmanette_hip_$v.so; [ $v = product ] && L=$PWD/manette_amd/libmanette_hip.so
  MANETTE_HIP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/bwd_${v}_nature -o run -- python3 tools/bwd_only.py --config breakout-nature-figar --reps 10 > $OUT/bwd_${v}_nature.log 2>&1 || exit $?
done
