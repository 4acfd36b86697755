# round-3 call: LSTM window kernels with their operands requested up front (forward epilogue
# weights, BPTT gates / cell states / weights, dxg gather, zero-frame partials) — LSTM tests, e2e,
# A/B of the LSTM bench vs the previous commit
set -u
OUT=gpurun_out/c32; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_lstm_gpu.py tests/test_e2e_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || exit $?
for k in 1 2; do
  MANETTE_HIP_LIB=manette_amd/libmanette_hip_base.so timeout -k 10 400 python bench.py --config mspacman-lstm-figar --no_cpu_baseline > $OUT/bench_base_$k.log 2>&1 || exit $?
  timeout -k 10 400 python bench.py --config mspacman-lstm-figar --no_cpu_baseline > $OUT/bench_prod_$k.log 2>&1 || exit $?
done
