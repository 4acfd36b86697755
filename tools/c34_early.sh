# round-3 call: NIPS conv kernel with its input rows, W1 staging and tag base requested together at
# block start (tools/patches/nips_conv_early_loads.patch, built as libmanette_hip_early.so) — kernel
# tests, e2e, learner tests on that library, A/B of the default bench vs the product library
set -u
OUT=gpurun_out/c34; mkdir -p $OUT
export TMPDIR=/tmp
MANETTE_HIP_LIB=manette_amd/libmanette_hip_early.so timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_e2e_gpu.py tests/test_learner_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || exit $?
for k in 1 2; do
  timeout -k 10 400 python bench.py --no_cpu_baseline > $OUT/bench_base_$k.log 2>&1 || exit $?
  MANETTE_HIP_LIB=manette_amd/libmanette_hip_early.so timeout -k 10 400 python bench.py --no_cpu_baseline > $OUT/bench_early_$k.log 2>&1 || exit $?
done
