# round-3 call: loss kernel critic-weight prefetch + single-chunk dense backward tiles (A/B by bench rows)
set -u
OUT=gpurun_out/c23; mkdir -p $OUT
export TMPDIR=/tmp
for L in manette_amd/libmanette_hip.so manette_amd/libmanette_hip_dbk.so; do
  MANETTE_HIP_LIB=$L timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_e2e_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/tests_$(basename $L .so).log 2>&1 || exit $?
done
for k in 1 2; do
  for v in base dbk; do
    MANETTE_HIP_LIB=manette_amd/libmanette_hip_$v.so timeout -k 10 400 python bench.py --no_cpu_baseline > $OUT/bench_${v}_$k.log 2>&1 || exit $?
  done
  timeout -k 10 400 python bench.py --no_cpu_baseline > $OUT/bench_prod_$k.log 2>&1 || exit $?
done
