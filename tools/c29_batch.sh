# round-3 call: batched loads in the RMSProp norm reduction (8 partials per lane) and the head
# weight gradient (16 rows per trip) — kernel tests, e2e, A/B bench vs the previous commit
set -u
OUT=gpurun_out/c29; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_e2e_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || exit $?
for k in 1 2 3; do
  MANETTE_HIP_LIB=manette_amd/libmanette_hip_base.so timeout -k 10 400 python bench.py --no_cpu_baseline > $OUT/bench_base_$k.log 2>&1 || exit $?
  timeout -k 10 400 python bench.py --no_cpu_baseline > $OUT/bench_prod_$k.log 2>&1 || exit $?
done
