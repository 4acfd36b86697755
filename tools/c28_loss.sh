# round-3 call: loss kernel A/B — base (HEAD~) vs product (critic weights early, V[b] reused) vs
# rewards as agent-scope relaxed atomics (MT_LOSS_RM_EARLY)
set -u
OUT=gpurun_out/c28; mkdir -p $OUT
export TMPDIR=/tmp
for L in hip hip_rmearly; do
  MANETTE_HIP_LIB=manette_amd/libmanette_$L.so timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_e2e_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/tests_$L.log 2>&1 || exit $?
done
for k in 1 2; do
  for L in hip_base hip hip_rmearly; do
    MANETTE_HIP_LIB=manette_amd/libmanette_$L.so timeout -k 10 400 python bench.py --no_cpu_baseline > $OUT/bench_${L}_$k.log 2>&1 || exit $?
  done
done
