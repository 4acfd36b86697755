# round-3 call: half-row NIPS conv blocks (MT_NIPS_HALF) — GPU suite, in-kernel probe, A/B bench
set -u
OUT=gpurun_out/c22; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread > $OUT/kern.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
echo "tests rc=$rc" > $OUT/suite.log
case $rc in 124|137|134|139) exit $rc;; esac
MANETTE_HIP_LIB=manette_amd/libmanette_hip_probe.so timeout -k 10 200 python tools/probe.py > $OUT/probe.txt 2>&1 || exit $?
MANETTE_HIP_LIB=manette_amd/libmanette_hip_probe.so timeout -k 10 200 python tools/probe.py --isolated > $OUT/probe_iso.txt 2>&1 || exit $?
for k in 1 2; do
  timeout -k 10 400 python bench.py --no_cpu_baseline > $OUT/bench_half_$k.log 2>&1 || exit $?
  MANETTE_HIP_LIB=manette_amd/libmanette_hip_nohalf.so timeout -k 10 400 python bench.py --no_cpu_baseline > $OUT/bench_nohalf_$k.log 2>&1 || exit $?
done
