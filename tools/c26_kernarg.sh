# round-3 call: device-memory kernel arguments (HIP_FORCE_DEV_KERNARG=1) vs the runtime default, A/B of the default bench
set -u
OUT=gpurun_out/c26; mkdir -p $OUT
export TMPDIR=/tmp
for k in 1 2; do
  timeout -k 10 400 python bench.py --no_cpu_baseline > $OUT/bench_def_$k.log 2>&1 || exit $?
  HIP_FORCE_DEV_KERNARG=1 timeout -k 10 400 python bench.py --no_cpu_baseline > $OUT/bench_devka_$k.log 2>&1 || exit $?
done
MANETTE_HIP_LIB=manette_amd/libmanette_hip_probe.so HIP_FORCE_DEV_KERNARG=1 timeout -k 10 200 python tools/probe.py > $OUT/probe_devka.txt 2>&1 || exit $?
