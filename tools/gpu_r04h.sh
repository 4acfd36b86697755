set -u
OUT=gpurun_out/r04h; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py::test_stacking_trunk_in_kernel_pull "tests/test_e2e_gpu.py" > $OUT/t1.log 2>&1; rc=$?; echo "t1 rc=$rc"; tail -2 $OUT/t1.log
case $rc in 124|137|134|139) exit $rc;; esac
for c in breakout-nature-figar seaquest-nature; do
  MT_ROLLOUT_AHEAD=1 MANETTE_HIP_LIB=$PWD/manette_amd/libmanette_hip_probe.so timeout -k 10 200 python tools/probe.py --config $c --updates 10 > $OUT/probe_$c.txt 2>&1; rc=$?; echo "probe $c rc=$rc"
  case $rc in 124|137|134|139) exit $rc;; esac
  timeout -k 10 300 python bench.py --config $c --no_cpu_baseline --trunk_sweep= > $OUT/bench_$c.log 2>&1; rc=$?; echo "bench $c rc=$rc"
  case $rc in 124|137|134|139) exit $rc;; esac
done
