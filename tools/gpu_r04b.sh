set -u
OUT=gpurun_out/r04b; mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; echo "smoke rc=$?"
timeout -k 10 700 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_kernels_gpu.py tests/test_e2e_gpu.py tests/test_dp_gpu.py tests/test_probe_gpu.py > $OUT/t1.log 2>&1; rc=$?; echo "t1 rc=$rc"; tail -3 $OUT/t1.log
case $rc in 124|137|134|139) exit $rc;; esac
for c in breakout-nature-figar seaquest-nature pong-nips; do
  timeout -k 10 300 python bench.py --config $c --no_cpu_baseline --trunk_sweep= > $OUT/bench_$c.log 2>&1; rc=$?; echo "$c rc=$rc"
  case $rc in 124|137|134|139) exit $rc;; esac
done
