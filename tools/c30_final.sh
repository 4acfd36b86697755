# round-3 closing call (after the half-row / loss / batched-load experiments): smoke, the whole GPU suite, the default bench three times back to back
# (run-to-run spread on one box), rocprof of bench.py --gpus 1 --steps 20 --warmup 5
set -u
OUT=gpurun_out/c30; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
echo "tests rc=$rc" > $OUT/suite.log
case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 400 python bench.py > $OUT/bench_1.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --no_cpu_baseline > $OUT/bench_2.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --no_cpu_baseline > $OUT/bench_3.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/prof.log 2>&1 || exit $?
