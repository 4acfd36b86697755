# full checkpoint call: smoke, the whole GPU suite, bench of every config, rocprof of the default bench (OUT=gpurun_out/<tag>)
set -u
OUT=${OUT:-gpurun_out/c16}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
echo "tests rc=$rc" > $OUT/suite.log
case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || exit $?
for c in breakout-nature-figar seaquest-nature breakout-pwyx-figar-rgb mspacman-lstm-figar; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no_cpu_baseline > $OUT/bench_$c.log 2>&1 || exit $?
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/prof.log 2>&1 || exit $?
