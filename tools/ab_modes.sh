# GPU-box A/B of env-var modes (tools only): optional GPU tests first (TESTS=1), then bench runs
# alternating the modes. MODES="name:VAR=v,VAR2=w name2:..." ; REPS="1 2"; BENCH_ARGS passed on.
set -o pipefail
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1; rc=$?
  echo "tests rc=$rc"; tail -1 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || exit 1
fi
for rep in ${REPS:-1 2}; do for m in ${MODES:-default:}; do name=${m%%:*}; envs=${m#*:}
  ( [ -n "$envs" ] && export ${envs//,/ }; timeout -k 10 150 python bench.py --no_cpu_baseline ${BENCH_ARGS:-} > gpurun_out/ab_$name.log 2>&1 ) || { echo "bench $name rc=$?"; exit 1; }
  python -c "
import json
for l in open('gpurun_out/ab_$name.log'):
    if l.startswith('{'):
        d=json.loads(l); h=d['macro_step_host_us']; print('$name', d['value'], d['ms_per_step'], h['launch_and_wait_us'], h['emulators_us'])
"; done; done
if [ -n "${TRACE:-}" ]; then timeout -k 10 100 python tools/host_trace.py > gpurun_out/host_trace.txt 2>&1; tail -13 gpurun_out/host_trace.txt; fi
