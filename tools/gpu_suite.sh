#!/bin/bash
# GPU-box sequence: smoke, gpu tests, bench. Each step has its own time limit; a fault-like
# exit (timeout 124/137, abort 134, segfault 139) stops the sequence, a test failure does not.
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a "$OUT/suite.log"
  case $rc in 124|137|134|139) echo "fault-like exit in $name, stopping" | tee -a "$OUT/suite.log"; exit $rc;; esac
  return 0
}
: > "$OUT/suite.log"
for step in ${STEPS:-smoke tests bench}; do
  case $step in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run tests 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread ;;
    bench) run bench 600 python bench.py ${BENCH_ARGS:-} ;;
    prof) run prof 600 bash tools/prof.sh ${PROF_NAME:-prof} ${PROF_ARGS:-} ;;
    pmc) run pmc 600 bash tools/pmc.sh ${PMC_NAME:-pmc} ${PMC_ARGS:-} ;;
    probe) MANETTE_HIP_LIB=$PWD/manette_amd/libmanette_hip_probe.so run probe 300 python tools/probe.py ${PROBE_ARGS:-} ;;
    variants)  # BENCH_VARIANTS="name1:args1;name2:args2" -> bench_<name>.log each
      IFS=';' read -ra VS <<< "${BENCH_VARIANTS:-}"
      for v in "${VS[@]}"; do run "bench_${v%%:*}" 300 python bench.py --no_cpu_baseline ${v#*:}; done ;;
  esac
done
