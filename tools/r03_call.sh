#!/bin/bash
# Round-3 GPU call driver: each step under its own time limit; a fault-like exit (timeout 124/137,
# abort 134, segfault 139) stops the sequence, a test failure (rc 1) does not.
#   STEPS="repro diag tests bench" OUT=gpurun_out/c1 bash tools/r03_call.sh
set -u
OUT=${OUT:-gpurun_out/r03}
mkdir -p "$OUT"
: > "$OUT/suite.log"
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a "$OUT/suite.log"
  case $rc in 124|137|134|139) echo "fault-like exit in $name, stopping" | tee -a "$OUT/suite.log"; exit $rc;; esac
  return 0
}
for step in ${STEPS:-tests bench}; do
  case $step in
    repro) run repro1 60 tools/bin/gemm_repro1; run repro0 60 tools/bin/gemm_repro0 ;;
    diag) MANETTE_HIP_LIB=$PWD/manette_amd/libmanette_hip_olddual.so run diag_olddual 180 python tools/dual_diag.py "$OUT/diag_olddual.npz"
          run diag_new 180 python tools/dual_diag.py "$OUT/diag_new.npz" ;;
    bar) run bar 60 tools/bin/bar_probe ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run tests 1200 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread ${TEST_ARGS:-} ;;
    bench) run bench 600 python bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS:-} ;;
    benchcfg) for c in ${CONFIGS:-}; do run "bench_$c" 600 python bench.py --config "$c" --steps 20 --warmup 5 --no_cpu_baseline; done ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no_cpu_baseline ;;
  esac
done
