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
    diag) MANETTE_HIP_LIB=$PWD/manette_amd/libmanette_hip_dual.so run diag_dual 180 python tools/dual_diag.py "$OUT/diag_dual.npz"
          run diag_product 180 python tools/dual_diag.py "$OUT/diag_product.npz"
          run repro1_real 60 tools/bin/gemm_repro1 "$OUT/diag_dual.npz"
          run repro0_real 60 tools/bin/gemm_repro0 "$OUT/diag_dual.npz"
          run dgrad1_real 60 tools/bin/dgrad_repro1 "$OUT/diag_dual.npz"
          run dgrad0_real 60 tools/bin/dgrad_repro0 "$OUT/diag_dual.npz"
          run dgrad1 60 tools/bin/dgrad_repro1 ;;
    ab) for v in ${VARIANTS:-base dual}; do  # bench of libmanette_hip_<v>.so beside the product, alternating
          MANETTE_HIP_LIB=$PWD/manette_amd/libmanette_hip_$v.so run "ab_$v" 300 python bench.py --no_cpu_baseline --trunk_sweep '' --steps 20 --warmup 5 --config ${AB_CONFIG:-pong-nips}
          run "ab_product_$v" 300 python bench.py --no_cpu_baseline --trunk_sweep '' --steps 20 --warmup 5 --config ${AB_CONFIG:-pong-nips}
        done ;;
    bar) run bar 60 tools/bin/bar_probe ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run tests 1200 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread ${TEST_ARGS:-} ;;
    vtests) for v in ${VARIANTS:-fb}; do  # GPU tests against libmanette_hip_<v>.so (VTK: a -k filter)
              MANETTE_HIP_LIB=$PWD/manette_amd/libmanette_hip_$v.so run "vtests_$v" 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread -k "${VTK:-NIPS or pong}"
            done ;;
    bench) run bench 600 python bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS:-} ;;
    benchcfg) for c in ${CONFIGS:-}; do run "bench_$c" 600 python bench.py --config "$c" --steps 20 --warmup 5 --no_cpu_baseline; done ;;
    prof) (export TMPDIR=/tmp; run prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5) ;;
    proflib) for v in ${VARIANTS:-product}; do for c in ${CONFIGS:-mspacman-lstm-figar}; do  # rocprof of a variant's bench
               L=$PWD/manette_amd/libmanette_hip_$v.so; [ "$v" = product ] && L=$PWD/manette_amd/libmanette_hip.so
               (export TMPDIR=/tmp MANETTE_HIP_LIB=$L; run "proflib_${v}_$c" 400 rocprofv3 --kernel-trace --stats -d "$OUT/proflib_${v}_$c" -o run -- python3 bench.py --config "$c" --steps 10 --warmup 3 --no_cpu_baseline --trunk_sweep '')
             done; done ;;
    pmc) for c in ${PMC_CONFIGS:-breakout-pwyx-figar-rgb}; do
           NAME=pmc_fwd_$c PASSES="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
             run "pmc_fwd_$c" 400 bash tools/pmc_any.sh tools/sweep_only.py --config "$c" --envs 32 --reps 10
         done ;;
    pbwd) MANETTE_HIP_LIB=$PWD/manette_amd/libmanette_hip_probe.so run probe_bwd 180 python tools/probe_bwd.py ;;
    probe) MANETTE_HIP_LIB=$PWD/manette_amd/libmanette_hip_probe.so run probe 300 python tools/probe.py ${PROBE_ARGS:-} ;;
    sweep) for c in ${SWEEP_CONFIGS:-breakout-pwyx-figar-rgb mspacman-lstm-figar}; do
             (export TMPDIR=/tmp; run "sweep_$c" 300 rocprofv3 --kernel-trace --stats -d "$OUT/sweep_$c" -o run -- python3 tools/sweep_only.py --config "$c" --envs 32 --reps 20)
           done ;;
  esac
done
