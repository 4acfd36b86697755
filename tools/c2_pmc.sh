set -u
OUT=gpurun_out/c2; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --config breakout-pwyx-figar-rgb --steps 20 --warmup 5 --no_cpu_baseline --trunk_sweep '' > $OUT/bench_pwyx.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config mspacman-lstm-figar --steps 20 --warmup 5 --no_cpu_baseline --trunk_sweep '' > $OUT/bench_lstm.log 2>&1 || exit $?
PASS1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
PASS2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_MFMA"
PASS3="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_COUNT"
NAME=c2/pmc_fwd PASSES="$PASS1;$PASS2;$PASS3" timeout -k 10 400 bash tools/pmc_any.sh tools/sweep_only.py --config breakout-pwyx-figar-rgb --envs 32 --reps 10 > $OUT/pmc_fwd.log 2>&1 || exit $?
NAME=c2/pmc_bwd PASSES="$PASS1;$PASS2;$PASS3" timeout -k 10 400 bash tools/pmc_any.sh tools/bwd_only.py --config breakout-pwyx-figar-rgb --reps 10 > $OUT/pmc_bwd.log 2>&1 || exit $?
