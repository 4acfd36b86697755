# round-3 call: persistent one-chunk direct conv (conv1: weights staged once per block)
set -u
OUT=gpurun_out/c8; mkdir -p $OUT
export TMPDIR=/tmp
# (tests: green in the first c8 run)
for v in product nopersist; do
  L=$PWD/manette_amd/libmanette_hip_$v.so; [ $v = product ] && L=$PWD/manette_amd/libmanette_hip.so
  for c in breakout-pwyx-figar-rgb mspacman-lstm-figar; do
    MANETTE_HIP_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/sweep_${v}_$c -o run -- python3 tools/sweep_only.py --config $c --envs 32 --reps 20 > $OUT/sweep_${v}_$c.log 2>&1 || exit $?
  done
done
PASS1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
PASS2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_MFMA"
NAME=c8/pmc_bwd_lstm PASSES="$PASS1;$PASS2" timeout -k 10 400 bash tools/pmc_any.sh tools/bwd_only.py --config mspacman-lstm-figar --reps 5 > $OUT/pmc_bwd_lstm.log 2>&1 || exit $?
NAME=c8/pmc_fwd_pwyx PASSES="$PASS1;$PASS2" timeout -k 10 400 bash tools/pmc_any.sh tools/sweep_only.py --config breakout-pwyx-figar-rgb --envs 32 --reps 10 > $OUT/pmc_fwd_pwyx.log 2>&1 || exit $?
