# r06: row_fc_kernel with 16-env tiles (MT_ROWFC_BM=16) vs 32 on the layered trunks' roofline launch
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for c in seaquest-nature breakout-nature-figar breakout-pwyx-figar-rgb; do for v in base fc16; do
  L=$GRAFT_REPO_ROOT/manette_amd/libmanette_hip_$v.so; [ $v = base ] && L=$GRAFT_REPO_ROOT/manette_amd/libmanette_hip.so
  (cd /tmp && MANETTE_HIP_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/rf_${v}_$c -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/trunk_only.py --config $c --reps 50 > $GRAFT_REPO_ROOT/gpurun_out/rf_${v}_$c.log 2>&1) || exit 1
done; done && \
VARIANTS="base fc16" CONFIGS="seaquest-nature" N=2 TAG=r06rf bash tools/ab_lib.sh
