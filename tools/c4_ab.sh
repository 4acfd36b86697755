# r06: parity subset on the product library (16-wave conv backward, 8-wave balanced conv1, 16-env fc
# tiles, padded JobPack), then kernel traces of the update (bwd_only) and of the roofline launch
# (trunk_only) for old / bwd16 / new, the bench A/B old vs base, and the LSTM bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_e2e_gpu.py tests/test_kernels_gpu.py tests/test_lstm_gpu.py -x -q --timeout 120 --timeout-method thread -k "pong or NIPS or norm_partials or stacking" > gpurun_out/r06c4_tests.log 2>&1 && \
REPS=20 CONFIG=pong-nips VARIANTS="old bwd16 new" bash tools/variant_prof.sh && \
for v in old new; do (cd /tmp && MANETTE_HIP_LIB=$GRAFT_REPO_ROOT/manette_amd/libmanette_hip_$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/tr_$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/trunk_only.py --config pong-nips --reps 50 > $GRAFT_REPO_ROOT/gpurun_out/tr_$v.log 2>&1) || exit 1; done && \
VARIANTS="old base" CONFIGS="pong-nips" N=2 TAG=r06c4 bash tools/ab_lib.sh && \
timeout -k 10 300 python bench.py --config mspacman-lstm-figar --no_cpu_baseline --trunk_sweep= --steps 20 > gpurun_out/r06c4_lstm.log 2>&1
