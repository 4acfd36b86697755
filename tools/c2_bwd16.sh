# r06: 16-wave nips_conv_bwd_kernel — parity subset, then kernel-trace A/B (old vs base), then bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_e2e_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "pong or NIPS" > gpurun_out/r06c2_tests.log 2>&1 && \
REPS=20 CONFIG=pong-nips VARIANTS="old" bash tools/variant_prof.sh && \
cp manette_amd/libmanette_hip.so manette_amd/libmanette_hip_new.so && REPS=20 CONFIG=pong-nips VARIANTS="new" bash tools/variant_prof.sh && \
VARIANTS="old base" CONFIGS="pong-nips" N=2 TAG=r06c2 bash tools/ab_lib.sh
