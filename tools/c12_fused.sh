# r06: the NIPS trunk as one launch (conv blocks + fused dense tiles) — parity, phase tables, kernel
# trace of the roofline launch, bench A/B against the two-launch trunk (prev)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_e2e_gpu.py tests/test_kernels_gpu.py tests/test_probe_gpu.py tests/test_learner_gpu.py -x -q --timeout 300 --timeout-method thread -k "pong or NIPS or stacking or probe or native_step" > gpurun_out/r06c12_tests.log 2>&1 && \
MANETTE_HIP_LIB=manette_amd/libmanette_hip_probe.so timeout -k 10 180 python -u tools/probe.py --config pong-nips --isolated > gpurun_out/r06c12_probe_iso.txt 2>&1 && \
MANETTE_HIP_LIB=manette_amd/libmanette_hip_probe.so timeout -k 10 180 python -u tools/probe.py --config pong-nips > gpurun_out/r06c12_probe_loop.txt 2>&1 && \
for v in prev base; do L=$GRAFT_REPO_ROOT/manette_amd/libmanette_hip_$v.so; [ $v = base ] && L=$GRAFT_REPO_ROOT/manette_amd/libmanette_hip.so; (cd /tmp && MANETTE_HIP_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/tf_$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/trunk_only.py --config pong-nips --reps 50 > $GRAFT_REPO_ROOT/gpurun_out/tf_$v.log 2>&1) || exit 1; done && \
VARIANTS="prev base" CONFIGS="pong-nips" N=3 TAG=r06fu bash tools/ab_lib.sh
