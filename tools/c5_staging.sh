set -o pipefail
cd $GRAFT_REPO_ROOT
MANETTE_HIP_LIB=manette_amd/libmanette_hip_probe.so timeout -k 10 180 python -u tools/probe.py --config pong-nips --isolated > gpurun_out/r06c5_probe_iso.txt 2>&1 && \
MANETTE_HIP_LIB=manette_amd/libmanette_hip_probe.so timeout -k 10 180 python -u tools/probe.py --config pong-nips > gpurun_out/r06c5_probe_loop.txt 2>&1 && \
STAGINGS="resized pooled zero_copy" CONFIGS="pong-nips breakout-nature-figar" N=1 TAG=r06st bash tools/ab_staging.sh
