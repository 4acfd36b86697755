set -o pipefail
cd $GRAFT_REPO_ROOT
export MANETTE_HIP_LIB=manette_amd/libmanette_hip_probe.so
timeout -k 10 180 python -u tools/probe.py --config pong-nips --isolated > gpurun_out/r06_probe_iso.txt 2>&1 && \
timeout -k 10 180 python -u tools/probe.py --config pong-nips > gpurun_out/r06_probe_loop.txt 2>&1 && \
unset MANETTE_HIP_LIB && \
timeout -k 10 400 bash tools/pmc_insts.sh r06_pmcinsts_pong pong-nips > gpurun_out/r06_pmcinsts.log 2>&1
