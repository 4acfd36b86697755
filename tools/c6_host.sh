set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_e2e_gpu.py -x -q --timeout 120 --timeout-method thread -k "breakout or pong" > gpurun_out/r06c6_tests.log 2>&1 && \
ENV_pd4="MH_PREFETCH_ROWS=4" VARIANTS="old base pd4" CONFIGS="pong-nips" N=2 TAG=r06h bash tools/ab_host.sh && \
VARIANTS="old base" CONFIGS="breakout-nature-figar" N=2 TAG=r06h bash tools/ab_host.sh && \
STAGINGS="pooled" CONFIGS="pong-nips breakout-nature-figar" N=1 TAG=r06st2 bash tools/ab_staging.sh
