set -o pipefail
cd $GRAFT_REPO_ROOT
ENV_pd4="MH_PREFETCH_ROWS=4" VARIANTS="old base pd4" CONFIGS="pong-nips" N=2 TAG=r06h2 bash tools/ab_host.sh && \
VARIANTS="old base" CONFIGS="breakout-nature-figar" N=2 TAG=r06h2 bash tools/ab_host.sh
