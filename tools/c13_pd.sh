set -o pipefail
cd $GRAFT_REPO_ROOT
ENV_pd4="MH_PREFETCH_ROWS=4" ENV_pd8="MH_PREFETCH_ROWS=8" VARIANTS="base pd4 pd8" CONFIGS="pong-nips breakout-nature-figar" N=2 TAG=r06pd bash tools/ab_host.sh
