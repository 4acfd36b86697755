#!/bin/bash
# dense dX chunk depth: xA = 256 (2 chunks at F = 512), xB = 64 (product 128)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VARIANTS="base xA xB" CONFIGS="breakout-nature-figar seaquest-nature pong-nips" N=2 TAG=c37 bash tools/ab_lib.sh
