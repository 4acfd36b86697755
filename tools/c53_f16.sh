#!/bin/bash
# NIPS dense layer: 16 K-splits of 32-env tiles (256 blocks, each column block's weights read once)
# against the product's 8 K-splits of 16-env tiles
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VARIANTS="base f16" CONFIGS="pong-nips" N=3 TAG=c53 bash tools/ab_lib.sh
