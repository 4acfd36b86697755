#!/bin/bash
# dense-layer gradient tiles: dA = dW on 64 x 64 tiles; dB = dX on 32 x 64; dC = dW with 160-deep chunks
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VARIANTS="base dA dB dC" CONFIGS="breakout-nature-figar seaquest-nature pong-nips" N=2 TAG=c34 bash tools/ab_lib.sh
