#!/bin/bash
# generic conv weight-gradient knobs: nA / nB = 8 / 2 K-chunks per split block (product 4); nC = 128-deep chunks
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VARIANTS="base nA nB nC" CONFIGS="breakout-nature-figar seaquest-nature mspacman-lstm-figar" N=2 TAG=c36 bash tools/ab_lib.sh
