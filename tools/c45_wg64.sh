#!/bin/bash
# chunk depth of the generic weight gradient for 64 output channels (product 64): wg32 / wg128
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VARIANTS="base wg32 wg128" CONFIGS="mspacman-lstm-figar breakout-pwyx-figar-rgb breakout-nature-figar" N=2 TAG=c45 bash tools/ab_lib.sh
