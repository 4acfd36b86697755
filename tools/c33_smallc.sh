#!/bin/bash
# M-tiles per wave of the 84x84 conv1 forward (DFwd / stack_conv1, 4 waves): s1 = 1, s4 = 4 (product 2)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VARIANTS="base s1 s4" CONFIGS="mspacman-lstm-figar breakout-pwyx-figar-rgb" N=2 TAG=c33 bash tools/ab_lib.sh
