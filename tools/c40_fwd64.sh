#!/bin/bash
# smaller tiles for the 64-channel direct forwards: g1 = conv4 on 1 x 4 waves (4 units a block);
# g2 / g3 = conv3 (pooled) on 2 x 2 / 1 x 4 waves
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VARIANTS="base g1 g2 g3" CONFIGS="mspacman-lstm-figar breakout-pwyx-figar-rgb" N=2 TAG=c40 bash tools/ab_lib.sh
