#!/bin/bash
# K-splits of the NATURE / PWYX dense layer (row_fc_kernel; product 7 / 10 = one per conv row):
# s4 = 4 (256 blocks at E = 32), s8 = 8 (512: two per CU)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VARIANTS="base s4 s8" CONFIGS="seaquest-nature breakout-nature-figar breakout-pwyx-figar-rgb" N=2 TAG=c49 bash tools/ab_lib.sh
