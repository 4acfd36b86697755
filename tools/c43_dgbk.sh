#!/bin/bash
# chunk depth of the generic backward-data GEMM (TileConvDgrad BK; product 64): dg128 / dg32
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VARIANTS="base dg128 dg32" CONFIGS="mspacman-lstm-figar breakout-pwyx-figar-rgb breakout-nature-figar" N=2 TAG=c43 bash tools/ab_lib.sh
