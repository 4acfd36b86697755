#!/bin/bash
# the backward-data k state only for CIN >= 64 (the thin CIN-32 tile back to 128 VGPRs): A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VARIANTS="base ks64" CONFIGS="mspacman-lstm-figar breakout-pwyx-figar-rgb" N=2 TAG=c32 bash tools/ab_lib.sh
