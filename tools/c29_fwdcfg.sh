#!/bin/bash
# tile sweeps of the direct forward convs (PWYX / LSTM trunk): fa = 32 -> 32 on 8 x 1 waves; fb = the
# pooled 64-channel layer on 8 x 1; fc / fd = the unpooled 64-channel layer on 4 x 2 / 8 x 1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VARIANTS="base fa fb fc fd" CONFIGS="mspacman-lstm-figar breakout-pwyx-figar-rgb" N=2 TAG=c29 bash tools/ab_lib.sh
