#!/bin/bash
# tile configurations of the unpooled 5x5 dX (MT_DX_CFG = WM, WN, TMW, CK): base 4,2,2,32;
# dxa 4,1,2,32 (4 waves, 4 accumulators); dxb 4,2,2,160 (5 taps per weight chunk); dxc 8,1,1,32
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VARIANTS="base dxa dxb dxc" CONFIGS="mspacman-lstm-figar" N=2 TAG=c27 bash tools/ab_lib.sh
