#!/bin/bash
# LSTM x-product split count (pick_splits target; product 128 -> ~50 slabs): xg16 / xg32 / xg64
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VARIANTS="base xg16 xg32 xg64" CONFIGS="mspacman-lstm-figar" N=2 TAG=c38 bash tools/ab_lib.sh
