#!/bin/bash
# poll interval of the conv blocks' wait for their env's publication (s_sleep 8 in the product):
# sl2 / sl16 — on the driver's Pong line (launch + wait per macro-step)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VARIANTS="base sl2 sl16" CONFIGS="pong-nips" N=3 TAG=c54 bash tools/ab_lib.sh
