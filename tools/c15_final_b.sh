#!/bin/bash
# r06 final set, part B: smoke + the whole GPU suite + the default bench (final_check.sh), then the
# 2-rank rehearsals of the N-GPU bench command (Pong, Seaquest) with the placement / bounded setup
cd $GRAFT_REPO_ROOT
bash tools/final_check.sh r06fb
