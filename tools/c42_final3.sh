#!/bin/bash
# round-6 final measurement set after the LSTM x-product cache and the conv4 tiles: smoke + the whole GPU suite, then every config's
# bench line with its CPU baseline (one box), then the 2-rank rehearsal of the N-GPU command
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06fc3 STEPS="smoke tests" bash tools/gpu_suite.sh || exit $?
TAG=r06fc3 CPU_ALL=1 bash tools/bench_all.sh || exit $?
TAG=r06fc3_dp2_lstm ARGS="--config mspacman-lstm-figar" bash tools/dp2_rehearsal.sh
