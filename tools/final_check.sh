#!/bin/bash
# Round-end check on the GPU box: smoke, the whole GPU suite and the default bench (gpu_suite.sh,
# OUT=gpurun_out/<tag>), then the 2-rank rehearsal of the N-GPU bench command on Pong and Seaquest.
set -u
TAG=${1:-final}
OUT=gpurun_out/$TAG STEPS="smoke tests bench" bash tools/gpu_suite.sh || exit $?
TAG=${TAG}_dp2_pong bash tools/dp2_rehearsal.sh || exit $?
TAG=${TAG}_dp2_seaquest ARGS="--config seaquest-nature" bash tools/dp2_rehearsal.sh
