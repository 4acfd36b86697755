#!/bin/bash
# round-6 closing set at the round's last code: smoke + the whole GPU suite, every config's bench line
# with its CPU baseline, the 2-rank rehearsal, then the windowed rocprof of the driver's command
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06fc4 STEPS="smoke tests" bash tools/gpu_suite.sh || exit $?
TAG=r06fc4 CPU_ALL=1 bash tools/bench_all.sh || exit $?
TAG=r06fc4_dp2_pong bash tools/dp2_rehearsal.sh || exit $?
bash tools/prof_driver.sh r06fc4_prof_driver > gpurun_out/r06fc4_prof_driver.rc 2>&1
