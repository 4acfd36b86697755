#!/bin/bash
# round-6 closing set at the last code (NATURE heads on 8 waves): smoke + the whole GPU suite, every config's bench line
# with its CPU baseline, the 2-rank rehearsal, then the windowed rocprof of the driver's command
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06fc7 STEPS="smoke tests" bash tools/gpu_suite.sh || exit $?
TAG=r06fc7 CPU_ALL=1 bash tools/bench_all.sh || exit $?
TAG=r06fc7_dp2_pong bash tools/dp2_rehearsal.sh || exit $?
bash tools/prof_driver.sh r06fc7_prof_driver > gpurun_out/r06fc7_prof_driver.rc 2>&1
