set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_lstm_gpu.py tests/test_dp_gpu.py tests/test_e2e_gpu.py -x -q --timeout 300 --timeout-method thread -k "norm_partials or launch_by_launch or registration or e2e" > gpurun_out/r06c10_tests.log 2>&1 && \
bash tools/c8_rowfc.sh && \
BENCH_ARGS="--pin_threads on" VARIANTS="base" CONFIGS="pong-nips breakout-nature-figar" N=2 TAG=r06pin_on bash tools/ab_host.sh && \
VARIANTS="base" CONFIGS="pong-nips breakout-nature-figar" N=2 TAG=r06pin_auto bash tools/ab_host.sh
