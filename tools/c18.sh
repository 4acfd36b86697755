# round-3 call: gray conv1 weight gradient on 4 M-tiles per wave (one tap group, no empty slots)
set -u
OUT=gpurun_out/c18; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -k "lstm or LSTM or PWYX" > $OUT/tests.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/bwd_lstm -o run -- python3 tools/bwd_only.py --config mspacman-lstm-figar --reps 10 > $OUT/bwd_lstm.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config mspacman-lstm-figar --steps 20 --warmup 5 --no_cpu_baseline > $OUT/bench_lstm.log 2>&1 || exit $?
