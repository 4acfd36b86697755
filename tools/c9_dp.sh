# round-3 call: rehearsal of bench.py's N > 1 path on one GPU (2 ranks on cuda:0, gloo all-reduce):
# the launcher command the driver uses, with --comm torch (RCCL refuses two ranks on one GPU)
set -u
OUT=gpurun_out/c9; mkdir -p $OUT
export TMPDIR=/tmp MT_BENCH_SHARED_GPU=1
for c in pong-nips mspacman-lstm-figar; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 2 --steps 10 --warmup 3 --config $c --comm torch --no_cpu_baseline --trunk_sweep '' > $OUT/dp2_$c.log 2>&1 || exit $?
done
