#!/bin/bash
# The driver's N-GPU bench command rehearsed with 2 ranks on one GPU (gloo all-reduce; RCCL refuses
# two ranks on one device): both ranks run the native rollout and the bucketed update side by side.
set -u
mkdir -p gpurun_out
MT_BENCH_SHARED_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --comm torch --steps 10 --warmup 3 \
  --no_cpu_baseline ${ARGS:-} > gpurun_out/${TAG:-dp2}.log 2>&1
echo "dp2 rc=$?"
