#!/usr/bin/env bash
# Round 4: RCCL inside the captured UL-leg graph on one GPU: torchrun world size 1 (nccl backend = RCCL), the per-set
# TB gather captured in the leg graphs (--graph-collectives, default), then the same with the gather between launches.
set -o pipefail
mkdir -p gpurun_out
PB="--no-cpu-baseline --no-extra-points --no-extra-workloads --steps 40 --warmup 4 --min-time 0 --tb-gather always"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 1 $PB > gpurun_out/r4n_nccl_graph.json 2> gpurun_out/r4n_nccl_graph.err || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29518 bench.py --gpus 1 $PB --no-graph-collectives > gpurun_out/r4n_nccl_eager.json \
  2> gpurun_out/r4n_nccl_eager.err
