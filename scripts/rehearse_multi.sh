#!/bin/bash
# Multi-rank rehearsal of the bench on a one-GPU box: torchrun with 2 and 4 ranks on GPU 0
# (gloo process group: RCCL refuses two ranks on one GPU), then the plain N=1 line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 3 \
      --warmup 1 --chains 16384 --backend gloo --same-device \
      > gpurun_out/rehearse_$n.json 2> gpurun_out/rehearse_$n.err || { echo "n=$n failed"; tail -20 gpurun_out/rehearse_$n.err; exit 1; }
  cut -c1-260 gpurun_out/rehearse_$n.json
done
