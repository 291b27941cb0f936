#!/bin/bash
# Multi-rank rehearsal of the bench on a one-GPU box: torchrun with 2 and 4 ranks on GPU 0
# (gloo process group: RCCL refuses two ranks on one GPU), default strong scaling (65,536
# chains split over the ranks).  The lines say "REHEARSAL ... same device".
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 3 \
      --warmup 1 --backend gloo --same-device \
      > gpurun_out/rehearse_$n.json 2> gpurun_out/rehearse_$n.err || { echo "n=$n failed"; tail -20 gpurun_out/rehearse_$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/rehearse_$n.json').read().strip().splitlines()[-1]); print(d['n_gpus'], d['scaling'], d['config']['chains_total'], d['config']['chains_per_gpu'], '%.4g' % d['value'], d['hist_yields'], d['config']['parallelism'])"
done
