#!/bin/bash
# Rehearse bench.py's N>1 path on a one-GPU box: N ranks share cuda:0 over gloo
# (RCCL refuses two ranks on one device).  The driver runs the real N>1 case
# with RCCL on an 8-GPU node.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for N in ${NS:-2 4}; do
  timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
      --master-port $((29500 + N)) bench.py --gpus $N --steps ${STEPS:-50} --warmup 5 --backend gloo \
      > gpurun_out/tr_n$N.json 2> gpurun_out/tr_n$N.err || { tail -30 gpurun_out/tr_n$N.err; exit 1; }
  cat gpurun_out/tr_n$N.json
done
