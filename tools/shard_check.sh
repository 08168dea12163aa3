#!/bin/bash
# Sharded path: its GPU tests (one GPU, rank contexts; multi-process over gloo), then the
# per-rank probe at configs[3] and configs[2].  Each step has its own time limit.
#   bash tools/shard_check.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
T=${1:-sh}
timeout -k 10 1000 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_shard_dist.py tests/test_shard_dispatcher.py \
    "tests/test_full_size.py::test_gpu_sharded_16m_x_1m_matches_oracle" -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
timeout -k 10 400 python -u tools/shard_probe.py --workload cfg3 --reps 20 > gpurun_out/${T}_shard_cfg3.log 2>&1 || { tail -20 gpurun_out/${T}_shard_cfg3.log; exit 2; }
cat gpurun_out/${T}_shard_cfg3.log
timeout -k 10 300 python -u tools/shard_probe.py --reps 30 > gpurun_out/${T}_shard_c2.log 2>&1 || { tail -20 gpurun_out/${T}_shard_c2.log; exit 3; }
cat gpurun_out/${T}_shard_c2.log
