#!/bin/bash
# Stamps of the sharded phase-2 emission at configs[3], world 2 / 8 (stamps build first).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
T=${1:-ss}
for w in 2 8; do
  timeout -k 10 300 python -u tools/stamps_shard.py --workload cfg3 --world $w --reps 10 > gpurun_out/${T}_w$w.txt 2>&1 || { tail -20 gpurun_out/${T}_w$w.txt; exit 1; }
  cat gpurun_out/${T}_w$w.txt
done
