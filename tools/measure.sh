#!/bin/bash
# Measurement pass on one box (no test suite): the default bench line, the stream line,
# the configs[3] line and the per-rank sharded probe at configs[3].  Each step has its
# own time limit; the chain stops at the first failure.
#   bash tools/measure.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
T=${1:-m}
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 3; }
cat gpurun_out/${T}_bench.json
timeout -k 10 300 python -u bench.py --workload stream --no-cpu-baseline > gpurun_out/${T}_stream.json 2> gpurun_out/${T}_stream.err || { tail -20 gpurun_out/${T}_stream.err; exit 4; }
cat gpurun_out/${T}_stream.json
timeout -k 10 300 python -u bench.py --workload cfg3 --no-cpu-baseline > gpurun_out/${T}_cfg3.json 2> gpurun_out/${T}_cfg3.err || { tail -20 gpurun_out/${T}_cfg3.err; exit 5; }
cat gpurun_out/${T}_cfg3.json
timeout -k 10 400 python -u tools/shard_probe.py --workload cfg3 --reps 20 --gated > gpurun_out/${T}_shard_cfg3.log 2>&1 || { tail -20 gpurun_out/${T}_shard_cfg3.log; exit 6; }
cat gpurun_out/${T}_shard_cfg3.log
