#!/bin/bash
# One GPU-box pass over every measurement DESIGN.md quotes: parity suite + smoke +
# default bench (tools/gpu_check.sh), the other bench workloads, the sharded
# per-rank probe, the launch-floor calibration, then the rocprof profile passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-rm}
bash tools/gpu_check.sh $TAG || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline --workers 1048576 --tasks 16000000 --steps 100 > gpurun_out/${TAG}_big.json 2>/dev/null || exit 2
timeout -k 10 200 python -u bench.py --mode deque > gpurun_out/${TAG}_deque.json 2>/dev/null || exit 3
timeout -k 10 300 python -u bench.py --workload stream > gpurun_out/${TAG}_stream.json 2>/dev/null || exit 4
timeout -k 10 200 python -u tools/shard_probe.py --world 2 4 8 > gpurun_out/${TAG}_shard.log 2>/dev/null || exit 5
timeout -k 10 200 python -u tools/host_rate_probe.py --world 1 2 4 8 > gpurun_out/${TAG}_hrp.log 2>/dev/null || exit 6
hipcc --offload-arch=gfx950 -O3 tools/microbench.hip -o gpurun_out/microbench && timeout -k 10 120 gpurun_out/microbench > gpurun_out/${TAG}_micro.log || exit 7
rm -f gpurun_out/microbench
bash tools_profile.sh ${2:-r01_v14} || exit 8
