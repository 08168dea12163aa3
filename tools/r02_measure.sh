#!/bin/bash
# Round-2 measurement pass (GPU box): full GPU suite + smoke + default bench (g5.sh),
# the other workloads, the sharded per-rank probe, the stream host split, stamps of
# configs[2], then kernel stats + PMC (FETCH_SIZE / WRITE_SIZE passes) of configs[2]
# and of the stream.  Every step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
T=${1:-r02}
bash tools/g5.sh $T || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --workers 1048576 --tasks 16000000 --steps 100 > gpurun_out/${T}_big.json 2>/dev/null || exit 2
timeout -k 10 200 python -u bench.py --mode deque --no-cpu-baseline > gpurun_out/${T}_deque.json 2>/dev/null || exit 3
timeout -k 10 300 python -u bench.py --workload stream > gpurun_out/${T}_stream.json 2>/dev/null || exit 4
timeout -k 10 300 python -u bench.py --workload stream --hb-frac 1.0 --steps 20 > gpurun_out/${T}_stream_storm.json 2>/dev/null || exit 5
timeout -k 10 200 python -u tools/shard_probe.py --world 2 4 8 > gpurun_out/${T}_shard.log 2>/dev/null || exit 6
timeout -k 10 200 python -u tools/stream_probe.py --pinned > gpurun_out/${T}_stream_probe.log 2>&1 || exit 7
timeout -k 10 200 python -u tools/stamps.py --reps 50 > gpurun_out/${T}_stamps.txt 2>&1 || exit 8
bash tools/prof_pmc.sh ${T}_c2 --steps 200 --warmup 20 > gpurun_out/${T}_pmc_c2.txt || exit 9
bash tools/prof_pmc.sh ${T}_stream --workload stream --steps 20 --warmup 3 > gpurun_out/${T}_pmc_stream.txt || exit 10
echo MEASURE_OK
