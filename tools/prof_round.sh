#!/bin/bash
# Round-4 measurements: the default bench line, then the configs[2] and configs[3]
# kernel traces + FETCH / WRITE passes (summaries into profiles/), then the stream's.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
T=${1:-r04}
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 3; }
cat gpurun_out/${T}_bench.json
timeout -k 10 180 python -u tools/stamps.py --reps 50 > gpurun_out/${T}_stamps.txt 2>&1 || { tail -20 gpurun_out/${T}_stamps.txt; exit 4; }
bash tools_profile.sh ${T}_c2 > gpurun_out/${T}_prof_c2.log 2>&1 || { tail -20 gpurun_out/${T}_prof_c2.log; exit 5; }
bash tools_profile.sh ${T}_c3 --workload cfg3 > gpurun_out/${T}_prof_c3.log 2>&1 || { tail -20 gpurun_out/${T}_prof_c3.log; exit 6; }
timeout -k 10 300 python -u bench.py --workload cfg3 --no-cpu-baseline > gpurun_out/${T}_cfg3.json 2> gpurun_out/${T}_cfg3.err || { tail -20 gpurun_out/${T}_cfg3.err; exit 7; }
cat gpurun_out/${T}_cfg3.json
bash tools/prof_pmc.sh ${T}_stream --workload stream --no-pcie-pass --steps 20 --warmup 3 > gpurun_out/${T}_spmc.txt 2>&1 \
    || { tail -20 gpurun_out/${T}_spmc.txt; exit 8; }
tail -12 gpurun_out/${T}_spmc.txt
