#!/bin/bash
# A round's measurement pass: the default bench line, stamps of the configs[2] tick, then
# kernel traces + FETCH / WRITE passes of configs[2], configs[3] and the configs[4] stream
# (tools_profile.sh; summaries into profiles/<tag>_* and profiles/traffic.json, which the
# bench lines read back as roofline.traffic), then the configs[3] and stream bench lines.
#   bash tools/prof_round.sh TAG   (then: python tools/prof_summary.py gpurun_out/prof_TAG_xx TAG_xx)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
T=${1:-r05}
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 3; }
cat gpurun_out/${T}_bench.json
timeout -k 10 180 python -u tools/stamps.py --reps 50 > gpurun_out/${T}_stamps.txt 2>&1 || { tail -20 gpurun_out/${T}_stamps.txt; exit 4; }
bash tools_profile.sh ${T}_c2 > gpurun_out/${T}_prof_c2.log 2>&1 || { tail -20 gpurun_out/${T}_prof_c2.log; exit 5; }
bash tools_profile.sh ${T}_c3 --workload cfg3 > gpurun_out/${T}_prof_c3.log 2>&1 || { tail -20 gpurun_out/${T}_prof_c3.log; exit 6; }
bash tools_profile.sh ${T}_st --workload stream --no-pcie-pass > gpurun_out/${T}_prof_st.log 2>&1 || { tail -20 gpurun_out/${T}_prof_st.log; exit 7; }
timeout -k 10 300 python -u bench.py --workload cfg3 --no-cpu-baseline > gpurun_out/${T}_cfg3.json 2> gpurun_out/${T}_cfg3.err || { tail -20 gpurun_out/${T}_cfg3.err; exit 8; }
cat gpurun_out/${T}_cfg3.json
timeout -k 10 300 python -u bench.py --workload stream --no-cpu-baseline > gpurun_out/${T}_stream.json 2> gpurun_out/${T}_stream.err || { tail -20 gpurun_out/${T}_stream.err; exit 9; }
cat gpurun_out/${T}_stream.json
