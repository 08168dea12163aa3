#!/bin/bash
# Round-3 closing measurements on one box: the whole GPU suite, smoke, the default bench
# line (configs[2]), the stream line (HBM-resident value + PCIe-inclusive pass), then the
# configs[2] kernel trace + FETCH / WRITE passes (tools_profile.sh) and the stream's
# (tools/prof_pmc.sh).  Each step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-fin}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 \
    || { tail -20 gpurun_out/${TAG}_smoke.log; exit 2; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
    || { tail -20 gpurun_out/${TAG}_bench.err; exit 3; }
cat gpurun_out/${TAG}_bench.json
timeout -k 10 300 python -u bench.py --workload stream --no-cpu-baseline > gpurun_out/${TAG}_stream.json 2> gpurun_out/${TAG}_stream.err \
    || { tail -20 gpurun_out/${TAG}_stream.err; exit 4; }
cat gpurun_out/${TAG}_stream.json
bash tools_profile.sh ${TAG}_c2 > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 5; }
bash tools/prof_pmc.sh ${TAG}_stream --workload stream --no-pcie-pass --steps 20 --warmup 3 > gpurun_out/${TAG}_spmc.txt 2>&1 \
    || { tail -20 gpurun_out/${TAG}_spmc.txt; exit 6; }
grep -v rocclr gpurun_out/${TAG}_spmc.txt | tail -8
