#!/bin/bash
# One iteration on the stream path: window / resident / full-size stream tests, the stream
# bench (HBM-resident batches) and its FETCH / WRITE passes.  Each step time-limited.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-it}
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_resident.py tests/test_gpu_window.py \
    tests/test_full_size.py tests/test_gpu_parity.py > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python -u bench.py --workload stream --no-cpu-baseline --no-pcie-pass > gpurun_out/${TAG}_stream.json 2> gpurun_out/${TAG}_stream.err \
    || { tail -20 gpurun_out/${TAG}_stream.err; exit 2; }
cat gpurun_out/${TAG}_stream.json
if [ "${PMC:-1}" = 1 ]; then
  bash tools/prof_pmc.sh ${TAG} --workload stream --no-pcie-pass --steps 20 --warmup 3 > gpurun_out/${TAG}_pmc.txt 2>&1 || { tail -20 gpurun_out/${TAG}_pmc.txt; exit 3; }
  grep -v rocclr gpurun_out/${TAG}_pmc.txt | tail -12
fi
