#!/bin/bash
# Device-resident batches: their tests, the window tests, the stream bench (HBM-resident
# value + PCIe-inclusive pass) and the resident stream timeline.  Each step time-limited.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-res}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_resident.py tests/test_gpu_window.py > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python -u bench.py --workload stream --no-cpu-baseline > gpurun_out/${TAG}_stream.json 2> gpurun_out/${TAG}_stream.err \
    || { tail -20 gpurun_out/${TAG}_stream.err; exit 2; }
cat gpurun_out/${TAG}_stream.json
bash tools/stream_timeline.sh ${TAG}_tl --resident > gpurun_out/${TAG}_tl.txt 2>&1 || { tail -20 gpurun_out/${TAG}_tl.txt; exit 3; }
cat gpurun_out/${TAG}_tl.txt
