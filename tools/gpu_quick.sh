#!/bin/bash
# GPU-box check after a change: the whole GPU suite, then the stream line and the host split.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-q}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python -u bench.py --workload stream > gpurun_out/${TAG}_stream.json 2> gpurun_out/${TAG}_stream.err \
    || { tail -20 gpurun_out/${TAG}_stream.err; exit 2; }
cat gpurun_out/${TAG}_stream.json
FAASBAL_STAGE_PROF=1 timeout -k 10 300 python -u tools/stream_probe.py --pinned > gpurun_out/${TAG}_probe.log 2>&1 || { tail -20 gpurun_out/${TAG}_probe.log; exit 3; }
tail -3 gpurun_out/${TAG}_probe.log
