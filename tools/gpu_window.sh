#!/bin/bash
# GPU-box check of the window ticks: their parity tests, then the full suite, smoke and
# the stream line.  Each step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-win}
timeout -k 10 300 python -u -m pytest tests/test_gpu_window.py -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_win.log 2>&1 || { tail -40 gpurun_out/${TAG}_win.log; exit 1; }
tail -3 gpurun_out/${TAG}_win.log
timeout -k 10 300 python -u -m pytest tests/test_full_size.py -x -v --timeout 200 --timeout-method thread -k stream \
    > gpurun_out/${TAG}_full.log 2>&1 || { tail -40 gpurun_out/${TAG}_full.log; exit 2; }
tail -3 gpurun_out/${TAG}_full.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 4; }
tail -2 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python -u bench.py --workload stream > gpurun_out/${TAG}_stream.json 2> gpurun_out/${TAG}_stream.err \
    || { tail -20 gpurun_out/${TAG}_stream.err; exit 3; }
cat gpurun_out/${TAG}_stream.json
timeout -k 10 300 python -u tools/stream_probe.py --pinned > gpurun_out/${TAG}_probe.log 2>&1 || { tail -20 gpurun_out/${TAG}_probe.log; exit 5; }
cat gpurun_out/${TAG}_probe.log
FAASBAL_COMMIT_NOW=1 timeout -k 10 300 python -u bench.py --workload stream > gpurun_out/${TAG}_stream_cnow.json 2>/dev/null || exit 6
python -c "import json; d=json.load(open('gpurun_out/${TAG}_stream_cnow.json')); print('commit_now', d['ms_per_step'], d['tick']['kernels_us_per_launch'])"
