#!/bin/bash
# Window / stream path: its GPU tests, then the configs[4] stream bench line (twice).
#   bash tools/stream_check.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
T=${1:-st}
timeout -k 10 700 python -u -m pytest tests/test_gpu_window.py "tests/test_full_size.py::test_gpu_stream_1m_workers_matches_oracle" \
    tests/test_gpu_resident.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 \
    || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --workload stream --no-cpu-baseline > gpurun_out/${T}_stream$i.json 2> gpurun_out/${T}_stream$i.err || { tail -20 gpurun_out/${T}_stream$i.err; exit 3; }
  python -c "import json; d=json.load(open('gpurun_out/${T}_stream$i.json')); print(round(d['ms_per_step']*1e3,2), 'us/tick', {k: round(v,1) for k,v in d['tick']['kernels_us_per_tick'].items()}, d['roofline']['frac'], d['roofline']['tick_frac'])"
done
