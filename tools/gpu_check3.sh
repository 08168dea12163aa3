#!/bin/bash
# GPU-box check: the whole GPU suite, then the configs[2], configs[3] (one GPU) and stream lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-g}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
for w in tick cfg3 stream; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > gpurun_out/${TAG}_$w.json 2> gpurun_out/${TAG}_$w.err \
      || { tail -20 gpurun_out/${TAG}_$w.err; exit 2; }
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_$w.json')); print('$w', round(d['ms_per_step']*1e3, 2), 'us/tick', round(d['value']/1e9, 2), 'G/s', d.get('roofline', {}).get('frac'), d['tick'].get('kernels_avg_ms', d['tick'].get('kernels_us_per_tick')))"
done
