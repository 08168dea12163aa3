#!/bin/bash
# A/B bench of env-switched variants on the GPU box: tools/ab.sh "ENV=1" "ENV=0" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for v in "$@"; do
  for rep in 1 2; do
    env $v timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 400 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 3; }
    python -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); print('$v', 'us/tick %.2f' % (d['ms_per_step']*1e3), {k: round(v*1e3,2) for k,v in d['tick']['kernels_avg_ms'].items()}, 'frac %.3f' % d['roofline']['frac'])"
  done
done
