#!/bin/bash
# A/B of env-switched variants at a chosen size: tools/ab_big.sh "<bench args>" "ENV=1" "ENV=0" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
BA=$1; shift
for v in "$@"; do
  env $v timeout -k 10 150 python -u bench.py --no-cpu-baseline $BA > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 3; }
  python -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); print('$v', 'us/tick %.2f' % (d['ms_per_step']*1e3), {k: round(v*1e3,2) for k,v in d['tick']['kernels_avg_ms'].items()}, 'dom %s frac %.3f' % (d['roofline']['kernel'], d['roofline']['frac']))"
done
