#!/bin/bash
# Stream bench (configs[4] per GPU) under several environment settings, one process each,
# alternated 4 times: tools/ab_stream_env.sh "VAR=a" "VAR=b" ...   (per-kernel us from the bench)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for rep in 1 2 3 4; do
  for V in "$@"; do
    env $V timeout -k 10 150 python -u bench.py --workload stream --steps 30 --warmup 3 > gpurun_out/abs.json 2> gpurun_out/abs.err || { tail -5 gpurun_out/abs.err; exit 3; }
    python3 -c "import json; d=json.load(open('gpurun_out/abs.json')); print('$V', 'us/tick %.1f' % (d['ms_per_step']*1e3), 'dev %.1f' % d['tick']['device_us_per_tick'], {k: round(v,1) for k,v in d['tick']['kernels_us_per_tick'].items()})"
  done
done
