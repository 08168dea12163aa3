#!/bin/bash
# Same-box A/B of the stream line under environment settings: tools/ab_stream.sh TAG "ENV_A" "ENV_B" ...
# (each setting run twice, alternated; prints ms per tick and kernels per tick; AB_ARGS: extra bench args).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=$1; shift
for rep in 1 2; do
  i=0
  for e in "$@"; do
    i=$((i+1))
    env $e timeout -k 10 300 python -u bench.py --workload stream $AB_ARGS > gpurun_out/${TAG}_${i}_${rep}.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_${i}_${rep}.json')); print('%-28s %.1f us/tick, kernels %.1f' % ('$e', d['ms_per_step']*1e3, d['tick'].get('device_us_per_tick', d['tick'].get('device_ms', 0) * 1e3)))"
  done
done
