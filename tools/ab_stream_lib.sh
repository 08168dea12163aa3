#!/bin/bash
# Stream bench (configs[4] per GPU) with several library builds, one process each, alternated
# 3 times: tools/ab_stream_lib.sh A.so B.so ...   (paths relative to the repo)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-3}); do
  for L in "$@"; do
    FAASBAL_LIB=$R/$L timeout -k 10 150 python -u bench.py --workload stream --steps 30 --warmup 3 > gpurun_out/abs.json 2> gpurun_out/abs.err || { tail -5 gpurun_out/abs.err; exit 3; }
    python3 -c "import json; d=json.load(open('gpurun_out/abs.json')); print('$(basename $L)', 'us/tick %.1f' % (d['ms_per_step']*1e3), 'dev %.1f' % d['tick']['device_us_per_tick'], {k: round(v,1) for k,v in d['tick']['kernels_us_per_tick'].items()})"
  done
done
