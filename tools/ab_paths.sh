#!/bin/bash
# A/B of fb_set_path knobs (FAASBAL_PATHS) with one library, alternated on one box: the
# committed and uncommitted per-tick times and the commit's in-tick delta (bench.py).
#   AB_ARGS="--workload cfg3" bash tools/ab_paths.sh TAG "qtiles=1" "" ...   ("" = defaults)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=$1; shift
for rep in 1 2 3; do
  for P in "$@"; do
    FAASBAL_PATHS="$P" timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-observed $AB_ARGS > gpurun_out/${TAG}_ab.json 2> gpurun_out/${TAG}_ab.err || { tail -5 gpurun_out/${TAG}_ab.err; exit 3; }
    python -c "import json; d=json.loads(open('gpurun_out/${TAG}_ab.json').read().strip().splitlines()[-1]); c=d.get('committed',{}); print('[$P]', 'committed %.2f' % (d['ms_per_step']*1e3), 'uncommitted %.2f' % (d.get('uncommitted',{}).get('ms_per_step',0)*1e3), 'commit %.2f' % (c.get('commit_in_tick_ms',0)*1e3), {k: round(v*1e3,2) for k,v in d['tick']['kernels_avg_ms'].items()})" | tee -a gpurun_out/${TAG}_ab.log
  done
done
