#!/bin/bash
# A/B of environment settings on the stream bench (HBM-resident batches, eager commits),
# alternated twice: tools/ab_stream_env.sh TAG "VAR=a" "VAR=b" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=$1; shift
for rep in 1 2; do
  for V in "$@"; do
    env $V timeout -k 10 200 python -u bench.py --workload stream --no-cpu-baseline --no-pcie-pass --steps 40 \
        > gpurun_out/${TAG}.json 2> gpurun_out/${TAG}.err || { tail -5 gpurun_out/${TAG}.err; exit 1; }
    python3 - gpurun_out/${TAG}.json "$V" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["tick"]["kernels_us_per_tick"]
print("%-26s %.1f us/tick, device %.1f:" % (sys.argv[2], d["ms_per_step"] * 1e3, d["tick"]["device_us_per_tick"]),
      " ".join("%s %.1f" % (n, v) for n, v in k.items()), flush=True)
PY
  done
done
