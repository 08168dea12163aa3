#!/bin/bash
# Host-side A/B on one box: the stream bench with eager commits on / off and polled /
# blocking waits (FAASBAL_WAIT_SPIN), alternated twice, then the configs[2] host split.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-ah}
for rep in 1 2; do
  for cfg in "1 " "1 --no-eager" "0 " "0 --no-eager"; do
    set -- $cfg
    SPIN=$1; shift
    FAASBAL_WAIT_SPIN=$SPIN timeout -k 10 200 python -u bench.py --workload stream --no-cpu-baseline --no-pcie-pass --steps 40 "$@" \
        > gpurun_out/${TAG}.json 2> gpurun_out/${TAG}.err || { tail -5 gpurun_out/${TAG}.err; exit 1; }
    python3 - gpurun_out/${TAG}.json "spin=$SPIN $*" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["tick"]["kernels_us_per_tick"]
print("%-22s %.1f us/tick, device %.1f:" % (sys.argv[2], d["ms_per_step"] * 1e3, d["tick"]["device_us_per_tick"]),
      " ".join("%s %.1f" % (n, v) for n, v in k.items()), flush=True)
PY
  done
done
for SPIN in 1 0; do
  FAASBAL_WAIT_SPIN=$SPIN timeout -k 10 200 python -u tools/hostobs_probe.py 2>&1 | tail -1 | sed "s/^/spin=$SPIN /" || exit 2
done
