#!/bin/bash
# A/B of kernel variant libraries (distributed-faas_amd/faasbal/ab/libfaasbal_<V>.so) on
# the stream bench (AB_WORKLOAD: another workload), alternated twice: tools/ab_libs.sh TAG V1 V2 ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=$1; shift
for rep in 1 2; do
  for V in "$@"; do
    FAASBAL_LIB=$R/distributed-faas_amd/faasbal/ab/libfaasbal_$V.so timeout -k 10 200 python -u bench.py --workload ${AB_WORKLOAD:-stream} \
        --no-cpu-baseline --no-pcie-pass --no-host-observed --steps ${AB_STEPS:-30} > gpurun_out/${TAG}_$V$rep.json 2> gpurun_out/${TAG}_$V$rep.err || { tail -5 gpurun_out/${TAG}_$V$rep.err; exit 1; }
    python3 - gpurun_out/${TAG}_$V$rep.json $V <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
t = d["tick"]
k = t.get("kernels_us_per_tick") or {n: v * 1e3 for n, v in t.get("kernels_avg_ms", {}).items()}
dev = t.get("device_us_per_tick", t.get("device_ms", 0) * 1e3)
print("%s: %.2f us/tick, device %.2f:" % (sys.argv[2], d["ms_per_step"] * 1e3, dev),
      " ".join("%s %.2f" % (n, v) for n, v in k.items()), flush=True)
PY
  done
done
