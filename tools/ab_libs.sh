#!/bin/bash
# A/B of kernel variant libraries (distributed-faas_amd/faasbal/ab/libfaasbal_<V>.so) on
# the stream bench, alternated twice: tools/ab_libs.sh TAG V1 V2 ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=$1; shift
for rep in 1 2; do
  for V in "$@"; do
    FAASBAL_LIB=$R/distributed-faas_amd/faasbal/ab/libfaasbal_$V.so timeout -k 10 200 python -u bench.py --workload stream \
        --no-cpu-baseline --no-pcie-pass --steps 30 > gpurun_out/${TAG}_$V$rep.json 2> gpurun_out/${TAG}_$V$rep.err || { tail -5 gpurun_out/${TAG}_$V$rep.err; exit 1; }
    python3 - gpurun_out/${TAG}_$V$rep.json $V <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["tick"]["kernels_us_per_tick"]
print("%s: %.1f us/tick, device %.1f:" % (sys.argv[2], d["ms_per_step"] * 1e3, d["tick"]["device_us_per_tick"]),
      " ".join("%s %.1f" % (n, v) for n, v in k.items()), flush=True)
PY
  done
done
