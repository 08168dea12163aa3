#!/bin/bash
# GPU box: per-process k_emit2 time vs UTCL1 translation counters on the stream bench, 4 processes.
# tools/tlb_probe.sh  -> gpurun_out/tlb_<i>/ (+ summary on stdout)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for i in $(seq 1 ${NPROC:-4}); do
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc ${PMC:-TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_REQUEST_sum} --output-format csv -d $R/gpurun_out/tlb_$i -o run -- \
      python3 $R/bench.py --workload stream --steps 20 --warmup 3 > $R/gpurun_out/tlb_$i.json 2> $R/gpurun_out/tlb_$i.err || { tail -5 $R/gpurun_out/tlb_$i.err; exit 1; }
  python3 $R/tools/pmc_kernels.py $R/gpurun_out/tlb_$i || exit 2
done
