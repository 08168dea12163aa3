#!/bin/bash
# k_emit2 WRITE_SIZE per dropped output array (tools/write_probe.py), one PMC pass per variant.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for m in 0 1 3 4 8 16 32; do
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/wp_$m -o run -- \
        python3 $R/tools/write_probe.py --run --mask $m > $R/gpurun_out/wp_$m.log 2>&1 || { tail -20 $R/gpurun_out/wp_$m.log; exit 1; }
    tail -1 $R/gpurun_out/wp_$m.log
done
python3 $R/tools/write_probe.py --summary $R/gpurun_out | tee $R/gpurun_out/wp_summary.txt
