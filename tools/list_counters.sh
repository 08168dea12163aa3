#!/bin/bash
# GPU box: the PMC counters rocprofv3 offers on this GPU (names only) -> gpurun_out/counters.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --list-avail > $R/gpurun_out/counters_raw.txt 2>&1 || true
grep -o -E "\b[A-Z][A-Z0-9_]+(\[[0-9:]+\])?" $R/gpurun_out/counters_raw.txt | sort -u > $R/gpurun_out/counters.txt
grep -i -E "UTCL|TLB|TRANS|PAGE" $R/gpurun_out/counters.txt | head -40
