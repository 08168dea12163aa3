#!/bin/bash
# Same-box A/B of two library builds: tools/ab_lib.sh <old.so> [world...]
# configs[2] bench, the 16M x 1M bench and the sharded per-rank probe, alternated.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
OLD=$1; shift
NEW=$R/distributed-faas_amd/faasbal/libfaasbal.so
for rep in 1 2; do
  for L in $OLD $NEW; do
    FAASBAL_LIB=$L timeout -k 10 120 python -u tools/host_rate_probe.py --world ${@:-2 8} 2>/dev/null | grep world | sed "s|^|$(basename $L) |" || exit 3
  done
done
bash tools/ab_big.sh "--steps 400" FAASBAL_LIB=$OLD FAASBAL_LIB=$NEW || exit 4
bash tools/ab_big.sh "--workers 1048576 --tasks 16000000 --steps 100" FAASBAL_LIB=$OLD FAASBAL_LIB=$NEW || exit 5
