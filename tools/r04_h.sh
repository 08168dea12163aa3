#!/bin/bash
# GPU suite on the in-tree library, then configs[2] and configs[3] A/B of ab/ variant
# builds (bench alternated 3x):  bash tools/r04_h.sh TAG "C2 variants" "C3 variants"
# (libraries distributed-faas_amd/faasbal/ab/libfaasbal_<V>.so)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=$1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
L=""; for V in $2; do L="$L distributed-faas_amd/faasbal/ab/libfaasbal_$V.so"; done
echo "== configs[2]"; bash tools/ab.sh $L || exit 2
L=""; for V in $3; do L="$L distributed-faas_amd/faasbal/ab/libfaasbal_$V.so"; done
echo "== configs[3]"; AB_ARGS="--workload cfg3" bash tools/ab.sh $L || exit 3
echo done
