#!/bin/bash
# One-GPU parity (parity + deque + window suites) on the in-tree library, then the
# configs[2] A/B of ab/ variants (tools/ab.sh, alternated 3x):  bash tools/r04_z.sh TAG V1 V2
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_deque.py tests/test_gpu_window.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
L=""; for V in "$@"; do L="$L distributed-faas_amd/faasbal/ab/libfaasbal_$V.so"; done
bash tools/ab.sh $L
