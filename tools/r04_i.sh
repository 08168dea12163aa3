#!/bin/bash
# Folded-commit A/B: GPU tests touching the fold on the in-tree library, then
# tools/commit_probe.py per ab/ variant, alternated 3x:  bash tools/r04_i.sh TAG V1 V2 ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "fold or config2 or golden_replay or stream or full_size" > gpurun_out/${TAG}_pytest.log 2>&1 \
    || { tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for rep in 1 2 3; do
  for V in "$@"; do
    FAASBAL_LIB=$R/distributed-faas_amd/faasbal/ab/libfaasbal_$V.so timeout -k 10 120 python -u tools/commit_probe.py \
        2> gpurun_out/${TAG}_$V.err || { tail -5 gpurun_out/${TAG}_$V.err; exit 2; }
  done
done
