#!/bin/bash
# Sharded tests on the in-tree library, then tools/shard_probe.py for the ab/ variants
# alternated twice:  bash tools/r04_s.sh TAG V1 V2 ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "shard or full_size" \
    > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for rep in 1 2; do
  for V in "$@"; do
    echo "== $V"; FAASBAL_LIB=$R/distributed-faas_amd/faasbal/ab/libfaasbal_$V.so timeout -k 10 200 python -u tools/shard_probe.py 2>&1 | grep -v amdgpu.ids || exit 3
  done
done
