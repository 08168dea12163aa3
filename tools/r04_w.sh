#!/bin/bash
# k_plan-path staged emission: parity on the in-tree library, then configs[3] A/B and
# each variant's trace + FETCH / WRITE passes:  bash tools/r04_w.sh TAG V1 V2
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py tests/test_gpu_deque.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -k "plan or config3 or fill_levels or full_size or cfg" > gpurun_out/${TAG}_pytest.log 2>&1 \
    || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
L=""; for V in "$@"; do L="$L distributed-faas_amd/faasbal/ab/libfaasbal_$V.so"; done
AB_ARGS="--workload cfg3" bash tools/ab.sh $L || exit 2
for V in "$@"; do
  FAASBAL_LIB=$R/distributed-faas_amd/faasbal/ab/libfaasbal_$V.so bash tools_profile.sh ${TAG}_$V --workload cfg3 > gpurun_out/${TAG}_prof_$V.log 2>&1 \
      || { tail -20 gpurun_out/${TAG}_prof_$V.log; exit 3; }
done
echo done
