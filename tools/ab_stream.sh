#!/bin/bash
# Same-box A/B of two library builds on the streaming tick: tools/ab_stream.sh <old.so>
# (event parity tests with the in-tree build first)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
OLD=$1
NEW=$R/distributed-faas_amd/faasbal/libfaasbal.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/abs_pytest.log 2>&1 || { tail -40 gpurun_out/abs_pytest.log; exit 11; }
tail -1 gpurun_out/abs_pytest.log
for rep in 1 2; do
  for L in $OLD $NEW; do
    FAASBAL_LIB=$L timeout -k 10 120 python -u bench.py --workload stream > gpurun_out/abs.json 2>gpurun_out/abs.err || { tail gpurun_out/abs.err; exit 12; }
    python -c "import json;d=json.load(open('gpurun_out/abs.json'));print('$(basename $L)', round(d['ms_per_step']*1e3,1), 'us/tick', round(d['value']/1e6,1), 'M/s', {k:round(v,1) for k,v in d['tick']['kernels_us_per_tick'].items()})"
  done
done
