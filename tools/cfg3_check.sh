#!/bin/bash
# One-GPU configs[3] path (k_plan2 / k_logscan / k_emit2 after k_plan2): the plan-path and
# full-size parity tests, then the configs[3] bench line twice.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
T=${1:-c3}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -k "plan or config3 or logscan or fill_levels" \
    "tests/test_full_size.py" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 \
    || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --workload cfg3 --no-cpu-baseline --no-host-observed > gpurun_out/${T}_cfg3_$i.json 2> gpurun_out/${T}_cfg3_$i.err || { tail -20 gpurun_out/${T}_cfg3_$i.err; exit 3; }
  python -c "import json; d=json.load(open('gpurun_out/${T}_cfg3_$i.json')); print(round(d['ms_per_step']*1e3,2), 'us/tick', {k: round(v*1e3,2) for k,v in d['tick']['kernels_avg_ms'].items()}, round(d['roofline']['tick_frac'],3))"
done
