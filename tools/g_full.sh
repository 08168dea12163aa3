#!/bin/bash
# GPU box: full GPU suite, smoke, default bench, then N stream-bench processes.  tools/g_full.sh TAG [N]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
T=$1; N=${2:-2}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { grep -E "FAIL|Error|error" gpurun_out/${T}_pytest.log | head -20; tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 2; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 3; }
python3 -c "import json; d=json.load(open('gpurun_out/${T}_bench.json')); print('c2 us/tick %.2f' % (d['ms_per_step']*1e3), 'frac %.3f' % d['roofline']['frac'], 'host_obs %.2f G/s' % (d['host_observed']['value']/1e9))"
for i in $(seq 1 $N); do
  timeout -k 10 150 python -u bench.py --workload stream --steps 30 --warmup 3 > gpurun_out/${T}_stream$i.json 2> gpurun_out/${T}_stream$i.err || { tail -5 gpurun_out/${T}_stream$i.err; exit 4; }
  python3 -c "import json; d=json.load(open('gpurun_out/${T}_stream$i.json')); print('stream us/tick %.1f' % (d['ms_per_step']*1e3), 'dev %.1f' % d['tick']['device_us_per_tick'], {k: round(v,1) for k,v in d['tick']['kernels_us_per_tick'].items()})"
done
