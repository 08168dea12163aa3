set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "event_sort or stream or random or golden" > gpurun_out/sort_pytest.log 2>&1 || { tail -40 gpurun_out/sort_pytest.log; exit 11; }
tail -2 gpurun_out/sort_pytest.log
for i in 1 2; do for w in 0 1; do
  FAASBAL_RS_WIDE=$w timeout -k 10 120 python -u bench.py --workload stream > gpurun_out/sort_ab_${w}_$i.json 2>gpurun_out/sort_ab.err || { tail gpurun_out/sort_ab.err; exit 12; }
  python -c "import json;d=json.load(open('gpurun_out/sort_ab_${w}_$i.json'));print('wide=$w', round(d['ms_per_step']*1e3,1), 'us/tick', round(d['value']/1e6,1), 'M/s', {k:round(v,1) for k,v in d['tick']['kernels_us_per_tick'].items()})"
done; done
