# GPU box: large-batch sort parity + stream bench at heartbeat storms (scan vs no-scan library)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "event_sort" --timeout 400 --timeout-method thread > gpurun_out/g6_pytest.log 2>&1 || { tail -30 gpurun_out/g6_pytest.log; exit 1; }
tail -2 gpurun_out/g6_pytest.log
for HB in 0.01 1.0 2.0; do
  for L in libfaasbal.so libfaasbal_noscan.so; do
    FAASBAL_LIB=$R/distributed-faas_amd/faasbal/$L timeout -k 10 300 python -u bench.py --workload stream --hb-frac $HB --steps 20 --warmup 3 > gpurun_out/g6_s.json 2> gpurun_out/g6_s.err || { tail -20 gpurun_out/g6_s.err; exit 3; }
    python -c "import json; d=json.load(open('gpurun_out/g6_s.json')); print('$HB $L', 'ms/tick %.3f' % d['ms_per_step'], 'events %.0f' % d['config']['events_per_tick'], {k: round(v,1) for k,v in d['tick']['kernels_us_per_tick'].items()})"
  done
done
timeout -k 10 60 ./tools/kpbench
