mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "shard or dispatch or gateway" > gpurun_out/e_pytest.log 2>&1 || { tail -30 gpurun_out/e_pytest.log; exit 1; }
tail -2 gpurun_out/e_pytest.log
timeout -k 10 200 python -u tools/shard_probe.py --reps 30 > gpurun_out/e_probe.log 2>&1 && timeout -k 10 200 python -u tools/shard_probe.py --reps 30 --scaling weak >> gpurun_out/e_probe.log 2>&1 || exit 2
cat gpurun_out/e_probe.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/e_bench.json 2> gpurun_out/e_bench.err || { tail -20 gpurun_out/e_bench.err; exit 3; }
cat gpurun_out/e_bench.json
