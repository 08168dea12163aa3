#!/bin/bash
# slab window ticks: the window / full-size tests, then the stream bench line
mkdir -p gpurun_out
T=${1:-f}
timeout -k 10 700 python -u -m pytest tests/test_gpu_window.py tests/test_full_size.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
timeout -k 10 300 python -u bench.py --workload stream --no-cpu-baseline > gpurun_out/${T}_stream.json 2> gpurun_out/${T}_stream.err || { tail -20 gpurun_out/${T}_stream.err; exit 3; }
cat gpurun_out/${T}_stream.json
