# GPU box: full GPU suite, smoke, default bench, --gpus 2 over gloo on one GPU
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
T=${1:-g5}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { grep -E "FAIL|Error|error" gpurun_out/${T}_pytest.log | head -20; tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 2; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 3; }
cat gpurun_out/${T}_bench.json
timeout -k 10 300 python -u bench.py --gpus 2 --backend gloo --steps 50 --warmup 5 > gpurun_out/${T}_bench2.json 2> gpurun_out/${T}_bench2.err || { tail -20 gpurun_out/${T}_bench2.err; exit 4; }
cat gpurun_out/${T}_bench2.json
