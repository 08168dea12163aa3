# GPU box: parity suite (fast files) + stream bench + rocprof stream stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
T=${1:-g7}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { grep -E "FAIL|Error|error" gpurun_out/${T}_pytest.log | head -20; tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
bash tools/prof_stream.sh ${T}_ps
