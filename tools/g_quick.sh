#!/bin/bash
# GPU box: selected GPU tests (-k expression), then the stream bench under rocprofv3 kernel stats.
# tools/g_quick.sh TAG "<pytest -k expr>" [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
T=$1; K=$2; shift 2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "$K" --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { grep -E "FAIL|Error|error" gpurun_out/${T}_pytest.log | head -20; tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
bash tools/prof_stream.sh ${T}_stream "$@"
