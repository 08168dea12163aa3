#!/bin/bash
# GPU suite on the current library, then a same-box A/B of the stream line between the
# variant libraries named on the command line: bash tools/r04_g.sh TAG V1 V2 ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
[ $# -gt 0 ] && bash tools/ab_libs.sh ${TAG}_ab "$@"
