# GPU box: parity suite + smoke + bench + stamps (tag $1)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
T=${1:-g}
bash tools/gpu_check.sh $T || exit 1
timeout -k 10 120 python -u tools/stamps.py > gpurun_out/${T}_stamps.txt 2>&1 || exit 2
cat gpurun_out/${T}_stamps.txt
