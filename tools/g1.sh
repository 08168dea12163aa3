set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 60 ./tools/chainbench > gpurun_out/g1_chain_wall.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/g1_chain -o run -- $GRAFT_REPO_ROOT/tools/chainbench > $GRAFT_REPO_ROOT/gpurun_out/g1_chain_prof.log 2>&1 || exit 2
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 200 --warmup 20 > gpurun_out/g1_bench.json 2>gpurun_out/g1_bench.err || exit 3
timeout -k 10 120 python -u tools/stamps.py > gpurun_out/g1_stamps.txt 2>&1 || exit 4
cat gpurun_out/g1_chain_wall.log gpurun_out/g1_stamps.txt
