# GPU box: quick parity (heartbeat + deque + full-size configs[2]) then stamps and A/B vs an old build
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_deque.py "tests/test_full_size.py::test_gpu_cfg2_full_matches_reference" -x -q --timeout 120 --timeout-method thread > gpurun_out/p.log 2>&1 || { tail -30 gpurun_out/p.log; exit 1; }
tail -1 gpurun_out/p.log
timeout -k 10 120 python -u tools/stamps.py > gpurun_out/st.txt 2>&1 || exit 2
cat gpurun_out/st.txt
[ -n "$1" ] && bash tools/ab2.sh $1 distributed-faas_amd/faasbal/libfaasbal.so
