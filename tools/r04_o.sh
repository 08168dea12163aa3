set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04o_pytest.log 2>&1 || { tail -30 gpurun_out/r04o_pytest.log; exit 1; }
tail -1 gpurun_out/r04o_pytest.log
bash tools/ab.sh distributed-faas_amd/faasbal/ab/libfaasbal_base.so distributed-faas_amd/faasbal/ab/libfaasbal_dpp.so
