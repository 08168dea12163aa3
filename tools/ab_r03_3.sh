set -o pipefail
cd $GRAFT_REPO_ROOT
L=distributed-faas_amd/faasbal
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab3_pytest.log 2>&1 || { tail -30 gpurun_out/ab3_pytest.log; exit 11; }
tail -1 gpurun_out/ab3_pytest.log
bash tools/ab_env.sh FAASBAL_F_EMIT=0 FAASBAL_F_EMIT=1 && FAASBAL_F_EMIT=1 bash tools/ab_env.sh FAASBAL_EMIT_CFIRST=0 FAASBAL_EMIT_CFIRST=1
