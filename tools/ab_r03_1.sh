set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_env.sh FAASBAL_F_EMIT=0 FAASBAL_F_EMIT=1 && bash tools/ab_env.sh FAASBAL_F_TICKET=0 FAASBAL_F_TICKET=1 && bash tools/ab.sh distributed-faas_amd/faasbal/libfaasbal.so distributed-faas_amd/faasbal/libfaasbal_noxcd.so
