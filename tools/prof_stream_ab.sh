# rocprof stream kernel stats for several library builds, alternated twice: tools/prof_stream_ab.sh A.so B.so ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
i=0
for rep in 1 2; do
  for L in "$@"; do
    i=$((i+1))
    FAASBAL_LIB=$R/$L bash tools/prof_stream.sh psab$i > /dev/null || exit 1
    echo "== $L"; python3 tools/pstat.py gpurun_out/psab$i | grep -v "=="
  done
done
