# rocprof stream kernel stats under several environment settings, alternated twice:
#   tools/prof_stream_env.sh "VAR=a" "VAR=b" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
i=0
for rep in 1 2; do
  for V in "$@"; do
    i=$((i+1))
    env $V bash tools/prof_stream.sh pse$i > gpurun_out/pse$i.txt || exit 1
    echo "== $V: $(head -1 gpurun_out/pse$i.txt | cut -c1-160)"; python3 tools/pstat.py gpurun_out/pse$i | grep -v "=="
  done
done
