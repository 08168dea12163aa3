# stream emit duration per process, default vs contiguous arena, interleaved: tools/emit_modes.sh N
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for i in $(seq 1 ${1:-6}); do
  for C in 0 1; do
    FAASBAL_CONTIG=$C FAASBAL_PRINT_ARENA=1 bash tools/prof_stream.sh em$i$C > /dev/null || exit 1
    echo "run $i contig $C: $(grep -h 'faasbal arena' gpurun_out/em$i$C.err | head -1) $(python3 tools/pstat.py gpurun_out/em$i$C | grep 'emit2<1, true, 3' | cut -c50-)"
  done
done
