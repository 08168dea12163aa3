# rocprofv3 kernel stats of configs[2] for several library builds: tools/prof_ab.sh A.so B.so ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
i=0
for L in "$@"; do
  i=$((i+1))
  FAASBAL_LIB=$R/$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pab$i -o run -- python3 $R/bench.py --steps 400 --warmup 20 --no-cpu-baseline --no-host-observed > $R/gpurun_out/pab$i.json 2> $R/gpurun_out/pab$i.err || exit 1
  echo "== $(basename $L): $(python3 -c "import json; d=json.load(open('$R/gpurun_out/pab$i.json')); print('us/tick %.2f' % (d['ms_per_step']*1e3))")"
  find $R/gpurun_out/pab$i -name "*kernel_stats.csv" -exec cut -d, -f1-4 {} \; | head -4
done
