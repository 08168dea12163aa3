# rocprofv3 kernel stats of the configs[4] stream bench: tools/prof_stream.sh TAG [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
T=$1; shift
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$T -o run -- python3 $R/bench.py --workload stream --steps 20 --warmup 3 "$@" > $R/gpurun_out/$T.json 2> $R/gpurun_out/$T.err || { tail -20 $R/gpurun_out/$T.err; exit 1; }
python3 -c "import json; d=json.load(open('$R/gpurun_out/$T.json')); print('$T ms/tick %.3f' % d['ms_per_step'], {k: round(v,1) for k,v in d['tick']['kernels_us_per_tick'].items()})"
find $R/gpurun_out/$T -name "*kernel_stats.csv" -exec cut -d, -f1-5 {} \; | head -30
