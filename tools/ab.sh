# A/B/C of library builds on configs[2], alternated: tools/ab3.sh A.so B.so C.so ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for rep in 1 2 3; do
  for L in "$@"; do
    FAASBAL_LIB=$R/$L timeout -k 10 150 python -u bench.py --no-cpu-baseline --no-host-observed --steps 400 $AB_ARGS > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 3; }
    python -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); print('$(basename $L)', 'us/tick %.2f' % (d['ms_per_step']*1e3), {k: round(v*1e3,2) for k,v in d['tick']['kernels_avg_ms'].items()}, 'dom %s frac %.3f' % (d['roofline']['kernel'], d['roofline']['frac']))"
  done
done
