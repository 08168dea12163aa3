#!/bin/bash
# Host-side split of the streaming tick (tools/stream_probe.py, pinned messages) with
# fb_tick_stage's own time split (FAASBAL_STAGE_PROF=1), and the stream bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=${1:-sh}
FAASBAL_STAGE_PROF=1 timeout -k 10 300 python -u tools/stream_probe.py --pinned > gpurun_out/${TAG}_probe.log 2>&1 || { tail -20 gpurun_out/${TAG}_probe.log; exit 1; }
tail -4 gpurun_out/${TAG}_probe.log
for th in 1 4 16; do
  FAASBAL_STAGE_THREADS=$th FAASBAL_STAGE_PROF=1 timeout -k 10 300 python -u tools/stream_probe.py --pinned > gpurun_out/${TAG}_probe_t$th.log 2>&1 || exit 2
  echo "threads $th"; tail -2 gpurun_out/${TAG}_probe_t$th.log
done
