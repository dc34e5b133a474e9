#!/bin/bash
# Kernel traces of bench.py's CG under several knob settings (one rocprofv3
# run each):  tools/trace_ab.sh "39=0" "40=4" ...   -> gpurun_out/tab/<tag>/
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
for k in "$@"; do
  tag=$(echo "k$k" | tr '=+' '__')
  mkdir -p $R/gpurun_out/tab/$tag
  (cd /tmp && MXSOLVE_KNOBS=$k timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d $R/gpurun_out/tab/$tag -o run -- python3 $R/bench.py --steps 200 --warmup 5 --no-cpu --no-solve > $R/gpurun_out/tab/$tag.log 2>&1)
  echo "== $k $(grep '^{' $R/gpurun_out/tab/$tag.log | tail -n 1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["avg_launch_ms"])')"
  python3 $R/tools/trace_medians.py $R/gpurun_out/tab/$tag > $R/gpurun_out/tab/$tag.med
  sed -n 1,6p $R/gpurun_out/tab/$tag.med
done
