#!/bin/bash
# Interleaved knob A/B on bench.py (GPU box): tools/ab_knobs.sh "9=1" "9=2" ...
# each argument is an MXSOLVE_KNOBS setting ("" = defaults); two rounds.
mkdir -p gpurun_out/ab
for round in 1 2; do
  for k in "$@"; do
    tag=$(echo "k$k" | tr '=+' '__')
    MXSOLVE_KNOBS=$k timeout -k 10 120 python bench.py --no-cpu --no-solve --no-asm --no-general --no-configs --steps 1000 > gpurun_out/ab/$tag.log 2>&1 || exit 1
    tail -n 1 gpurun_out/ab/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$k', d['value'], d['roofline']['avg_launch_ms'], d['spmv_standalone']['avg_ms'], d['cg_fusion_mode'])"
  done
done
