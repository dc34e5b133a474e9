#!/bin/bash
# GPU-box profiling recipe (run from the repo root under gpurun).
# 1) kernel trace + stats of a short bench; 2) FETCH_SIZE and 3) WRITE_SIZE in
# separate --pmc passes (never combined with runtime/sys tracing); 4) the
# FETCH_SIZE calibration stream (known bytes at 8 and 16 B per lane).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
ARGS="--steps ${STEPS:-50} --warmup 5 --no-cpu --no-solve --no-asm --no-configs --grid ${GRID:-256}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 $R/bench.py $ARGS > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv --kernel-include-regex 'spmv|cg_|fold|stream_read' -d $OUT/fetch -o run -- python3 $R/bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv --kernel-include-regex 'spmv|cg_|fold|stream_read' -d $OUT/write -o run -- python3 $R/bench.py $ARGS > $OUT/write.log 2>&1
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -f csv --kernel-include-regex stream_read -d $OUT/calib -o run -- python3 $R/tools/calib_stream.py > $OUT/calib.log 2>&1
