#!/bin/bash
# Kernel-trace medians of the standalone MatMult for several library builds:
#   tools/ab_spmv_trace.sh TAG lib1.so lib2.so ...   (SPMV_DIMS, SPMV_KIND env)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
for L in "$@"; do
  for rep in 1 2; do
    (cd /tmp && MXSOLVE_LIB=$R/$L timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d $R/gpurun_out/trab_${TAG}/$(basename $L .so)_$rep -o run -- python3 $R/tools/spmv_only.py ${SPMV_KIND:-poisson3d} ${SPMV_DIMS:-256} 50 > /dev/null 2>&1)
  done
done
