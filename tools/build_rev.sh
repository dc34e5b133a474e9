#!/bin/bash
# Build libmxsolve.so of git revision $1 into ab/$2.so (A/B baselines for tools/lib_ab.py)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
WT=/tmp/mx_wt_$2
rm -rf $WT && git -C $R worktree add -f --detach $WT $1 >/dev/null 2>&1
make -s -j8 -C $WT/mpi-petsc4py-example_amd/csrc >/dev/null
mkdir -p $R/ab && cp $WT/mpi-petsc4py-example_amd/lib/libmxsolve.so $R/ab/$2.so
git -C $R worktree remove --force $WT
echo "ab/$2.so"
