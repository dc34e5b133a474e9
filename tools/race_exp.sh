#!/bin/bash
# Read-before-write / assembly-race experiments.  Each
# step: name, env knobs, command.  A step whose log shows a GPU fault, an
# abort or a time limit ends the script (nothing more runs on the GPU).
#   bash tools/race_exp.sh STEP...   (steps are the case names below)
R=$(pwd)
mkdir -p gpurun_out/race
run() {   # tag knobs cmd...
  local tag=$1 knobs=$2; shift 2
  echo "== $tag knobs=$knobs $(date +%T)"
  MXSOLVE_KNOBS=$knobs timeout -k 10 300 "$@" > gpurun_out/race/$tag.log 2>&1
  local rc=$?
  echo "   rc=$rc"; grep -E "passed|failed|bad|DIFF|illegal|Error" gpurun_out/race/$tag.log | tail -5
  if [ $rc -ge 2 ] || grep -q "illegal memory access\|Memory access fault\|core dumped" gpurun_out/race/$tag.log; then
    echo "   stop: fault, abort or time limit"; exit 1
  fi
}
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
for step in "$@"; do
  case $step in
    cg_poison_nocontig) run $step "81=2+82=1024+18=0" $PYT tests/test_gpu_cgfuse.py -k "one_rank or ranks" ;;
    cg_poison)          run $step "81=2+82=1024" $PYT tests/test_gpu_cgfuse.py -k "one_rank or ranks" ;;
    cg_cache_nopoison)  run $step "81=1+82=1024" $PYT tests/test_gpu_cgfuse.py -k "one_rank or ranks" ;;
    cg_poison_ranks)    run $step "81=2+82=1024" $PYT tests/test_gpu_cgfuse.py -k "ranks" ;;
    asm_nosync)         DIAG_SOLVE=1 run $step "83=0" python -u tools/asm_race.py convdiff3d 128 40 ;;
    asm_nosync_nocontig) DIAG_SOLVE=1 run $step "83=0+18=0" python -u tools/asm_race.py convdiff3d 128 40 ;;
    asm_nosync_nosdma)  HSA_ENABLE_SDMA=0 DIAG_SOLVE=1 run $step "83=0" python -u tools/asm_race.py convdiff3d 128 40 ;;
    alias_contig)       run $step "" ./tools/contig_alias 8 150 1 1024 81920 ;;
    alias_contig_small) run $step "" ./tools/contig_alias 8 200 1 1024 16384 ;;
    x_probe_contig)     run $step "81=1+82=1024" python -u tools/contig_x_probe.py 2 ;;
    x_probe_nocontig)   run $step "81=1+82=1024+18=0" python -u tools/contig_x_probe.py 2 ;;
    alias_contig_nt)    run $step "" ./tools/contig_alias 8 200 1 1024 16384 1 ;;
    alias_plain)        run $step "" ./tools/contig_alias 8 150 0 1024 81920 ;;
    alias_contig_1t)    run $step "" ./tools/contig_alias 1 300 1 1024 81920 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== all steps done"
