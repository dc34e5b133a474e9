#!/bin/bash
# One parameterised GPU-box runner (replaces round 3's one-off gpu_r3*.sh).
#
#   gpurun --timeout S -- bash tools/gpu_run.sh TAG STEP [STEP ...]
#
# Each STEP runs under its own time limit, writes gpurun_out/TAG_STEP.log (or
# .json), and appends the exact command to gpurun_out/TAG_commands.txt so every
# summary copied into profiles/ can name the command that produced it.  The
# first failing step ends the run (no GPU step after a failure).
#
# Steps:
#   suite            the whole GPU test suite (as the driver runs it)
#   tests:EXPR       pytest -m gpu -k EXPR
#   smoke            __graft_entry__.smoke()
#   bench20          bench.py --steps 20 --warmup 5 (the driver's K/W class)
#   bench            bench.py with its defaults (K = 500)
#   benchfast        bench.py --steps 100 --no-cpu --no-asm --no-general
#   shm2             N = 2 rehearsal on one GPU (MXSOLVE_TRANSPORT=shm, torchrun)
#   shm2fail         the same with the mode2/graph leg failing (the line must still print)
#   shm2stall        the same with rank 1 stalling 40 s in the mode2/eager leg under an 8-s leg
#                    budget (BUDGET): the watchdog aborts the leg, the line still prints
#   prof             tools/profile.sh (trace + FETCH/WRITE PMC passes + calibration)
#   configs          tools/bench_configs.py (C2/C3/C4/C5-share converged solves)
#   general:LEGS     tools/bench_general.py LEGS (comma separated)
#   c4prof           rocprofv3 kernel trace of bench_general.py c4 + gmres_roofline.py
#   py:SCRIPT[:ARGS] python3 SCRIPT ARGS (ARGS separated by @)
#   trace:SCRIPT[:ARGS] rocprofv3 kernel trace of python3 SCRIPT ARGS + trace_medians.py
#   bin:PATH[:ARGS]  a prebuilt probe binary (e.g. tools/mdot_probe)
#   pmc:REGEX:SCRIPT[:ARGS] tools/pmc_kernels.sh (one rocprofv3 --pmc pass per counter
#                    group) over python3 SCRIPT ARGS for kernels matching REGEX, then pmc_table.py
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
(while true; do date > $O/hb; sleep 30; done) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT

NSTEP=0
run() {   # run NAME SECONDS CMD... ; output to $O/TAG_NAME.log (TAG_NAME_<n>.log when NAME repeats)
  local name=$1 secs=$2; shift 2
  NSTEP=$((NSTEP + 1))
  local log=$O/${TAG}_${name}.log
  [ -e "$log" ] && log=$O/${TAG}_${name}_${NSTEP}.log
  echo "[$(date +%T)] $name: $*" | tee -a $O/${TAG}_commands.txt
  timeout -k 10 "$secs" "$@" > "$log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then
    echo "step $name failed rc=$rc"; tail -40 "$log"; exit $rc
  fi
  tail -3 "$log"
}

for step in "$@"; do
  case $step in
    suite) run suite 1100 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread --durations=20 ;;
    tests:*) run "tests_${step#tests:}" 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${step#tests:}" ;;
    smoke) run smoke 400 python3 -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench20) run bench20 500 python3 -u bench.py --steps 20 --warmup 5 ;;
    bench) run bench 500 python3 -u bench.py ;;
    benchfast) run benchfast 300 python3 -u bench.py --steps 100 --no-cpu --no-asm --no-general ;;
    shm2) MXSOLVE_TRANSPORT=shm run shm2 400 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
            --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 50 --warmup 5 ;;
    shm2fail) MXSOLVE_TRANSPORT=shm MXSOLVE_BENCH_FAIL_LEG=mode2/graph run shm2fail 400 python3 -u -m torch.distributed.run \
                --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 50 --warmup 5 ;;
    shm2stall) MXSOLVE_TRANSPORT=shm MXSOLVE_BENCH_LEG_BUDGET_S=${BUDGET:-8} MXSOLVE_BENCH_STALL_LEG=mode2/eager:40 \
                 run shm2stall 400 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
                 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 2 --steps 50 --warmup 5 ;;
    prof) run prof 1000 bash tools/profile.sh ;;
    configs) run configs 700 python3 -u tools/bench_configs.py ;;
    c4prof) run c4prof 600 rocprofv3 --kernel-trace --stats -f csv -d $O/${TAG}_c4trace -o run -- \
              python3 -u tools/bench_general.py c4
            run c4roof 120 python3 tools/gmres_roofline.py $O/${TAG}_c4trace 530 ;;
    general:*) run general 700 python3 -u tools/bench_general.py $(echo "${step#general:}" | tr , ' ') ;;
    py:*) s=${step#py:}; scr=${s%%:*}; a=""; [ "$s" != "$scr" ] && a=$(echo "${s#*:}" | tr @ ' ')
          run "py_$(basename "$scr" .py)" 900 python3 -u "$scr" $a ;;
    trace:*) s=${step#trace:}; scr=${s%%:*}; a=""; [ "$s" != "$scr" ] && a=$(echo "${s#*:}" | tr @ ' ')
             nm=$(basename "$scr" .py)
             run "trace_$nm" 600 rocprofv3 --kernel-trace --stats -f csv -d $O/${TAG}_trace_$nm -o run -- python3 -u "$scr" $a
             run "med_$nm" 120 python3 tools/trace_medians.py $O/${TAG}_trace_$nm ;;
    bin:*) s=${step#bin:}; b=${s%%:*}; a=""; [ "$s" != "$b" ] && a=$(echo "${s#*:}" | tr @ ' ')
           run "bin_$(basename "$b")" 300 "$b" $a ;;
    pmc:*) s=${step#pmc:}; rx=${s%%:*}; s=${s#*:}; scr=${s%%:*}; a=""; [ "$s" != "$scr" ] && a=$(echo "${s#*:}" | tr @ ' ')
           TAG=${TAG}_pmc REGEX="$rx" run "pmc_$(basename "$scr" .py)" 900 bash tools/pmc_kernels.sh python3 "$R/$scr" $a
           run "pmctab_$(basename "$scr" .py)" 120 python3 tools/pmc_table.py $O/pmc_${TAG}_pmc ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "all steps done"
