# round 3: SQ counters of the 27-point and 7-point z-march MatMults in CG (where the waves spend their cycles)
cd /root/repo
(while true; do date > gpurun_out/hb; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
export TMPDIR=/tmp
mkdir -p gpurun_out/sq27 gpurun_out/sq7
C="SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex zm27 -f csv -d gpurun_out/sq27 -o run -- python3 tools/knob_runs.py poisson3d27 512,512,64 30 45=6 > gpurun_out/r3h_sq27.log 2>&1 || { tail -20 gpurun_out/r3h_sq27.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "spmv_pair_zm_kernel" -f csv -d gpurun_out/sq7 -o run -- python3 tools/knob_runs.py poisson3d 256,256,256 30 9=2 > gpurun_out/r3h_sq7.log 2>&1 || { tail -20 gpurun_out/r3h_sq7.log; exit 1; }
for d in sq27 sq7; do python3 - gpurun_out/$d/run_counter_collection.csv <<'PY'
import csv, sys, statistics, collections
d = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    d[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in d.items():
    print(k, {c: round(statistics.median(v)) for c, v in sorted(cs.items())})
PY
done
echo all done
