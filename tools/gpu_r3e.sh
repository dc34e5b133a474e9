# round 3: multi-rank mode 5 parity, the P = 8 interior-rank proxy A/B + trace
cd /root/repo
(while true; do date > gpurun_out/hb; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multirank.py::test_distributed_mode5 "tests/test_gpu_cgfuse.py::test_mode5_recomputed_product" > gpurun_out/r3e_unit.log 2>&1 || { tail -40 gpurun_out/r3e_unit.log; exit 1; }
tail -2 gpurun_out/r3e_unit.log
timeout -k 10 400 python -u tools/rank_proxy.py 3 200 9=1 9=2 9=5 > gpurun_out/r3e_proxy.log 2>&1 || { tail -30 gpurun_out/r3e_proxy.log; exit 1; }
grep '^{' gpurun_out/r3e_proxy.log
export TMPDIR=/tmp
mkdir -p gpurun_out/proxytrace
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/proxytrace -o run -- python3 tools/rank_proxy.py 1 100 9=1 9=2 9=5 > gpurun_out/r3e_proxytrace.log 2>&1 || { tail -30 gpurun_out/r3e_proxytrace.log; exit 1; }
head -2 gpurun_out/proxytrace/run_kernel_trace.csv

timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/r3e_bench20.json 2> gpurun_out/r3e_bench20.err || { tail -20 gpurun_out/r3e_bench20.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r3e_bench20.json').read().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac'],json.dumps(d['assembly_host_csr']))"
timeout -k 10 400 python3 tools/bench_general.py asm > gpurun_out/r3e_asm.log 2>&1 || { tail -20 gpurun_out/r3e_asm.log; exit 1; }
grep '^{' gpurun_out/r3e_asm.log
for c in c2 c4 c5share; do
  timeout -k 10 200 python3 bench.py --cpu-config $c >> gpurun_out/r3e_cpucfg.log 2>&1 || { tail -20 gpurun_out/r3e_cpucfg.log; exit 1; }
done
grep '^{' gpurun_out/r3e_cpucfg.log
echo all done
