# round 3: final bench lines + the other BASELINE configurations
cd /root/repo
(while true; do date > gpurun_out/hb; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r3l_bench20.json 2> gpurun_out/r3l_bench20.err || { tail -20 gpurun_out/r3l_bench20.err; exit 1; }
timeout -k 10 300 python3 bench.py --steps 500 --warmup 50 --no-cpu --no-asm > gpurun_out/r3l_bench500.json 2> gpurun_out/r3l_bench500.err || { tail -20 gpurun_out/r3l_bench500.err; exit 1; }
for f in r3l_bench20 r3l_bench500; do python3 -c "import json;d=json.loads(open('gpurun_out/$f.json').read().splitlines()[-1]);print('$f', d['value'],d['ms_per_step'],d['roofline']['frac'],d['cg_iter_frac'],d['cg_xbatch'],d['converged_its_per_s'])"; done
timeout -k 10 600 python3 tools/bench_configs.py > gpurun_out/r3l_configs.log 2>&1 || { tail -20 gpurun_out/r3l_configs.log; exit 1; }
grep '^{' gpurun_out/r3l_configs.log
echo all done
