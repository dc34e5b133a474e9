# round 3: final bench lines (driver's K = 20 with the CPU leg, K = 500) and the rocprof profile
cd /root/repo
(while true; do date > gpurun_out/hb; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r3k_bench20.json 2> gpurun_out/r3k_bench20.err || { tail -20 gpurun_out/r3k_bench20.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r3k_bench20.json').read().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['cg_iter_frac'],d['converged_its_per_s'])"
timeout -k 10 300 python3 bench.py --steps 500 --warmup 50 --no-cpu --no-asm > gpurun_out/r3k_bench500.json 2> gpurun_out/r3k_bench500.err || { tail -20 gpurun_out/r3k_bench500.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r3k_bench500.json').read().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['cg_iter_frac'],d['converged_its_per_s'])"
STEPS=50 timeout -k 10 900 bash tools/profile.sh || { echo profile failed; exit 1; }
echo all done
