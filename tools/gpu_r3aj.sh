# round 3 (session 2, end of round): full suite, smoke, bench lines (driver K = 20 and K = 500), rocprof profile, configurations
cd /root/repo
(while true; do date > gpurun_out/hb; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread --durations=15 > gpurun_out/r3aj_suite.log 2>&1 || { tail -40 gpurun_out/r3aj_suite.log; exit 1; }
tail -2 gpurun_out/r3aj_suite.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3aj_smoke.log 2>&1 || { tail -20 gpurun_out/r3aj_smoke.log; exit 1; }
tail -1 gpurun_out/r3aj_smoke.log
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r3aj_bench20.json 2> gpurun_out/r3aj_bench20.err || { tail -20 gpurun_out/r3aj_bench20.err; exit 1; }
timeout -k 10 400 python3 bench.py > gpurun_out/r3aj_bench500.json 2> gpurun_out/r3aj_bench500.err || { tail -20 gpurun_out/r3aj_bench500.err; exit 1; }
for f in r3aj_bench20 r3aj_bench500; do python3 -c "import json;d=json.loads(open('gpurun_out/$f.json').read().splitlines()[-1]);print('$f', d['value'],d['ms_per_step'],d['roofline']['frac'],d['cg_iter_frac'],d['converged_its_per_s'])"; done
bash tools/profile.sh > gpurun_out/r3aj_prof.log 2>&1 || { tail -20 gpurun_out/r3aj_prof.log; exit 1; }
timeout -k 10 600 python3 tools/bench_configs.py > gpurun_out/r3aj_configs.log 2>&1 || { tail -20 gpurun_out/r3aj_configs.log; exit 1; }
grep '^{' gpurun_out/r3aj_configs.log
echo all done
