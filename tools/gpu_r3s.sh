# round 3 (session 2): full GPU suite, default bench line, rocprof profile
cd /root/repo
(while true; do date > gpurun_out/hb; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r3s_suite.log 2>&1 || { tail -40 gpurun_out/r3s_suite.log; exit 1; }
tail -2 gpurun_out/r3s_suite.log
timeout -k 10 400 python3 bench.py > gpurun_out/r3s_bench.json 2> gpurun_out/r3s_bench.err || { tail -20 gpurun_out/r3s_bench.err; exit 1; }
tail -1 gpurun_out/r3s_bench.json | cut -c1-600
timeout -k 10 300 python3 bench.py --steps 500 --warmup 50 --no-cpu --no-asm > gpurun_out/r3s_bench500.json 2> gpurun_out/r3s_bench500.err || { tail -20 gpurun_out/r3s_bench500.err; exit 1; }
bash tools/profile.sh > gpurun_out/r3s_prof.log 2>&1 || { tail -20 gpurun_out/r3s_prof.log; exit 1; }
echo all done
