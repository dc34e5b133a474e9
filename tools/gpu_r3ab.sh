# round 3 (session 2): GMRES step / back substitution staged in LDS
cd /root/repo
(while true; do date > gpurun_out/hb; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q -k "gmres or c4_full or convdiff or eigen or lu" --timeout 600 --timeout-method thread > gpurun_out/r3ab_tests.log 2>&1 || { tail -40 gpurun_out/r3ab_tests.log; exit 1; }
tail -2 gpurun_out/r3ab_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3ab_c4 -o run -f csv -- python3 tools/bench_general.py c4 > gpurun_out/r3ab_c4.log 2>&1 || { tail -20 gpurun_out/r3ab_c4.log; exit 1; }
grep '^{' gpurun_out/r3ab_c4.log
timeout -k 10 300 python3 -u tools/bench_configs.py > gpurun_out/r3ab_configs.log 2>&1 || { tail -20 gpurun_out/r3ab_configs.log; exit 1; }
grep '^{' gpurun_out/r3ab_configs.log
echo all done
