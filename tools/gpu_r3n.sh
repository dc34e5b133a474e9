# round 3 (session 2): chunk MDot/MAXPY, 27-point fma form -- tests, A/B, traces
cd /root/repo
(while true; do date > gpurun_out/hb; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -s -k "pair_lean_kernel or pair_code or gmres or c4_full or c5_share or jacobi_by_code or mdot or maxpy" --timeout 600 --timeout-method thread > gpurun_out/r3n_tests.log 2>&1 || { tail -40 gpurun_out/r3n_tests.log; exit 1; }
tail -3 gpurun_out/r3n_tests.log
timeout -k 10 300 python3 -u tools/gmres_ab.py 256 3 "50=2" "50=1" "50=0" "51=0" > gpurun_out/r3n_ab.log 2>&1 || { tail -20 gpurun_out/r3n_ab.log; exit 1; }
cat gpurun_out/r3n_ab.log
timeout -k 10 300 python3 -u tools/op_ab.py poisson3d27 512x512x64 3 "53=1" "53=0" > gpurun_out/r3n_ab27.log 2>&1 || { tail -20 gpurun_out/r3n_ab27.log; exit 1; }
cat gpurun_out/r3n_ab27.log
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r3n_tr -o run -f csv -- python3 tools/gmres_trace.py 256 60 > gpurun_out/r3n_tr.log 2>&1 || { tail -20 gpurun_out/r3n_tr.log; exit 1; }
timeout -k 10 300 python3 -u tools/bench_general.py c4 > gpurun_out/r3n_c4.log 2>&1 || { tail -20 gpurun_out/r3n_c4.log; exit 1; }
grep '^{' gpurun_out/r3n_c4.log
echo all done
