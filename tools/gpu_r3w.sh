# round 3 (session 2): symmetric 27-point p.Ap pass
cd /root/repo
(while true; do date > gpurun_out/hb; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v -s -k "mode5 or c5_share" --timeout 600 --timeout-method thread > gpurun_out/r3w_tests.log 2>&1 || { tail -40 gpurun_out/r3w_tests.log; exit 1; }
tail -2 gpurun_out/r3w_tests.log
timeout -k 10 300 python3 -u tools/cg_ab.py poisson3d27 512,512,64 3 "59=1" "59=0" "55=0" > gpurun_out/r3w_ab.log 2>&1 || { tail -20 gpurun_out/r3w_ab.log; exit 1; }
cat gpurun_out/r3w_ab.log
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r3w_c5 -o run -f csv -- python3 tools/c5_trace.py 100 "59=1" > gpurun_out/r3w_c5.log 2>&1 || { tail -20 gpurun_out/r3w_c5.log; exit 1; }
echo all done
