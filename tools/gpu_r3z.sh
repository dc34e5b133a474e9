# round 3 (session 2): plane-pipelined 27-point z-march
cd /root/repo
(while true; do date > gpurun_out/hb; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -s -k "poisson3d27 or 27 or c5_share or c5_p8" --timeout 600 --timeout-method thread > gpurun_out/r3z_tests.log 2>&1 || { tail -40 gpurun_out/r3z_tests.log; exit 1; }
tail -2 gpurun_out/r3z_tests.log
timeout -k 10 400 python3 -u tools/cg_ab.py poisson3d27 512,512,64 3 "60=1" "60=0" "60=1+56=6" "60=1+56=7" "60=1+45=7" "60=1+45=7+56=7" > gpurun_out/r3z_ab.log 2>&1 || { tail -20 gpurun_out/r3z_ab.log; exit 1; }
cat gpurun_out/r3z_ab.log
timeout -k 10 200 python3 -u tools/mult_ab.py poisson3d27 512x512x64 5 "60=0" "45=7" > gpurun_out/r3z_mult.log 2>&1 || { tail -20 gpurun_out/r3z_mult.log; exit 1; }
cat gpurun_out/r3z_mult.log
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r3z_c5 -o run -f csv -- python3 tools/c5_trace.py 100 "60=1" "55=0" > gpurun_out/r3z_c5.log 2>&1 || { tail -20 gpurun_out/r3z_c5.log; exit 1; }
echo all done
