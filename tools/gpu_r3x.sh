# round 3 (session 2): symmetric 5/7-point p.Ap pass
cd /root/repo
(while true; do date > gpurun_out/hb; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v -s -k "mode5_nonsym or c3_full or c2_full" --timeout 600 --timeout-method thread > gpurun_out/r3x_tests.log 2>&1 || { tail -40 gpurun_out/r3x_tests.log; exit 1; }
tail -2 gpurun_out/r3x_tests.log
timeout -k 10 300 python3 -u tools/cg_ab.py poisson3d 256,256,256 5 "59=1" "59=0" > gpurun_out/r3x_ab.log 2>&1 || { tail -20 gpurun_out/r3x_ab.log; exit 1; }
timeout -k 10 300 python3 -u tools/cg_ab.py poisson2d 4096,4096,1 3 "59=1" "59=0" >> gpurun_out/r3x_ab.log 2>&1 || { tail -20 gpurun_out/r3x_ab.log; exit 1; }
cat gpurun_out/r3x_ab.log
echo all done
