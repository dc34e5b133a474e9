# round 3 (session 2): 27-point mode 5 with the resident residual-update grid
cd /root/repo
(while true; do date > gpurun_out/hb; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v -s -k "mode5 or c5_share or poisson3d27 or north_star or c5_p8" --timeout 600 --timeout-method thread > gpurun_out/r3v_tests.log 2>&1 || { tail -40 gpurun_out/r3v_tests.log; exit 1; }
tail -2 gpurun_out/r3v_tests.log
timeout -k 10 300 python3 -u tools/cg_ab.py poisson3d27 512,512,64 3 "55=0" "55=1" "55=1+56=4" "55=1+56=6" > gpurun_out/r3v_ab.log 2>&1 || { tail -20 gpurun_out/r3v_ab.log; exit 1; }
cat gpurun_out/r3v_ab.log
timeout -k 10 600 python3 tools/bench_configs.py > gpurun_out/r3v_configs.log 2>&1 || { tail -20 gpurun_out/r3v_configs.log; exit 1; }
grep '^{' gpurun_out/r3v_configs.log
echo all done
