# round 3 (session 2): chunk MDot with lane-distributed sums; GMRES basis placement A/B
cd /root/repo
(while true; do date > gpurun_out/hb; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v -s -k "gmres or c4_full or jacobi_by_code" --timeout 600 --timeout-method thread > gpurun_out/r3p_tests.log 2>&1 || { tail -40 gpurun_out/r3p_tests.log; exit 1; }
tail -2 gpurun_out/r3p_tests.log
timeout -k 10 400 python3 -u tools/gmres_op_ab.py 256 3 "54=0" "54=256" "54=4096" "18=0" "50=1" > gpurun_out/r3p_ab.log 2>&1 || { tail -20 gpurun_out/r3p_ab.log; exit 1; }
cat gpurun_out/r3p_ab.log
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r3p_tr -o run -f csv -- python3 tools/gmres_trace.py 256 60 > gpurun_out/r3p_tr.log 2>&1 || { tail -20 gpurun_out/r3p_tr.log; exit 1; }
echo all done
