# round 3 (session 2): coded z-march + one-pass MDot -- tests, A/B, C4 trace
cd /root/repo
(while true; do date > gpurun_out/hb; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -s -k "pair_code_zmarch or distributed_code_zmarch or c4_full or gmres or jacobi_by_code" --timeout 600 --timeout-method thread > gpurun_out/r3m_tests.log 2>&1 || { tail -40 gpurun_out/r3m_tests.log; exit 1; }
tail -3 gpurun_out/r3m_tests.log
timeout -k 10 300 python3 -u tools/gmres_ab.py 256 3 "52=1" "52=0" "50=0" "50=0+52=0" > gpurun_out/r3m_ab.log 2>&1 || { tail -20 gpurun_out/r3m_ab.log; exit 1; }
cat gpurun_out/r3m_ab.log
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r3m_tr -o run -f csv -- python3 tools/gmres_trace.py 256 60 > gpurun_out/r3m_tr.log 2>&1 || { tail -20 gpurun_out/r3m_tr.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r3m_calib -o run -f csv -- python3 tools/calib_stream.py > gpurun_out/r3m_calib.log 2>&1 || { tail -20 gpurun_out/r3m_calib.log; exit 1; }
timeout -k 10 300 python3 -u tools/bench_general.py c4 > gpurun_out/r3m_c4.log 2>&1 || { tail -20 gpurun_out/r3m_c4.log; exit 1; }
grep '^{' gpurun_out/r3m_c4.log
echo all done
