# round 3 (session 2): full GPU suite with the plane-pipelined 27-point default, slowest tests listed
cd /root/repo
(while true; do date > gpurun_out/hb; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread --durations=30 > gpurun_out/r3aa_suite.log 2>&1 || { tail -60 gpurun_out/r3aa_suite.log; exit 1; }
tail -40 gpurun_out/r3aa_suite.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3aa_smoke.log 2>&1 || { tail -20 gpurun_out/r3aa_smoke.log; exit 1; }
tail -1 gpurun_out/r3aa_smoke.log
timeout -k 10 600 python3 tools/bench_configs.py > gpurun_out/r3aa_configs.log 2>&1 || { tail -20 gpurun_out/r3aa_configs.log; exit 1; }
grep '^{' gpurun_out/r3aa_configs.log
echo all done
