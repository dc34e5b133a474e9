# the whole GPU test suite, as the driver runs it at round end
cd /root/repo
(while true; do date > gpurun_out/hb; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 1150 python -u -m pytest -x -q -m gpu --timeout 900 --timeout-method thread tests > gpurun_out/suite.log 2>&1
rc=$?
tail -25 gpurun_out/suite.log
exit $rc
