# round 3 (session 2): C4 profile with the chunk MDot / coded z-march; all configurations
cd /root/repo
(while true; do date > gpurun_out/hb; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3r_c4 -o run -f csv -- python3 tools/bench_general.py c4 > gpurun_out/r3r_c4.log 2>&1 || { tail -20 gpurun_out/r3r_c4.log; exit 1; }
grep '^{' gpurun_out/r3r_c4.log
timeout -k 10 600 python3 tools/bench_configs.py > gpurun_out/r3r_configs.log 2>&1 || { tail -20 gpurun_out/r3r_configs.log; exit 1; }
grep '^{' gpurun_out/r3r_configs.log
echo all done
