# round 3: mode-5 knob A/B at 256^3 (non-temporal reads, grids, unroll, x batch)
cd /root/repo
(while true; do date > gpurun_out/hb; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 500 python -u tools/cg_ab.py poisson3d 256,256,256 5 9=5 9=5+29=4 9=5+29=4+12=16384 9=5+29=4+12=12288 9=5+29=4+12=32768 > gpurun_out/r3j_ab.log 2>&1 || { tail -20 gpurun_out/r3j_ab.log; exit 1; }
grep '^{' gpurun_out/r3j_ab.log
echo all done
