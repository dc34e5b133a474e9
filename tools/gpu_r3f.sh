# round 3: P = 4 / P = 2 interior-rank proxies; C5-share 27-point z-march variants under a kernel trace
cd /root/repo
(while true; do date > gpurun_out/hb; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
export TMPDIR=/tmp
for Z in 64 128; do
  PLANES=$Z timeout -k 10 400 python -u tools/rank_proxy.py 3 150 9=1 9=2 9=5 > gpurun_out/r3f_proxy$Z.log 2>&1 || { tail -30 gpurun_out/r3f_proxy$Z.log; exit 1; }
  grep '^{' gpurun_out/r3f_proxy$Z.log
done
mkdir -p gpurun_out/c5trace
timeout -k 10 400 rocprofv3 --kernel-trace -f csv -d gpurun_out/c5trace -o run -- python3 tools/knob_runs.py poisson3d27 512,512,64 100 45=3 45=4 45=6 42=1+45=4 42=1+45=6 42=1+45=8 > gpurun_out/r3f_c5.log 2>&1 || { tail -30 gpurun_out/r3f_c5.log; exit 1; }
grep '^{' gpurun_out/r3f_c5.log
python3 tools/trace_kernels.py gpurun_out/c5trace/run_kernel_trace.csv zm27 12
echo all done
