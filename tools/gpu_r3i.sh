# round 3: 27-point forms 2 / 3 parity + C5-share A/B under a kernel trace
cd /root/repo
(while true; do date > gpurun_out/hb; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_vcodes.py -k "lean_kernel" > gpurun_out/r3i_unit.log 2>&1 || { tail -40 gpurun_out/r3i_unit.log; exit 1; }
tail -2 gpurun_out/r3i_unit.log
mkdir -p gpurun_out/c5trace3
timeout -k 10 400 rocprofv3 --kernel-trace -f csv -d gpurun_out/c5trace3 -o run -- python3 tools/knob_runs.py poisson3d27 512,512,64 100 49=1 49=3+45=5 49=3+45=4 49=3+45=6 49=1+45=6 > gpurun_out/r3i_c5.log 2>&1 || { tail -30 gpurun_out/r3i_c5.log; exit 1; }
grep '^{' gpurun_out/r3i_c5.log
python3 tools/trace_kernels.py gpurun_out/c5trace3/run_kernel_trace.csv zm27 12
echo all done
