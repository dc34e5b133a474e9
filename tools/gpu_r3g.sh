# round 3: the 27-point z-march forms -- parity, then C5-share variants under a kernel trace
cd /root/repo
(while true; do date > gpurun_out/hb; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_vcodes.py \
  "tests/test_gpu_multirank.py::test_distributed_row_pairs" "tests/test_gpu_fullsize.py::test_c5_share_full_parity" \
  "tests/test_gpu_multirank.py::test_c5_p8_weak_scaling_properties" > gpurun_out/r3g_unit.log 2>&1 || { tail -40 gpurun_out/r3g_unit.log; exit 1; }
tail -2 gpurun_out/r3g_unit.log
mkdir -p gpurun_out/c5trace2
timeout -k 10 400 rocprofv3 --kernel-trace -f csv -d gpurun_out/c5trace2 -o run -- python3 tools/knob_runs.py poisson3d27 512,512,64 100 48=1 48=0 45=4 45=8 49=2+45=3 > gpurun_out/r3g_c5.log 2>&1 || { tail -30 gpurun_out/r3g_c5.log; exit 1; }
grep '^{' gpurun_out/r3g_c5.log
python3 tools/trace_kernels.py gpurun_out/c5trace2/run_kernel_trace.csv zm27 12
echo all done
