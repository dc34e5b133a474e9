# round 3: mode 5 + 27-point z-march parity, A/B, then the P = 8 / C2 / C5 tests
cd /root/repo
(while true; do date > gpurun_out/hb; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rccl_watchdog.py tests/test_gpu_cgfuse.py tests/test_gpu_vcodes.py > gpurun_out/r3c_unit.log 2>&1 || { tail -40 gpurun_out/r3c_unit.log; exit 1; }
tail -3 gpurun_out/r3c_unit.log
timeout -k 10 300 python -u tools/cg_ab.py poisson3d 256,256,256 4 9=2 9=5 9=5+46=0 > gpurun_out/r3c_c3ab.log 2>&1 || { tail -30 gpurun_out/r3c_c3ab.log; exit 1; }
cat gpurun_out/r3c_c3ab.log
timeout -k 10 300 python -u tools/cg_ab.py poisson3d27 512,512,64 4 45=3 45=4 45=5 45=6 42=1+45=4 42=1+45=6 > gpurun_out/r3c_c5ab.log 2>&1 || { tail -30 gpurun_out/r3c_c5ab.log; exit 1; }
cat gpurun_out/r3c_c5ab.log
timeout -k 10 1100 python -u -m pytest -v --timeout 900 --timeout-method thread \
  tests/test_gpu_multirank.py::test_north_star_partition_p8 \
  tests/test_gpu_multirank.py::test_c5_p8_weak_scaling_properties \
  tests/test_gpu_fullsize.py::test_c2_full_parity > gpurun_out/r3c_tests.log 2>&1
rc=$?
tail -30 gpurun_out/r3c_tests.log
exit $rc
