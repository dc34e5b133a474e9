# round 3: bench lines with CG mode 5 (auto), mode A/B at other sizes, profile, full GPU suite
cd /root/repo
(while true; do date > gpurun_out/hb; sleep 30; done) &
HB=$!
trap "kill $HB" EXIT
set -o pipefail
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r3d_bench20.json 2> gpurun_out/r3d_bench20.err || { tail -20 gpurun_out/r3d_bench20.err; exit 1; }
cat gpurun_out/r3d_bench20.json
timeout -k 10 300 python3 bench.py --steps 500 --warmup 50 --no-cpu > gpurun_out/r3d_bench500.json 2> gpurun_out/r3d_bench500.err || { tail -20 gpurun_out/r3d_bench500.err; exit 1; }
timeout -k 10 300 python -u tools/cg_ab.py poisson3d 128,128,128 4 9=1 9=2 9=5 > gpurun_out/r3d_ab128.log 2>&1 || { tail -20 gpurun_out/r3d_ab128.log; exit 1; }
timeout -k 10 300 python -u tools/cg_ab.py poisson2d 4096,4096,1 4 9=2 9=5 > gpurun_out/r3d_abc2.log 2>&1 || { tail -20 gpurun_out/r3d_abc2.log; exit 1; }
cat gpurun_out/r3d_ab128.log gpurun_out/r3d_abc2.log | grep '^{'
STEPS=50 timeout -k 10 900 bash tools/profile.sh || { echo profile failed; exit 1; }
echo done
