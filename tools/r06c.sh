set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 120 ./tools/gather_probe 24 9 > gpurun_out/r06c_gather24.txt 2>&1 || exit 1
timeout -k 10 120 ./tools/gather_probe 22 9 > gpurun_out/r06c_gather22.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu --no-configs --no-general --no-asm > gpurun_out/r06c_bench_random.log 2>&1 || exit 1
TAG=r06c_cold REGEX="dot_partials|spmv" PMC_PASSES="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_REQUEST_sum;FETCH_SIZE;TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" bash tools/pmc_kernels.sh python3 $R/tools/cold_probe.py 256 5 || exit 1
python3 tools/cold_pmc_table.py gpurun_out/pmc_r06c_cold > gpurun_out/r06c_cold_pmc.txt 2>&1
bash tools/ab_knobs.sh "" "11=64" "11=512" "11=4096" > gpurun_out/r06c_skew_ab.txt 2>&1
echo done
