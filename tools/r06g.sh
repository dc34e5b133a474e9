# round 6 step g: CB / assembly tests, bench legs (host CSR copy, random
# pattern), PMC request counts of the random-pattern MatMult's two passes
set -o pipefail
R=$(pwd)
bash tools/gpu_run.sh r06g "tests:cb or index_widths or assembly" || exit 1
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 --no-cpu --no-configs --no-general > gpurun_out/r06g_bench.log 2>&1 || exit 1
TAG=r06g_rand REGEX="cb_|spmv" PMC_PASSES="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum;WRITE_SIZE TCC_EA0_WRREQ_64B_sum;FETCH_SIZE" bash tools/pmc_kernels.sh python3 $R/tools/random_spmv.py 24 || exit 1
python3 tools/pmc_table.py gpurun_out/pmc_r06g_rand > gpurun_out/r06g_rand_pmc.txt 2>&1
echo done
