# round 6: per-kernel traffic + durations of the configuration legs (C5 share,
# C2, C4, C3) with the library's defaults
set -o pipefail
R=$(pwd)
export TMPDIR=/tmp
for cfg in "c5:poisson3d27 512 512 64 cg 50" "c2:poisson2d 4096 4096 1 cg 100" "c4:convdiff3d 256 256 256 gmres 60" "c3:poisson3d 256 256 256 cg 100"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $R/gpurun_out/r06o_trace_$tag -o run -- python3 $R/tools/config_run.py $args > $R/gpurun_out/r06o_trace_$tag.log 2>&1) || exit 1
  TAG=r06o_$tag REGEX="spmv|cg_|mdot|maxpy|gm_" PMC_PASSES="TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum;WRITE_SIZE" bash tools/pmc_kernels.sh python3 $R/tools/config_run.py $args || exit 1
  python3 tools/traffic_table.py gpurun_out/pmc_r06o_$tag gpurun_out/r06o_trace_$tag > gpurun_out/r06o_traffic_$tag.txt 2>&1
done
echo done
