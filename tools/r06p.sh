# round 6: VALU instruction counts of the C5 share and C3 CG kernels
set -o pipefail
R=$(pwd)
export TMPDIR=/tmp
for cfg in "c5:poisson3d27 512 512 64 cg 50" "c3:poisson3d 256 256 256 cg 100"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  TAG=r06p_$tag REGEX="spmv|cg_pb" PMC_PASSES="SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES SQ_WAVES SQ_INSTS_SALU" bash tools/pmc_kernels.sh python3 $R/tools/config_run.py $args || exit 1
  python3 tools/pmc_table.py gpurun_out/pmc_r06p_$tag > gpurun_out/r06p_valu_$tag.txt 2>&1
done
echo done
