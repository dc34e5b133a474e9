#!/bin/bash
# Where the MatMult's time goes: wave-state, VALU, TA/TCP counters for the
# 256^3 row-pair MatMult standalone (tools/spmv_only.py) and inside CG (bench.py).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
(cd /tmp && timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/counters.txt 2>&1) || true
export PMC_PASSES="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM;\
TA_TA_BUSY_sum TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE;\
SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_IFETCH;\
FETCH_SIZE;\
WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
TAG=solo REGEX=spmv_sell $R/tools/pmc_kernels.sh python3 $R/tools/spmv_only.py poisson3d 256 50
TAG=cg REGEX=spmv_sell $R/tools/pmc_kernels.sh python3 $R/bench.py --steps 50 --warmup 5 --no-cpu --no-solve
