#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, each under its own limit)
# over an arbitrary command:  TAG=x REGEX=kernel-regex tools/pmc_kernels.sh <cmd...>
# PMC_PASSES (optional): counter groups separated by ';' replacing the default five.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_${TAG:-run}
mkdir -p $OUT
export TMPDIR=/tmp
DEFAULT="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SMEM;\
FETCH_SIZE;\
WRITE_SIZE TCC_HIT_sum TCC_MISS_sum;\
TA_TA_BUSY_sum TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum;\
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_WR SQ_IFETCH"
IFS=';' read -ra GROUPS_ <<< "${PMC_PASSES:-$DEFAULT}"
i=0
for P in "${GROUPS_[@]}"; do
  i=$((i+1))
  case " ${PASSES:-$(seq -s ' ' 1 ${#GROUPS_[@]})} " in *" $i "*) ;; *) continue ;; esac
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $P -f csv --kernel-include-regex "${REGEX:-.}" -d $OUT/p$i -o run -- "$@" > $OUT/p$i.log 2>&1) || { echo "pass $i failed: $P" >> $OUT/failed.txt; exit 1; }
done
