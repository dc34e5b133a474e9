#!/bin/bash
# PMC passes over tools/spmv_only.py (one pass per counter group, each under its own limit)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc${TAG:-}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
ARGS="${SPMV_ARGS:-poisson3d 256 20 ${SPMV_KNOBS:-}}"
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SMEM" \
         "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
         "TA_TA_BUSY_sum TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_WR SQ_IFETCH"; do
  i=$((i+1))
  case " ${PASSES:-1 2 3 4 5} " in *" $i "*) ;; *) continue ;; esac
  timeout -s KILL 90 rocprofv3 --pmc $P -f csv --kernel-include-regex spmv_sell -d $OUT/p$i -o run -- python3 $R/tools/spmv_only.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed: $P" >> $OUT/failed.txt; exit 1; }
done
