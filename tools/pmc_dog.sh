#!/bin/bash
# PMC passes over the fused DoG kernels (run on the GPU box): tools/pmc_dog.sh OUT [env assignments]
set -o pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
for v in "$@"; do export $v; done
B="python3 tools/dog_bench.py --reps 1 --device-only"
R="--kernel-include-regex k_dog|k_minmax"
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS $R -d $OUT/p1 -o p1 --output-format csv -- $B > $OUT/p1.log 2>&1 &&
timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE $R -d $OUT/p2 -o p2 --output-format csv -- $B > $OUT/p2.log 2>&1 &&
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE $R -d $OUT/p3 -o p3 --output-format csv -- $B > $OUT/p3.log 2>&1 &&
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE $R -d $OUT/p4 -o p4 --output-format csv -- $B > $OUT/p4.log 2>&1 &&
python3 tools/pmc_summary.py $OUT > $OUT/pmc.md
