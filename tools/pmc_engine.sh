#!/bin/bash
# PMC passes over one RL iteration of the engine kernels (run on the GPU box).
# usage: tools/pmc_engine.sh OUTDIR [extra bench args]
set -o pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
B="python3 bench.py --steps 1 --warmup 0 --no-timing --no-cpu-baseline --no-default-mode --no-strong-line --no-legacy-line $*"
R="--kernel-include-regex k_xpass|k_xrows|k_xtile|k_colpass|k_col2f|k_zdirect|k_zdma|k_zdmc|k_yzy"
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS $R -d $OUT/p1 -o p1 --output-format csv -- $B > $OUT/p1.log 2>&1 &&
timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE $R -d $OUT/p2 -o p2 --output-format csv -- $B > $OUT/p2.log 2>&1 &&
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE $R -d $OUT/p3 -o p3 --output-format csv -- $B > $OUT/p3.log 2>&1 &&
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE $R -d $OUT/p4 -o p4 --output-format csv -- $B > $OUT/p4.log 2>&1
