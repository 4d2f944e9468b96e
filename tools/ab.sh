#!/bin/bash
# A/B bench runs on the GPU box: tools/ab.sh OUTDIR "ENV1" "ENV2" ... (each ENV a space-separated
# list of VAR=value, "-" for none); one bench line per variant in OUTDIR/ab_<i>.json
set -o pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for e in "$@"; do
  [ "$e" = "-" ] && e=""
  env $e timeout -k 10 200 python3 bench.py --steps 5 --no-cpu-baseline > $OUT/ab_$i.log 2>&1 || exit 1
  tail -1 $OUT/ab_$i.log > $OUT/ab_$i.json
  i=$((i+1))
done
