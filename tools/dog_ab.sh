#!/bin/bash
# A/B of the fused DoG tile shapes on the GPU box: one kernel trace per variant.
# usage: tools/dog_ab.sh OUT "ENV=VAL ENV2=VAL" "ENV=VAL" ...
set -o pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i+1))
  env $v true || exit 1
  (export $v; timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/v$i -o k --output-format csv -- python3 tools/dog_bench.py --reps 3 --device-only > $OUT/v$i.log 2>&1) || exit $?
  echo "== v$i: $v" >> $OUT/summary.txt
  grep '^{' $OUT/v$i.log | tail -1 >> $OUT/summary.txt
  python3 - $OUT/v$i/k_kernel_stats.csv >> $OUT/summary.txt <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_dog" in r["Name"] or "k_minmax(" in r["Name"]:
        name = r["Name"].split("::")[-1][:48]
        print("  %-48s max %8.1f us  avg %8.1f us" % (name, float(r["MaxNs"]) / 1e3, float(r["AverageNs"]) / 1e3))
PY
done
