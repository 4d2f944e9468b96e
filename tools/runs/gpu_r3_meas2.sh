#!/bin/bash
# round-3 final pass 2: engine PMC traffic; DoG bench, kernel trace and PMC
export TMPDIR=/tmp
O=gpurun_out/r3m2
mkdir -p $O
tools/pmc_engine.sh $O/pmc || exit 1
python3 tools/pmc_summary.py $O/pmc --json $O/pmc_traffic.json --dims 540,540,536 > $O/pmc.md || exit 2
timeout -k 10 300 python3 -u tools/dog_bench.py > $O/dog.log 2>&1 || exit 3
grep '^{' $O/dog.log | tail -1 > $O/dog.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/dogkt -o k --output-format csv -- python3 tools/dog_bench.py --reps 3 --device-only > $O/dogkt.log 2>&1 || exit 4
cp $(ls $O/dogkt/*/k_kernel_stats.csv $O/dogkt/k_kernel_stats.csv 2>/dev/null | head -1) $O/dog_kernel_stats.csv
tools/pmc_dog.sh $O/dogpmc || exit 5
