#!/bin/bash
# round 5 (l): where the C4 pipeline's non-RL stages spend their time -- kernel trace of two
# timepoints (tools/c4_pipeline.py) -- and a fresh DoG bench line with its kernel trace
export TMPDIR=/tmp
O=gpurun_out/r5l
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/c4kt -o k --output-format csv -- python3 tools/c4_pipeline.py --timepoints 2 > $O/c4kt.log 2>&1 || exit 1
cp $(ls $O/c4kt/*/k_kernel_stats.csv $O/c4kt/k_kernel_stats.csv 2>/dev/null | head -1) $O/c4_kernel_stats.csv
timeout -k 10 300 python3 tools/dog_bench.py > $O/dog.log 2>&1 || exit 2
grep '^{' $O/dog.log | tail -1 > $O/dog.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dogkt -o k --output-format csv -- python3 tools/dog_bench.py --reps 3 --device-only > $O/dogkt.log 2>&1 || exit 3
cp $(ls $O/dogkt/*/k_kernel_stats.csv $O/dogkt/k_kernel_stats.csv 2>/dev/null | head -1) $O/dog_kernel_stats.csv
cat $O/dog.json
echo done-l
