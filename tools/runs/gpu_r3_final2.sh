#!/bin/bash
# round-3 (session 2) final pass 2: DoG bench, kernel trace and PMC; the C4 pipeline
# (the engine kernels are unchanged since gpu_r3_meas2.sh: its PMC summary stands)
export TMPDIR=/tmp
O=gpurun_out/r3f2
mkdir -p $O
timeout -k 10 300 python3 -u tools/dog_bench.py > $O/dog.log 2>&1 || exit 3
grep '^{' $O/dog.log | tail -1 > $O/dog.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/dogkt -o k --output-format csv -- python3 tools/dog_bench.py --reps 3 --device-only > $O/dogkt.log 2>&1 || exit 4
cp $(ls $O/dogkt/*/k_kernel_stats.csv $O/dogkt/k_kernel_stats.csv 2>/dev/null | head -1) $O/dog_kernel_stats.csv
tools/pmc_dog.sh $O/dogpmc || exit 5
timeout -k 10 400 python3 -u tools/c4_pipeline.py > $O/c4.log 2>&1 || exit 6
grep '^{' $O/c4.log | tail -1 > $O/c4.json
