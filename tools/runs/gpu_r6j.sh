#!/bin/bash
# round 6 (j): measurement refresh at HEAD -- the bench line, its kernel trace and PMC
# traffic (tools/measure.sh), the C5 rank bench + kernel trace, the DoG bench + trace,
# the C4 pipeline
export TMPDIR=/tmp
O=gpurun_out/r6j
mkdir -p $O
bash tools/measure.sh $O/m || { echo "measure failed"; exit 1; }
tail -c 600 $O/m/bench.json; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c5kt -o k --output-format csv -- python3 bench.py --c5-rank --steps 4 --warmup 1 --no-cpu-baseline > $O/c5.log 2>&1 || { echo "c5 failed"; exit 1; }
tail -1 $O/c5.log > $O/c5.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dogkt -o k --output-format csv -- python3 tools/dog_bench.py --reps 3 --device-only > $O/dog_bench.log 2>&1 || { echo "dog failed"; exit 1; }
tail -3 $O/dog_bench.log
timeout -k 10 400 python3 tools/c4_pipeline.py > $O/c4.log 2>&1 || { echo "c4 failed"; exit 1; }
tail -3 $O/c4.log
echo done-r6j
