#!/bin/bash
# round 6 (ab): the pipelined DoG z stage (k_dog_xy parts on the call's stream, k_dog_zconv
# chunks on a second one).  Prediction: k_dog_zconv (1.12 ms, HBM-bound, no LDS) overlaps the
# VALU-bound k_dog_xy (1.39 ms) of later parts; the combined 10.8 GB bound at ~5.8 TB/s is
# 1.87 ms against 2.51 ms back to back: -0.2..0.4 ms per 768^3 view if the CUs co-schedule the
# two kernels, less the tails of 4 part launches.  H = 192 and 128 measured.
export TMPDIR=/tmp
O=gpurun_out/r6ab
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_dog.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc = 0 ] || { grep -E "FAILED|Error" $O/tests.log | head; exit 1; }
for r in 1 2 3; do
  for cfg in "0 192" "1 192" "1 128" "1 256"; do
    set -- $cfg
    SPIMDECON_DOG_PIPE=$1 SPIMDECON_DOG_PIPE_CHUNK=$2 timeout -k 10 200 python3 tools/dog_bench.py --reps 5 --device-only > $O/bench_$1_$2_$r.log 2>&1 || { echo "bench failed"; tail -3 $O/bench_$1_$2_$r.log; exit 1; }
    echo "pipe=$1 H=$2 rep $r $(tail -1 $O/bench_$1_$2_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_device_resident"])')"
  done
done
echo done-r6ab
