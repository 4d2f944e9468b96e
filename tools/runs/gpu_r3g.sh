#!/bin/bash
# round-3: full GPU suite, then z-pass stagger-group A/B
export TMPDIR=/tmp
O=gpurun_out/r3g
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=15 > $O/gpu_tests.log 2>&1 || exit 1
Q="--no-cpu-baseline --no-strong-line --no-default-mode"
for g in 8 1; do
  SPIMDECON_ZSTAG_GROUP=$g timeout -k 10 200 python3 bench.py $Q > $O/bench_sg$g.log 2>&1 || exit 2
done
