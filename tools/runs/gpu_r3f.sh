#!/bin/bash
# round-3: y-pass register prefetch A/B (540 / C3 1050 / C4-like 800) + DoG defaults trace
export TMPDIR=/tmp
O=gpurun_out/r3f
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dog.py tests/test_gpu_configs.py::test_c4_dog_768_matches_oracle_on_crops -x -q --timeout 250 --timeout-method thread > $O/dog_tests.log 2>&1 || exit 9
Q="--no-cpu-baseline --no-strong-line --no-default-mode"
for y in 2 0; do
  SPIMDECON_YPF=$y timeout -k 10 200 python3 bench.py $Q > $O/b540_ypf$y.log 2>&1 || exit 1
done
for y in 1 0; do
  SPIMDECON_YPF=$y timeout -k 10 300 python3 bench.py $Q --strong --steps 5 --warmup 1 > $O/bc3_ypf$y.log 2>&1 || exit 2
  SPIMDECON_YPF=$y timeout -k 10 300 python3 bench.py $Q --shape 768 768 768 --views 8 --ksize 31 --psftype OPTIMIZATION_I --lam 0.006 --steps 5 --warmup 1 > $O/bc4_ypf$y.log 2>&1 || exit 3
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/dogkt -o k --output-format csv -- python3 tools/dog_bench.py --reps 3 --device-only > $O/dog.log 2>&1 || exit 4
