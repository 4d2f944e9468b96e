#!/bin/bash
# round-3: DoG persistent xy (tests + A/B + PMC), z-pass stagger-group A/B
export TMPDIR=/tmp
O=gpurun_out/r3h
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dog.py tests/test_gpu_configs.py::test_c4_dog_768_matches_oracle_on_crops -x -q --timeout 250 --timeout-method thread > $O/dog_tests.log 2>&1 || exit 1
tools/dog_ab.sh $O/dogab "SPIMDECON_DOG_XY_ROUNDS=1" "SPIMDECON_DOG_XY_ROUNDS=4" "SPIMDECON_DOG_Z_BY=16" || exit 2
tools/pmc_dog.sh $O/dogpmc || exit 3
Q="--no-cpu-baseline --no-strong-line --no-default-mode"
for g in 8 1 4; do
  SPIMDECON_ZSTAG_GROUP=$g timeout -k 10 200 python3 bench.py $Q > $O/bench_sg$g.log 2>&1 || exit 4
done
