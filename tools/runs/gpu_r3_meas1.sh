#!/bin/bash
# round-3 final pass 1: the fixed aspect test, smoke(), the bench line, its kernel trace
export TMPDIR=/tmp
O=gpurun_out/r3m1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py::test_c5_decomposition_matches_oracle_256x256x128 -q -rA --timeout 250 --timeout-method thread > $O/aspect.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 500 python3 -u bench.py > $O/bench.log 2>&1 || exit 3
tail -1 $O/bench.log > $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o k --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-strong-line > $O/kt.log 2>&1 || exit 4
cp $(ls $O/kt/*/k_kernel_stats.csv $O/kt/k_kernel_stats.csv 2>/dev/null | head -1) $O/kernel_stats.csv
