#!/bin/bash
# round 5 (c): per-phase s_memtime stamps of the x tiles (diagnostic build, no PF) at 540 /
# 1050 / 2100; A/B of the persistent prefetch tiles (PF at 2100 = default, PF from 1050, no
# PF) on C3 (--strong) and the C5 rank slab; parity of the default build at 1050 / 2100
export TMPDIR=/tmp
O=gpurun_out/r5c
mkdir -p $O
B="python3 -u bench.py --steps 1 --warmup 1 --no-timing --no-cpu-baseline --no-default-mode --no-strong-line"
S=$PWD/exp/libspimdecon_stamp.so
SPIMDECON_LIB=$S timeout -k 10 200 $B > $O/s540.log 2>&1 || exit 1
SPIMDECON_LIB=$S timeout -k 10 200 $B --psftype OPTIMIZATION_I --lam 0.006 > $O/s540t.log 2>&1 || exit 2
SPIMDECON_LIB=$S timeout -k 10 300 $B --strong > $O/s1050.log 2>&1 || exit 3
SPIMDECON_LIB=$S timeout -k 10 300 $B --c5-rank > $O/s2100.log 2>&1 || exit 4
for f in s540 s540t s1050 s2100; do echo "== $f"; grep xt_stamp $O/$f.log | tail -4; done
T="python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-default-mode"
for v in main pf1050 nopf; do
  if [ $v = main ]; then L=""; else L=$PWD/exp/libspimdecon_$v.so; fi
  SPIMDECON_LIB=$L timeout -k 10 300 $T --strong > $O/c3_$v.log 2>&1 || exit 6
  tail -1 $O/c3_$v.log > $O/c3_$v.json
  SPIMDECON_LIB=$L timeout -k 10 300 $T --c5-rank > $O/c5_$v.log 2>&1 || exit 7
  tail -1 $O/c5_$v.log > $O/c5_$v.json
done

# exchange overlap window at C3's 8-rank y-slab decomposition (8 local slabs on one GPU)
timeout -k 10 300 python3 -u bench.py --strong --local-slabs 8 --steps 3 --warmup 1 --no-cpu-baseline --no-default-mode > $O/c3x8.log 2>&1 || exit 8
tail -1 $O/c3x8.log > $O/c3x8.json
# streaming references
timeout -k 10 300 tools/zpattern_bench > $O/zpattern.txt 2>&1 || exit 9
timeout -k 10 600 python -u -m pytest tests/test_gpu_rl.py tests/test_gpu_golden.py tests/test_gpu_multidevice.py tests/test_gpu_scale.py::test_c5_rank_slab_geometry_vs_rocfft -m gpu -x -q --timeout 500 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 5
echo done-c
