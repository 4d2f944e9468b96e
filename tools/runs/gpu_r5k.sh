#!/bin/bash
# round 5 (k): main = quotient image prefetch at 64 threads per pair (1050) + the
# wave-specialised 1050 y pass (k_ycol_ws; SPIMDECON_YPF=0 = the plain k_col2f).  A/B on one
# box, alternated twice: C3 main vs main YPF=0 vs upipe64 (two-slot update pipeline at 64
# threads, built without k_ycol_ws: compare with YPF=0); C4 main vs qpf7 (800-point quotient
# prefetching its 7 image float4 per row under 168 VGPRs); then the parity tests on main
export TMPDIR=/tmp
O=gpurun_out/r5k
mkdir -p $O
T="python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-default-mode"
timeout -k 10 300 python -u -m pytest tests/test_gpu_rl.py -m gpu -x -q -k "prefetch_bit_identical" --timeout 200 --timeout-method thread > $O/tests_ws.log 2>&1
rc=$?; tail -2 $O/tests_ws.log; [ $rc -eq 0 ] || exit 5
for k in 1 2; do
for v in main ypf0 upipe64; do
  L=""; Y=1
  [ $v = ypf0 ] && Y=0
  [ $v = upipe64 ] && L=$PWD/exp/libspimdecon_$v.so
  SPIMDECON_YPF=$Y SPIMDECON_LIB=$L timeout -k 10 300 $T --strong > $O/c3_${v}_$k.log 2>&1 || exit 1
  tail -1 $O/c3_${v}_$k.log > $O/c3_${v}_$k.json
done
for v in main qpf7; do
  if [ $v = main ]; then L=""; else L=$PWD/exp/libspimdecon_$v.so; fi
  SPIMDECON_LIB=$L timeout -k 10 300 $T --size 768 --views 8 --ksize 31 --psftype OPTIMIZATION_I --lam 0.006 --no-strong-line > $O/c4_${v}_$k.log 2>&1 || exit 2
  tail -1 $O/c4_${v}_$k.log > $O/c4_${v}_$k.json
done
done
python3 tools/ab_summary.py $O/c3_*.json $O/c4_*.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_rl.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 5
echo done-k
