#!/bin/bash
# round 5 (y2): 4-pair quotient tiles at 800 (q800) vs main, C4, alternated twice; then the PSF
# extraction bench with its HIP API trace
export TMPDIR=/tmp
O=gpurun_out/r5y2
mkdir -p $O
T="python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-default-mode"
for k in 1 2; do
for v in main q800; do
  if [ $v = main ]; then L=""; else L=$PWD/exp/libspimdecon_$v.so; fi
  SPIMDECON_LIB=$L timeout -k 10 300 $T --size 768 --views 8 --ksize 31 --psftype OPTIMIZATION_I --lam 0.006 --no-strong-line > $O/c4_${v}_$k.log 2>&1 || exit 2
  tail -1 $O/c4_${v}_$k.log > $O/c4_${v}_$k.json
done
done
python3 tools/ab_summary.py $O/c4_*.json
timeout -k 10 300 python3 tools/psf_bench.py > $O/psf.log 2>&1 && tail -1 $O/psf.log
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats -d $O/kt -o k --output-format csv -- python3 tools/psf_bench.py --reps 3 > $O/kt.log 2>&1
echo done-y2
