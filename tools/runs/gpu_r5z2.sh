#!/bin/bash
# round 5 (z2): the 4-pair update tiles with their own DFT lane map and pitch (main: AM 3,
# pitch L + 14 at 1050 / L + 8 at 800) vs AM 0 (am0); C3 and C4 alternated twice; the RL and
# PSF / pipeline parity tests on main (PSF samples with per-bead corner weights); the C4
# pipeline's stage times
export TMPDIR=/tmp
O=gpurun_out/r5z2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_rl.py tests/test_gpu_configs.py tests/test_gpu_psf.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 5
T="python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-default-mode"
for k in 1 2; do
for v in main am0; do
  if [ $v = main ]; then L=""; else L=$PWD/exp/libspimdecon_$v.so; fi
  SPIMDECON_LIB=$L timeout -k 10 300 $T --strong > $O/c3_${v}_$k.log 2>&1 || exit 1
  tail -1 $O/c3_${v}_$k.log > $O/c3_${v}_$k.json
  SPIMDECON_LIB=$L timeout -k 10 300 $T --size 768 --views 8 --ksize 31 --psftype OPTIMIZATION_I --lam 0.006 --no-strong-line > $O/c4_${v}_$k.log 2>&1 || exit 2
  tail -1 $O/c4_${v}_$k.log > $O/c4_${v}_$k.json
done
done
python3 tools/ab_summary.py $O/c3_*.json $O/c4_*.json
timeout -k 10 400 python3 -u tools/c4_pipeline.py --timepoints 3 > $O/c4p.log 2>&1 || exit 3
grep '^{' $O/c4p.log | tail -1 > $O/c4p.json
python3 -c "
import json; d=json.load(open('$O/c4p.json'))
print('c4p', d['total_s'], [(t['t'], round(t['stage_ms']['extract_psf'],1), round(t['s'],3)) for t in d['timepoints']])"
echo done-z2
