#!/bin/bash
# round 5 (u): PSF extraction with pooled per-view buffers / streams and 32 loads ahead in the
# bead sums (main) vs before (r5z): PSF and pipeline tests on main, then the C4 pipeline's
# stage times for both, alternated
export TMPDIR=/tmp
O=gpurun_out/r5u
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_psf.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 5
for k in 1 2; do
for v in main r5z; do
  if [ $v = main ]; then L=""; else L=$PWD/exp/libspimdecon_$v.so; fi
  SPIMDECON_LIB=$L timeout -k 10 400 python3 -u tools/c4_pipeline.py --timepoints 3 > $O/c4p_${v}_$k.log 2>&1 || exit 1
  grep '^{' $O/c4p_${v}_$k.log | tail -1 > $O/c4p_${v}_$k.json
  python3 -c "
import json; d=json.load(open('$O/c4p_${v}_$k.json'))
print('$v $k', d['total_s'], [(t['t'], round(t['stage_ms']['extract_psf'],1), round(t['stage_ms']['prepare_inputs'],1), round(t['s'],3)) for t in d['timepoints']])"
done
done
echo done-u
