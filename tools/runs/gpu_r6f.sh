#!/bin/bash
# round 6 (f): the new multi-slab tests (pull kernel, concurrent boundary launches), the
# engine classes of every BASELINE geometry at HEAD (wall-time x passes), and the pull
# kernel against hipMemcpyAsync for the local halo copies of C3's 8-slab emulation
# (one GPU: both are shader copies here -- the blit kernel vs k_pull_copy -- so the
# prediction is equal within 5 % of the 0.38 ms exchange; the SDMA / xGMI comparison
# needs two GPUs)
export TMPDIR=/tmp
O=gpurun_out/r6f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_multidevice.py -x -q --timeout 500 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc = 0 ] || exit 1
bash tools/engine_classes.sh $O/classes || exit 1
for k in 1 2; do
  for pull in copy kernel; do
    SPIMDECON_PULL=$pull timeout -k 10 240 python3 bench.py --no-cpu-baseline --strong --local-slabs 8 --steps 4 --warmup 1 --no-default-mode --no-strong-line > $O/pull_${pull}_$k.json 2> $O/pull_${pull}_$k.err || { echo "pull $pull failed"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/pull_${pull}_$k.json').read().strip().splitlines()[-1]); k=d['kernel_ms']
print('pull $pull $k value %.1f ms %.2f halo_exchange %.3f window %.3f' % (d['value'], d['ms_per_step'], k['halo_exchange']['avg_ms'], k['exchange_window']['avg_ms']))"
  done
done
echo done-r6f
