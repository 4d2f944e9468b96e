#!/bin/bash
# round 4 (q): the refresh's test half (tools/runs/gpu_r4_final.sh tests: whole -m gpu suite, smoke),
# then gpu_r4p.sh's A/B (y-pass prefetch at every length, SPIMDECON_YPF=2, vs the default)
bash tools/runs/gpu_r4_final.sh tests || exit $?
bash tools/runs/gpu_r4p.sh
