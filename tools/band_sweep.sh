set -o pipefail
mkdir -p gpurun_out/band
export TMPDIR=/tmp
SPIMDECON_BAND=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_rl.py -x -q --timeout 120 --timeout-method thread > gpurun_out/band/tests.log 2>&1 || exit 1
for b in 0 1 2 3 4 6 17; do
  SPIMDECON_BAND=$b timeout -k 10 200 python3 bench.py --steps 5 --no-cpu-baseline > gpurun_out/band/b$b.log 2>&1 || exit 1
  tail -1 gpurun_out/band/b$b.log > gpurun_out/band/b$b.json
done
