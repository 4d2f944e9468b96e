export TMPDIR=/tmp
mkdir -p gpurun_out/r3b
timeout -k 10 240 python -u -m pytest tests/test_gpu_dog.py tests/test_gpu_configs.py::test_c4_dog_768_matches_oracle_on_crops -x -q --timeout 200 --timeout-method thread > gpurun_out/r3b/dog_tests.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3b/dogkt -o k --output-format csv -- python3 tools/dog_bench.py --reps 3 --device-only > gpurun_out/r3b/dog.log 2>&1 || exit 2
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_multidevice.py::test_c3_strong_decomposition_exchange_accounting -x -v -s --timeout 880 --timeout-method thread > gpurun_out/r3b/tests.log 2>&1 || exit 3
