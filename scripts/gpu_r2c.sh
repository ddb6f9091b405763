# round 2, call c: multi-device tests, the whole GPU suite, extended dual-issue probe, bench (lib mode)
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out/r2c &&
timeout -k 10 300 python -u -m pytest tests/test_multi_device.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r2c/multi.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2c/gpu_tests.log 2>&1 &&
timeout -k 10 180 ./scripts/ubench_dual 8 > gpurun_out/r2c/dual8.txt 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r2c/bench.log 2>&1 &&
timeout -k 10 300 python -u bench.py --devices 0,0 --no-cpu-baseline > gpurun_out/r2c/bench_00.log 2>&1
