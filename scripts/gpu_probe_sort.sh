cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out/sortp &&
timeout -k 10 120 ./scripts/sort_probe > gpurun_out/sortp/sort.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline > gpurun_out/sortp/bench_c5.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c4 --steps 2 --no-cpu-baseline > gpurun_out/sortp/bench_c4.log 2>&1
