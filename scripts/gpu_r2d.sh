# round 2, call d: PMC passes at HEAD (K1, K2) + FETCH_SIZE calibration + kernel-trace stats of the bench
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out/r2d &&
bash scripts/pmc_head.sh gpurun_out/r2d/pmc > gpurun_out/r2d/pmc.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2d/trace -o trace -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r2d/trace_bench.log 2>&1
