# round 2, call h: kernel trace of the C5 and C3 steps at HEAD
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out/r2h || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2h/c5 -o c5 -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --config c5 > gpurun_out/r2h/c5.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2h/c3 -o c3 -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r2h/c3.log 2>&1
