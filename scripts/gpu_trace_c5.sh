cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && out=gpurun_out/$1 && mkdir -p $out &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/c5 -o c5 -- python3 bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > $out/c5.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/c3 -o c3 -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $out/c3.log 2>&1
