# round 2, call x: where C5's non-K1 step time goes -- host stage times of
# sketch_core (GALAHGPU_HOST_PROFILE) and a kernel + memory-copy trace
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && out=gpurun_out/r2x && mkdir -p $out || exit 2
export GALAHGPU_HOST_PROFILE=1
timeout -k 10 300 python3 -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > $out/c5.json 2> $out/c5_host.err || exit $?
timeout -k 10 300 python3 -u bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline > $out/c3.json 2> $out/c3_host.err || exit $?
unset GALAHGPU_HOST_PROFILE
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $out/trace -o c5 -- python3 bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > $out/trace.log 2>&1
