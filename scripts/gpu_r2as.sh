# round 2, call as: C5 host stages of sketch_core (GALAHGPU_HOST_PROFILE) after fusing the index passes,
# with the run-table tests; and a kernel + copy trace
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && out=gpurun_out/r2as && mkdir -p $out || exit 2
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -n 1 $out/tests.log; [ $rc -eq 0 ] || exit $rc
GALAHGPU_HOST_PROFILE=1 timeout -k 10 300 python3 -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $out/c5.json 2> $out/c5_host.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $out/trace -o c5 -- python3 bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > $out/trace.log 2>&1
tail -n 14 $out/c5_host.err
python3 -c "import json; d=json.load(open('$out/c5.json')); print(d['ms_per_step'], d['phase_ms'])"
