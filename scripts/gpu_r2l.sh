# round 2, call l: radix-sorted host merge + threaded ANI: multi-device tests, C4 / C3 / devices 0,0 benches
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out/r2l || exit 2
echo "== tests" && timeout -k 10 600 python3 -u -m pytest tests/test_multi_device.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2l/tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/r2l/tests.log; [ $rc -eq 0 ] || exit $rc
b() { local n=$1; shift; echo "== $n" && timeout -k 10 400 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/r2l/$n.json 2> gpurun_out/r2l/$n.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['ms_per_step'], d['phase_ms'])" gpurun_out/r2l/$n.json; }
b c4 --config c4 && b c3 && b c3_dev00 --devices 0,0
