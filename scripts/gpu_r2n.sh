# round 2, call n: batched run walk + compact entries: parity, benches, K2 PMC
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out/r2n || exit 2
echo "== tests" && timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py tests/test_multi_device.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2n/tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/r2n/tests.log; [ $rc -eq 0 ] || exit $rc
b() { local n=$1; shift; echo "== $n" && timeout -k 10 400 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/r2n/$n.json 2> gpurun_out/r2n/$n.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['ms_per_step'], d['phase_ms'])" gpurun_out/r2n/$n.json; }
b c3 && b c5 --config c5 && b c4 --config c4 &&
bash scripts/k2_pmc.sh gpurun_out/r2n/pmc_c3 > gpurun_out/r2n/pmc_c3.log 2>&1 && bash scripts/k2_pmc.sh gpurun_out/r2n/pmc_c5 --config c5 > gpurun_out/r2n/pmc_c5.log 2>&1
