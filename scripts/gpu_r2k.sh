# round 2, call k: 32-bit-key index build: GPU suite, C3/C5/C4 benches, kernel trace at C5
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out/r2k || exit 2
echo "== tests" && timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2k/tests.log 2>&1; rc=$?; tail -n 5 gpurun_out/r2k/tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in c3 c5 c4; do
  echo "== $cfg" && timeout -k 10 400 python3 -u bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r2k/$cfg.json 2> gpurun_out/r2k/$cfg.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['ms_per_step'], d['phase_ms'])" gpurun_out/r2k/$cfg.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2k/trace_c5 -o c5 -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --config c5 > gpurun_out/r2k/trace_c5.log 2>&1
