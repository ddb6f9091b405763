# round 2, call i: parallel run index in sketch_core: full GPU suite, host stage profile at C5, C5/C3 benches
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out/r2i || exit 2
echo "== tests" && timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2i/tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/r2i/tests.log; [ $rc -eq 0 ] || exit $rc
echo "== c5 host profile" && GALAHGPU_HOST_PROFILE=1 timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --config c5 > gpurun_out/r2i/c5.json 2> gpurun_out/r2i/c5.err || exit $?
tail -n 7 gpurun_out/r2i/c5.err
echo "== c3" && timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r2i/c3.json 2> gpurun_out/r2i/c3.err || exit $?
for f in c5 c3; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step'], d['phase_ms'], d['roofline']['kernels'][0]['avg_ms'])" gpurun_out/r2i/$f.json; done
