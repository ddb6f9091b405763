# round 2, call af: full GPU suite + smoke + C3 bench at HEAD (row-range index in)
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && out=gpurun_out/r2af && mkdir -p $out || exit 2
echo "== tests" && timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -n 3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke" && timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
tail -n 1 $out/smoke.log
echo "== bench" && timeout -k 10 600 python3 -u bench.py --no-cpu-baseline > $out/bench_c3.json 2> $out/bench_c3.err || exit $?
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['steps'])" $out/bench_c3.json
