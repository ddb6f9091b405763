# round 2, call w: K1 A/B at C3 and C5 (lib_g00 = previous HEAD; lib_gB = MULHI +
# K2A128; lib = + INNER), then the full GPU suite + smoke on lib, then the PMC
# passes at HEAD for the issue model
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && out=gpurun_out/r2w && mkdir -p $out || exit 2
for r in 1 2; do
  for cfg in c3 c5; do
    for v in lib_g00 lib_gB lib; do
      GALAHGPU_LIB=galah_amd/$v/libgalahgpu.so timeout -k 10 300 python3 -u bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline > $out/bench_${cfg}_${v}_$r.json 2> $out/bench_${cfg}_${v}_$r.err || exit $?
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['phase_ms'])" $out/bench_${cfg}_${v}_$r.json "$cfg $v"
    done
  done
done
echo "== tests"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -n 2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
tail -n 1 $out/smoke.log
echo "== pmc"
bash scripts/pmc_head.sh $out/pmc > $out/pmc.log 2>&1; rc=$?; tail -n 3 $out/pmc.log; exit $rc
