# round 2, call au: K1 workgroups per CU re-checked at HEAD (GALAHGPU_K1_WG_PER_CU 56 / 112 / 224), C3
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && out=gpurun_out/r2au && mkdir -p $out || exit 2
for r in 1 2; do
  for w in 56 112 224; do
    GALAHGPU_K1_WG_PER_CU=$w timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $out/bench_w${w}_$r.json 2> $out/bench_w${w}_$r.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['roofline']['avg_launch_ms'])" $out/bench_w${w}_$r.json "wg/cu=$w"
  done
done
