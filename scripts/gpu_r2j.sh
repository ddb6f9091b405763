# round 2, call j: PMC passes at HEAD (issue model refresh), ingest probe (streamed gg_precluster_files vs host decode, peak RSS), C4 bench
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out/r2j || exit 2
echo "== pmc" && bash scripts/pmc_head.sh gpurun_out/r2j/pmc > gpurun_out/r2j/pmc.log 2>&1; rc=$?; tail -n 3 gpurun_out/r2j/pmc.log; [ $rc -eq 0 ] || exit $rc
echo "== c4" && timeout -k 10 400 python3 -u bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r2j/c4.json 2> gpurun_out/r2j/c4.err || exit $?
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['phase_ms'])" gpurun_out/r2j/c4.json
echo "== ingest" && timeout -k 10 900 python3 -u scripts/ingest_probe.py --files 256 --len 3000000 --threads 16 --repeat 1,4 --dir /tmp/gg_ingest > gpurun_out/r2j/ingest.json 2> gpurun_out/r2j/ingest.err; rc=$?; cat gpurun_out/r2j/ingest.json; rm -rf /tmp/gg_ingest; exit $rc
