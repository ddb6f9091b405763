# round 2, call q: device vs host parse at 16 and 1 ingest threads
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out/r2q || exit 2
for t in 16 1; do for mode in device host; do
  echo "== $mode t=$t" && GALAHGPU_PARSE=$mode timeout -k 10 600 python3 -u scripts/ingest_probe.py --files 128 --len 3000000 --threads $t --repeat 1 --dir /tmp/gg_ingest > gpurun_out/r2q/ingest_${mode}_t$t.json 2> gpurun_out/r2q/ingest_${mode}_t$t.err || exit $?
  cat gpurun_out/r2q/ingest_${mode}_t$t.json
done; done
rm -rf /tmp/gg_ingest
