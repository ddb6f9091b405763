# round 2, call p: device-side FASTA parsing: tests, ingest probe with both parse modes
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out/r2p || exit 2
echo "== tests" && timeout -k 10 900 python3 -u -m pytest tests/test_device_parse.py tests/test_multi_device.py tests/test_sketch_cache.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2p/tests.log 2>&1; rc=$?; tail -n 15 gpurun_out/r2p/tests.log; [ $rc -eq 0 ] || exit $rc
echo "== ingest device" && GALAHGPU_PARSE=device timeout -k 10 900 python3 -u scripts/ingest_probe.py --files 256 --len 3000000 --threads 16 --repeat 1,4 --dir /tmp/gg_ingest > gpurun_out/r2p/ingest_device.json 2> gpurun_out/r2p/ingest_device.err || exit $?
cat gpurun_out/r2p/ingest_device.json
echo "== ingest host" && GALAHGPU_PARSE=host timeout -k 10 900 python3 -u scripts/ingest_probe.py --files 256 --len 3000000 --threads 16 --repeat 1 --dir /tmp/gg_ingest > gpurun_out/r2p/ingest_host.json 2> gpurun_out/r2p/ingest_host.err; rc=$?
cat gpurun_out/r2p/ingest_host.json; rm -rf /tmp/gg_ingest; exit $rc
