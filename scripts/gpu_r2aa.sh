# round 2, call aa: file-ingest probe at HEAD incl. the sketch cache (cold / warm)
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && out=gpurun_out/r2aa && mkdir -p $out || exit 2
timeout -k 10 600 python3 -u scripts/ingest_probe.py --files 256 --threads 16 --dir /tmp/gg_ingest > $out/ingest.json 2> $out/ingest.err; rc=$?
tail -c 1500 $out/ingest.json; exit $rc
