# round 2, call an: pure host gzip decode (libdeflate, no parse or pack) of the ingest probe's files on
# 16 and 1 threads, beside the ingest probe itself (gg_pack_files / gg_precluster_files on the same files)
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && out=gpurun_out/r2an && mkdir -p $out || exit 2
timeout -k 10 600 python3 -u scripts/ingest_probe.py --files 256 --threads 16 --dir /tmp/gg_ingest > $out/ingest.json 2> $out/ingest.err || exit $?
for t in 16 1; do timeout -k 10 120 ./scripts/gunzip_probe $t /tmp/gg_ingest/*.fna.gz > $out/gunzip_t$t.json 2>&1 || exit $?; cat $out/gunzip_t$t.json; done
python3 -c "import json; d=json.load(open('$out/ingest.json')); print('pack_gz_s', d['pack_gz_s'], 'precluster_files_gz_s', d['precluster_files_gz_s'])"
