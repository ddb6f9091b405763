# round 2, call ao: host packer partial-chunk steps -- ingest probe at 60- and 80-column lines with the
# new packer (lib) and the previous one (lib_g00), and pure gzip decode of the same files
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && out=gpurun_out/r2ao && mkdir -p $out || exit 2
for w in 60 80; do
  timeout -k 10 600 python3 -u scripts/ingest_probe.py --files 256 --threads 16 --line $w --dir /tmp/gg_ingest_$w --repeat 1 > $out/ingest_${w}_new.json 2> $out/ingest_${w}_new.err || exit $?
  GALAHGPU_LIB=galah_amd/lib_g00/libgalahgpu.so timeout -k 10 600 python3 -u scripts/ingest_probe.py --files 256 --threads 16 --line $w --dir /tmp/gg_ingest_$w --repeat 1 --reuse > $out/ingest_${w}_old.json 2> $out/ingest_${w}_old.err || exit $?
  timeout -k 10 120 ./scripts/gunzip_probe 16 /tmp/gg_ingest_$w/*.fna.gz > $out/gunzip_${w}.json 2>&1 || exit $?
  for v in new old; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'pack_plain', d['pack_plain_gbases_per_s'], 'pack_gz', d['pack_gz_gbases_per_s'], 'files_gz_s', d['precluster_files_gz_s'])" $out/ingest_${w}_$v.json "$w $v"; done
  cat $out/gunzip_${w}.json
done
