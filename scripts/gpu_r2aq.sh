# round 2, call aq: AVX2 packer steps vs SSE4.1 (GALAHGPU_NO_AVX2=1), 60 and 80 columns, files generated first
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && out=gpurun_out/r2aq && mkdir -p $out || exit 2
for w in 60 80; do
  timeout -k 10 600 python3 -u scripts/ingest_probe.py --files 256 --threads 16 --line $w --dir /tmp/gg_ingest_$w --repeat 1 > $out/gen_$w.json 2> $out/gen_$w.err || exit $?
done
sync
for r in 1 2; do
  for w in 60 80; do
    for v in sse avx2; do
      if [ $v = sse ]; then export GALAHGPU_NO_AVX2=1; else unset GALAHGPU_NO_AVX2; fi
      timeout -k 10 600 python3 -u scripts/ingest_probe.py --files 256 --threads 16 --line $w --dir /tmp/gg_ingest_$w --repeat 1 --reuse > $out/ingest_${w}_${v}_$r.json 2> $out/ingest_${w}_${v}_$r.err || exit $?
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'pack_plain', d['pack_plain_gbases_per_s'], 'pack_gz', d['pack_gz_gbases_per_s'], 'files_gz_s', d['precluster_files_gz_s'])" $out/ingest_${w}_${v}_$r.json "$w $v $r"
    done
  done
done
unset GALAHGPU_NO_AVX2
for t in 1; do timeout -k 10 120 ./scripts/gunzip_probe $t /tmp/gg_ingest_60/*.fna.gz > $out/gunzip_60_t$t.json 2>&1; cat $out/gunzip_60_t$t.json; done
