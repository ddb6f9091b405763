# round 2, call ae: per-part K2 latency of an M-device call (row-balanced parts), row-range index off / on
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && out=gpurun_out/r2ae && mkdir -p $out || exit 2
for rg in 0 1; do
  GALAHGPU_INDEX_RANGE=$rg timeout -k 10 300 python3 -u scripts/k2_range_probe.py > $out/c3_r$rg.txt 2>&1 || exit $?
  grep '"M"' $out/c3_r$rg.txt | sed "s/^/c3 range=$rg /"
done
for rg in 0 1; do
  GALAHGPU_INDEX_RANGE=$rg timeout -k 10 400 python3 -u scripts/k2_range_probe.py --genomes 100000 --parts 1,8 --reps 3 > $out/c4_r$rg.txt 2>&1 || exit $?
  grep '"M"' $out/c4_r$rg.txt | sed "s/^/c4 range=$rg /"
done
