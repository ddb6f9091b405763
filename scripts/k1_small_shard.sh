cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r03_w
for g in 1250 2500 5000; do
  timeout -k 10 200 python3 -u bench.py --genomes $g --steps 30 --warmup 5 --no-cpu-baseline --no-files > gpurun_out/r03_w/g$g.log 2>&1 || exit $?
  tail -n 1 gpurun_out/r03_w/g$g.log > gpurun_out/r03_w/g$g.json
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03_w/prof -o g1250 -- python3 -u bench.py --genomes 1250 --steps 30 --warmup 5 --no-cpu-baseline --no-files > gpurun_out/r03_w/prof.log 2>&1
