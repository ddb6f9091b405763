# round 2, call r: the driver's multi-rank launch shape on one GPU (rank 0 drives repeated-ordinal
# shards, the other ranks join the gloo barriers) and the sharded path's overhead at 1/2/4/8 shards
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out/r2r || exit 2
echo "== torchrun 2 ranks" && timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --devices 0,0 --no-cpu-baseline > gpurun_out/r2r/torchrun2.json 2> gpurun_out/r2r/torchrun2.err || exit $?
grep '^{' gpurun_out/r2r/torchrun2.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['n_gpus'], d['value'], d['ms_per_step'], d['phase_ms'])"
for d in 0,0,0,0 0,0,0,0,0,0,0,0; do
  echo "== devices $d" && timeout -k 10 600 python3 -u bench.py --steps 3 --warmup 1 --devices $d --no-cpu-baseline > gpurun_out/r2r/dev_$d.json 2> gpurun_out/r2r/dev_$d.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['config']['parallelism'], d['value'], d['ms_per_step'], d['phase_ms'])" gpurun_out/r2r/dev_$d.json
done
