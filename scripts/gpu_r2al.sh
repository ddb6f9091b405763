# round 2, call al: C2 (1k genomes) bench, C5 K1 PMC pass (VALU / LDS per wave-k-mer vs C3),
# and the driver's 2-rank launch shape rehearsed on one GPU (--devices 0,0)
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && out=gpurun_out/r2al && mkdir -p $out || exit 2
timeout -k 10 300 python3 -u bench.py --config c2 --no-cpu-baseline > $out/bench_c2.json 2> $out/bench_c2.err || exit $?
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c2', d['value'], d['ms_per_step'], d['phase_ms'])" $out/bench_c2.json
timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-include-regex sketch_candidates --output-format csv -d $out/pmc_c5 -o p1 -- python3 bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline > $out/pmc_c5.log 2>&1 || exit $?
timeout -k 10 400 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --devices 0,0 --steps 5 --warmup 1 --no-cpu-baseline > $out/torchrun2.json 2> $out/torchrun2.err || exit $?
tail -n 1 $out/torchrun2.json | cut -c1-300
