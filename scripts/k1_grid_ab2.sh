cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out/r3af
for w in 56 112 224 28; do
  for cfg in c3 c5; do
    GALAHGPU_K1_WG_PER_CU=$w timeout -k 10 300 python3 -u bench.py --config $cfg --steps 6 --warmup 2 --no-cpu-baseline --no-files > gpurun_out/r3af/wg${w}_$cfg.log 2>&1 || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/r3af/wg${w}_$cfg.log').read().strip().splitlines()[-1]);print('$w','$cfg',d['ms_per_step'],d['kernel_ms_per_step'])"
  done
done
