# K1 change: parity (sketch tests incl. every k in 5..32 tested and the full-size configs), bench, PMC at HEAD
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && out=gpurun_out/$1 && mkdir -p $out &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py tests/test_multi_device.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/bench.log 2>&1 &&
bash scripts/pmc_head.sh $out/pmc > $out/pmc.log 2>&1
