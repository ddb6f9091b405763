cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && out=gpurun_out/$1 && mkdir -p $out &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $out/bench_c3.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline > $out/bench_c5.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c4 --steps 2 --no-cpu-baseline > $out/bench_c4.log 2>&1
