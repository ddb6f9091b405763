cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out/r2a &&
timeout -k 10 90 ./scripts/ubench_valu2 8 > gpurun_out/r2a/ubench8.txt 2>&1 &&
timeout -k 10 90 ./scripts/ubench_valu2 4 > gpurun_out/r2a/ubench4.txt 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --output-format csv -d gpurun_out/r2a/pmc_ub -o ub -- ./scripts/ubench_valu2 8 > gpurun_out/r2a/pmc_ub.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2a/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r2a/bench.log 2>&1 &&
(timeout -k 10 60 rocprofv3 -L > gpurun_out/r2a/counters.txt 2>&1; echo done)
