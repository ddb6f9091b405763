# round 2, call b: dual-issue probe + its PMC pass, full-size parity tests, K1 PMC at HEAD
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out/r2b &&
timeout -k 10 120 ./scripts/ubench_dual 8 > gpurun_out/r2b/dual8.txt 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/r2b/pmc_dual -o dual -- ./scripts/ubench_dual 8 > gpurun_out/r2b/pmc_dual.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_full_size.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r2b/full_size.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-include-regex sketch_candidates --output-format csv -d gpurun_out/r2b/pmc_k1 -o k1 -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r2b/pmc_k1.log 2>&1
