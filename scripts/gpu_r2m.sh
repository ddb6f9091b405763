# round 2, call m: PMC passes for K2 (and K1 as the traffic calibration) at C3 and C5
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out/r2m || exit 2
bash scripts/k2_pmc.sh gpurun_out/r2m/c3 && bash scripts/k2_pmc.sh gpurun_out/r2m/c5 --config c5
