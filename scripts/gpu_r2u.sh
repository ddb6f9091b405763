# round 2, call u: VALU issue costs of SGPR-sourced VOP3 forms, 64-bit min forms
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out/r2u || exit 2
timeout -k 10 240 ./scripts/ubench_dual 8 > gpurun_out/r2u/dual8.txt 2>&1
