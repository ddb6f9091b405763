cd "${GRAFT_REPO_ROOT}" && export TMPDIR=/tmp && mkdir -p gpurun_out/r4v && \
timeout -k 10 300 python3 -u -m pytest tests/test_inflate.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4v/head.log 2>&1; echo "head rc=$?"; \
GALAHGPU_LIB=galah_amd/lib_ab/libgalahgpu.so timeout -k 10 300 python3 -u -m pytest tests/test_inflate.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4v/ab.log 2>&1; echo "ab rc=$?"
