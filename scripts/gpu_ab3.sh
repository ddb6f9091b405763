# A/B/C of K1 variants: lib (queue), lib_alt (queue, 7 waves/SIMD), lib_alt2 (no queue)
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && out=gpurun_out/$1 && mkdir -p $out &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py -x -q --timeout 300 --timeout-method thread > $out/tests_main.log 2>&1 &&
GALAHGPU_LIB=galah_amd/lib_alt/libgalahgpu.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "sketch or edge or other_k or synthetic" --timeout 300 --timeout-method thread > $out/tests_alt.log 2>&1 &&
for r in 1 2; do
  for v in lib lib_alt lib_alt2; do
    for c in c3 c5; do
      GALAHGPU_LIB=galah_amd/$v/libgalahgpu.so timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $out/bench_${v}_${c}_$r.log 2>&1 || exit 1
    done
  done
done
