# round 2, call ak: the GPU suite with the row-range index off (GALAHGPU_INDEX_RANGE=0), and the
# multi-device tests with the gate kernel forced (GALAHGPU_PAIRS_KERNEL=gate)
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && out=gpurun_out/r2ak && mkdir -p $out || exit 2
GALAHGPU_INDEX_RANGE=0 timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $out/tests_range0.log 2>&1; rc=$?; tail -n 1 $out/tests_range0.log; [ $rc -eq 0 ] || exit $rc
GALAHGPU_PAIRS_KERNEL=gate timeout -k 10 600 python3 -u -m pytest tests/test_multi_device.py -q --timeout 300 --timeout-method thread > $out/tests_multi_gate.log 2>&1; rc=$?; tail -n 1 $out/tests_multi_gate.log; exit $rc
