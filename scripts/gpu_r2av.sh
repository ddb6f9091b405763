# round 2, call av: the new mixed-length s=10000 multi-device test, then the whole multi-device file
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && out=gpurun_out/r2av && mkdir -p $out || exit 2
timeout -k 10 600 python3 -u -m pytest tests/test_multi_device.py -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -n 14 $out/tests.log; exit $rc
