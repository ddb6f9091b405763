"""The streamed ingest (gg::PackStream) behind gg_precluster_files /
gg_sketch_files, on CPU: every genome equals gg_pack_files' packing for
1-7 packing threads, 1-4 consumers and budgets down to one byte (no
deadlock), the lowest failing file is the one reported, and an abort wakes
a consumer waiting for a genome nobody will pack."""
import os
import subprocess

from conftest import ROOT, golden_path, golden_names

BIN = os.path.join(ROOT, "tests", "cpp", "build", "test_pack_stream")


def test_pack_stream():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")])
    paths = [golden_path(n) for n in golden_names()]
    r = subprocess.run([BIN] + paths, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "ok"
