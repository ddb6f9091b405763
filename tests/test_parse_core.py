"""The device parser's bit-parallel classification (galah_amd/csrc/parse_core.hpp,
used by parse.hip passes 2 and 3) on the host: classify / roles / run_starts /
packed_codes / place against a byte-by-byte restatement of pack.cpp's byte
rules over 400k random 32-byte chunks (every block limit, line, header and
base state at entry), and compress against its definition
(tests/cpp/test_parse_core.cpp).  The device kernels themselves are checked
end to end against the host packer in test_device_parse.py (GPU)."""
import os
import subprocess

from conftest import ROOT


def test_parse_core_equals_bytewise_rules():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")])
    r = subprocess.run([os.path.join(ROOT, "tests", "cpp", "build", "test_parse_core")], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok 400000")
