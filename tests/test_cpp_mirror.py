"""The C++ mirror of the reference interface (include/galah_finch.hpp),
compiled against libgalahgpu.so: cache / parse tests on CPU, the
src/finch.rs:85-107 known answer on the GPU."""
import os
import subprocess

import pytest

from conftest import GOLD_DATA, ROOT

BIN = os.path.join(ROOT, "tests", "cpp", "build", "test_finch_mirror")


@pytest.fixture(scope="module")
def binary():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")])
    return BIN


def test_cpp_mirror_host_parts(binary):
    r = subprocess.run([binary], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


@pytest.mark.gpu
def test_cpp_mirror_finch_hello_world(binary):
    r = subprocess.run([binary, GOLD_DATA], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "ok"
