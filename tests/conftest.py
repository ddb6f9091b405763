import glob
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLD = os.path.join(ROOT, "tests", "golden")
GOLD_DATA = os.path.join(GOLD, "data")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")


# The default paths at the BASELINE configs and the multi-device path run
# first, so that a GPU run cut short (pytest -x, a box lost mid-run) still
# carries evidence for them; the rest keeps its file order.
_FIRST = ("test_full_size.py", "test_multi_device.py")


def pytest_collection_modifyitems(session, config, items):
    def rank(item):
        name = os.path.basename(str(item.fspath))
        return _FIRST.index(name) if name in _FIRST else len(_FIRST)
    items[:] = [it for _, it in sorted(enumerate(items), key=lambda p: (rank(p[1]), p[0]))]


def golden_names():
    with np.load(os.path.join(GOLD, "sketches_k21_s1000.npz")) as z:
        return [str(x) for x in z["names"]]


def golden_path(name):
    return os.path.join(GOLD_DATA, name + ".gz")


def load_golden_sketches():
    with np.load(os.path.join(GOLD, "sketches_k21_s1000.npz")) as z:
        return [str(x) for x in z["names"]], z["sketches"].copy(), z["lens"].copy()


def load_golden_pairs():
    rows = []
    with open(os.path.join(GOLD, "pairs_k21_s1000.tsv")) as f:
        next(f)
        for line in f:
            i, j, c, t, a = line.split()
            rows.append((int(i), int(j), int(c), int(t), np.float32(a)))
    return rows


@pytest.fixture(scope="session")
def golden():
    names, sk, lens = load_golden_sketches()
    return {"names": names, "sketches": sk, "lens": lens, "pairs": load_golden_pairs(),
            "paths": [golden_path(n) for n in names]}


_XCHECK = []


def xcheck_module():
    """galah_amd bound to libgalahgpu_xcheck.so: the product library plus the
    cross-check pair kernels (GALAHGPU_PAIRS_KERNEL=table|merge, pairs.hip),
    which the product libgalahgpu.so does not carry.  A second module object
    over a second library in the same process (one HIP runtime)."""
    if not _XCHECK:
        import importlib.util
        lib = os.path.join(ROOT, "galah_amd", "lib", "libgalahgpu_xcheck.so")
        spec = importlib.util.spec_from_file_location("galah_amd_xcheck", os.path.join(ROOT, "galah_amd", "__init__.py"))
        mod = importlib.util.module_from_spec(spec)
        old = os.environ.get("GALAHGPU_LIB")
        os.environ["GALAHGPU_LIB"] = lib
        try:
            spec.loader.exec_module(mod)
        finally:
            if old is None:
                os.environ.pop("GALAHGPU_LIB")
            else:
                os.environ["GALAHGPU_LIB"] = old
        _XCHECK.append(mod)
    return _XCHECK[0]


@pytest.fixture(scope="session")
def gpu_ctx():
    import galah_amd
    ctx = galah_amd.Context(k=21, sketch_size=1000, seed=0)
    yield ctx
    ctx.close()
