"""Per-call wall time and per-kernel-class HIP-event ms of repeated
gg_precluster_files calls on C2-like gzip files (the files-leg outliers:
which class grows in a slow call).  Usage: python scripts/ingest_var.py [files] [calls]"""
import concurrent.futures as cf
import json
import os
import shutil
import sys
import tempfile
import time
import zlib

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import galah_amd as ga  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 8
glen = 3000000
d = tempfile.mkdtemp(prefix="gg_var_", dir=os.environ.get("TMPDIR") or "/tmp")
try:
    def write(g):
        rng = np.random.default_rng(g)
        seq = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, glen)]
        body = np.concatenate([seq.reshape(-1, 80), np.full((glen // 80, 1), 10, np.uint8)], axis=1).tobytes()
        c = zlib.compressobj(6, zlib.DEFLATED, 31)
        p = os.path.join(d, "g%05d.fna.gz" % g)
        with open(p, "wb") as f:
            f.write(c.compress(b">g%d\n" % g + body) + c.flush())
        return p

    with cf.ThreadPoolExecutor(16) as ex:
        paths = list(ex.map(write, range(n)))
    with ga.Context(k=21, sketch_size=1000, seed=0, host_threads=16) as ctx:
        ctx.precluster_files(paths, 0.95)
        for c in range(calls):
            ctx.timing_enable(True)
            t1 = time.perf_counter()
            ctx.precluster_files(paths, 0.95)
            w = time.perf_counter() - t1
            ks = {name: round(ctx.timing_read(k)["ms"], 2) for name, k in ga.INGEST_KERNELS.items()}
            ks["k1"] = round(ctx.timing_read(ga.KERNEL_SKETCH)["ms"], 2)
            ctx.timing_enable(False)
            print(json.dumps({"call": c, "s": round(w, 4), "ms": ks, "phases": {k: round(v, 2) for k, v in ctx.phase_times().items()}}), flush=True)
finally:
    shutil.rmtree(d, ignore_errors=True)
