"""Device vs host gzip inflate on C2-like files (synthetic 3 Mbp genomes,
80 columns, zlib -6), timed through gg_precluster_files; one JSON line.
usage: python scripts/inflate_probe.py [n_files] [steps]"""
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

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
glen = 3000000
d = tempfile.mkdtemp(prefix="gg_inflate_", dir=os.environ.get("TMPDIR") or "/tmp")
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
    out = {"files": n, "gz_bytes": sum(os.path.getsize(p) for p in paths)}
    res = {}
    modes = os.environ.get("PROBE_MODES", "host,device").split(",")
    for mode in modes:
        os.environ["GALAHGPU_INFLATE"] = mode
        with ga.Context(k=21, sketch_size=1000, host_threads=16) as ctx:
            ctx.precluster_files(paths, np.float32(0.95))  # (warm-up: buffers sized for the batches)
            ts = []
            for _ in range(steps):
                t0 = time.perf_counter()
                pairs, _ = ctx.precluster_files(paths, np.float32(0.95))
                ts.append(time.perf_counter() - t0)
            res[mode] = pairs
            out[mode] = {"s": [round(x, 4) for x in ts], "gbases_per_s": round(n * glen / min(ts) / 1e9, 2),
                         "phases": ctx.phase_times(), "inflate_host": ctx.fallbacks()["inflate_host"]}
    if len(res) == 2:
        out["same_pairs"] = bool(np.array_equal(res["host"], res["device"]))
    print(json.dumps(out), flush=True)
finally:
    shutil.rmtree(d, ignore_errors=True)
