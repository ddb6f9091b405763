"""A/B of the gzip files leg: the bench's clustered C2 files (synth_device,
as bench.py files_leg writes them) against inflate_probe's independent random
genomes, each timed in this fresh process.  usage: python scripts/files_data_ab.py [n]"""
import concurrent.futures as cf
import json
import os
import shutil
import sys
import tempfile
import time
import zlib

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import galah_amd as ga  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
glen = 3000000
d = tempfile.mkdtemp(prefix="gg_fab_", dir=os.environ.get("TMPDIR") or "/tmp")
try:
    with ga.Context(k=21, sketch_size=1000, seed=0) as ctx:
        dw = torch.empty(n * glen // 16, dtype=torch.int32, device="cuda")
        ctx.synth_device(n, glen, 10, 0.05, 1, dw)
        torch.cuda.synchronize()
        words = dw.cpu().numpy().view(np.uint32)
        del dw
    acgt = np.frombuffer(b"ACGT", np.uint8)
    shifts = (np.uint32(30) - 2 * np.arange(16, dtype=np.uint32))[None, :]
    nl = np.full((glen // 80, 1), 10, np.uint8)

    def write(args):
        kind, g = args
        if kind == "synth":
            w = words[g * glen // 16:(g + 1) * glen // 16]
            seq = acgt[((w[:, None] >> shifts) & np.uint32(3)).reshape(-1)]
            head = b">genome_%d synthetic C2\n" % g
        else:
            seq = acgt[np.random.default_rng(g).integers(0, 4, glen)]
            head = b">g%d\n" % g
        body = np.concatenate([seq.reshape(-1, 80), nl], axis=1).tobytes()
        c = zlib.compressobj(6, zlib.DEFLATED, 31)
        p = os.path.join(d, "%s%05d.fna.gz" % (kind, g))
        with open(p, "wb") as f:
            f.write(c.compress(head + body) + c.flush())
        return p

    out = {}
    for kind in ("synth", "random", "synth"):
        with cf.ThreadPoolExecutor(16) as ex:
            paths = list(ex.map(write, [(kind, g) for g in range(n)]))
        with ga.Context(k=21, sketch_size=1000, host_threads=16) as ctx:
            ctx.precluster_files(paths, np.float32(0.95))
            ts = []
            for _ in range(3):
                t0 = time.perf_counter()
                ctx.precluster_files(paths, np.float32(0.95))
                ts.append(round(time.perf_counter() - t0, 4))
        out.setdefault(kind, []).append({"s": ts, "gz_bytes": sum(os.path.getsize(p) for p in paths)})
        for p in paths:
            os.remove(p)
        print(kind, ts, flush=True)
    print(json.dumps(out))
finally:
    shutil.rmtree(d, ignore_errors=True)
