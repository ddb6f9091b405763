"""The files leg (1,000 C2-like gzip files through gg_precluster_files) timed
in three process states: fresh; beside a 10 GB torch tensor; beside a second
context that ran the C3 sketch + pairs step (its scratch held).  usage:
python scripts/files_state_ab.py [n]"""
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
d = tempfile.mkdtemp(prefix="gg_fst_", dir=os.environ.get("TMPDIR") or "/tmp")


def write(g):
    seq = np.frombuffer(b"ACGT", np.uint8)[np.random.default_rng(g).integers(0, 4, glen)]
    body = np.concatenate([seq.reshape(-1, 80), np.full((glen // 80, 1), 10, np.uint8)], axis=1).tobytes()
    c = zlib.compressobj(6, zlib.DEFLATED, 31)
    p = os.path.join(d, "g%05d.fna.gz" % g)
    with open(p, "wb") as f:
        f.write(c.compress(b">g%d\n" % g + body) + c.flush())
    return p


def timed(paths):
    with ga.Context(k=21, sketch_size=1000, host_threads=16) as ctx:
        ctx.precluster_files(paths, np.float32(0.95))
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            ctx.precluster_files(paths, np.float32(0.95))
            ts.append(round(time.perf_counter() - t0, 4))
    return ts


try:
    with cf.ThreadPoolExecutor(16) as ex:
        paths = list(ex.map(write, range(n)))
    out = {"fresh": timed(paths)}
    print("fresh", out["fresh"], flush=True)
    big = torch.empty(10 * 2**30, dtype=torch.uint8, device="cuda")
    big.fill_(1)
    torch.cuda.synchronize()
    out["torch_10GB"] = timed(paths)
    print("torch_10GB", out["torch_10GB"], flush=True)
    del big
    torch.cuda.empty_cache()
    N, L = 10000, 3000000
    main = ga.Context(k=21, sketch_size=1000, seed=0)
    dw = torch.empty(N * L // 16, dtype=torch.int32, device="cuda")
    runs = main.synth_device(N, L, 10, 0.05, 1, dw)
    shards = [(dw, ga.device_runs(runs, "cuda"), N)]
    main.precluster_shards(shards, np.float32(0.95))
    torch.cuda.synchronize()
    out["beside_c3_ctx"] = timed(paths)
    print("beside_c3_ctx", out["beside_c3_ctx"], flush=True)
    main.close()
    del dw, shards
    torch.cuda.empty_cache()
    out["after_close"] = timed(paths)
    print("after_close", out["after_close"], flush=True)
    print(json.dumps(out))
finally:
    shutil.rmtree(d, ignore_errors=True)
