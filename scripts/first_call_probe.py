"""Why is the first timed gg_precluster_files call after a warm-up slower
(bench files leg: 0.0585 s against a median of 0.0489)?  One context, a
warm-up call, then CALLS timed calls, in three runs: right after the
warm-up, after an idle pause (GPU clocks fall back), and with a second
warm-up call.  usage: python scripts/first_call_probe.py FILES CALLS"""
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

n, calls = int(sys.argv[1]), int(sys.argv[2])
glen = 3000000
d = tempfile.mkdtemp(prefix="gg_first_", dir=os.environ.get("TMPDIR") or "/tmp")
try:
    def write(g):
        rng = np.random.default_rng(g)
        seq = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, glen)]
        body = np.concatenate([seq.reshape(-1, 80), np.full((glen // 80, 1), 10, np.uint8)], axis=1).tobytes()
        p = os.path.join(d, "g%05d.fna.gz" % g)
        c = zlib.compressobj(6, zlib.DEFLATED, 31)
        with open(p, "wb") as f:
            f.write(c.compress(b">g%d\n" % g + body) + c.flush())
        return p

    with cf.ThreadPoolExecutor(16) as ex:
        paths = list(ex.map(write, range(n)))
    for mode in ("after_warmup", "after_idle_2s", "two_warmups", "after_warmup"):
        with ga.Context(k=21, sketch_size=1000, seed=0, host_threads=16) as ctx:
            ctx.precluster_files(paths, 0.95)
            if mode == "two_warmups":
                ctx.precluster_files(paths, 0.95)
            if mode == "after_idle_2s":
                time.sleep(2.0)
            ts, ph = [], []
            for _ in range(calls):
                t0 = time.perf_counter()
                ctx.precluster_files(paths, 0.95)
                ts.append(round(time.perf_counter() - t0, 4))
                ph.append({k: round(v, 1) for k, v in ctx.phase_times().items()})
            print(json.dumps({"mode": mode, "s": ts, "phases_ms": ph[:2]}), flush=True)
finally:
    shutil.rmtree(d, ignore_errors=True)
