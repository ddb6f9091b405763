"""Interleaved A/B of device-inflate settings on C2-like gzip files: one
context, calls alternating between the settings (environment knobs read per
call), per-kernel-class HIP-event ms of each call (one lane, no overlap:
GALAHGPU_GZ_LANES=1) and the wall time of default-lane calls.

usage: python scripts/ingest_ab.py FILES CALLS 'NAME:K=V,K=V' ['NAME:K=V' ...]
  e.g. python scripts/ingest_ab.py 400 4 'tight:' 'full:GALAHGPU_GZ_TIGHT=0'
One JSON line per setting: medians over the calls."""
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

n = int(sys.argv[1])
calls = int(sys.argv[2])
settings = []
for spec in sys.argv[3:]:
    name, _, kv = spec.partition(":")
    env = dict(x.split("=", 1) for x in kv.split(",") if x)
    settings.append((name, env))
fmt = os.environ.get("AB_FORMAT", "gz")
glen = 3000000
d = tempfile.mkdtemp(prefix="gg_ab_", dir=os.environ.get("TMPDIR") or "/tmp")


def bgzf(data, level=6, block=65280):
    out = []
    for i in range(0, max(len(data), 1), block):
        chunk = data[i:i + block]
        c = zlib.compressobj(level, zlib.DEFLATED, -15)
        body = c.compress(chunk) + c.flush()
        hdr = bytes([0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 66, 67, 2, 0]) + (len(body) + 25).to_bytes(2, "little")
        out.append(hdr + body + zlib.crc32(chunk).to_bytes(4, "little") + len(chunk).to_bytes(4, "little"))
    out.append(bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000"))
    return b"".join(out)


try:
    def write(g):
        rng = np.random.default_rng(g)
        seq = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, glen)]
        body = np.concatenate([seq.reshape(-1, 80), np.full((glen // 80, 1), 10, np.uint8)], axis=1).tobytes()
        text = b">g%d\n" % g + body
        p = os.path.join(d, "g%05d.fna.gz" % g)
        with open(p, "wb") as f:
            if fmt == "bgzf":
                f.write(bgzf(text))
            else:
                c = zlib.compressobj(6, zlib.DEFLATED, 31)
                f.write(c.compress(text) + c.flush())
        return p

    with cf.ThreadPoolExecutor(16) as ex:
        paths = list(ex.map(write, range(n)))
    import re

    def regrows(ctx):
        m = re.search(r"scratch regrows (\d+) \(([0-9.]+) ms\)", ctx.info_line())
        return (int(m.group(1)), float(m.group(2))) if m else (0, 0.0)

    res = {name: {"wall": [], "lane1_wall": [], "ms": {}, "regrow": []} for name, _ in settings}
    with ga.Context(k=21, sketch_size=1000, seed=0, host_threads=16) as ctx:
        for name, env in settings:  # (warm-up: buffers sized for each setting)
            os.environ.update(env)
            ctx.precluster_files(paths, 0.95)
            for k in env:
                os.environ.pop(k, None)
        for c in range(calls):
            for name, env in settings:
                os.environ.update(env)
                r0 = regrows(ctx)
                t1 = time.perf_counter()
                ctx.precluster_files(paths, 0.95)
                res[name]["wall"].append(time.perf_counter() - t1)
                r1 = regrows(ctx)
                res[name]["regrow"].append([r1[0] - r0[0], round(r1[1] - r0[1], 2)])
                os.environ["GALAHGPU_GZ_LANES"] = "1"
                ctx.timing_enable(True)
                t1 = time.perf_counter()
                ctx.precluster_files(paths, 0.95)
                res[name]["lane1_wall"].append(time.perf_counter() - t1)
                for kn, k in list(ga.INGEST_KERNELS.items()) + [("k1", ga.KERNEL_SKETCH)]:
                    res[name]["ms"].setdefault(kn, []).append(ctx.timing_read(k)["ms"])
                ctx.timing_enable(False)
                os.environ.pop("GALAHGPU_GZ_LANES")
                for k in env:
                    os.environ.pop(k, None)
        info = ctx.info_line()
    for name, _ in settings:
        r = res[name]
        print(json.dumps({"setting": name, "files": n, "format": fmt, "calls": calls,
                          "wall_median_s": round(float(np.median(r["wall"])), 4),
                          "wall_s": [round(x, 4) for x in r["wall"]],
                          "regrows_per_call": r["regrow"],
                          "gbases_per_s": round(n * glen / float(np.median(r["wall"])) / 1e9, 2),
                          "lane1_wall_median_s": round(float(np.median(r["lane1_wall"])), 4),
                          "kernel_ms_median": {k: round(float(np.median(v)), 3) for k, v in r["ms"].items()}}),
              flush=True)
    print(json.dumps({"info_line": info}), flush=True)
finally:
    shutil.rmtree(d, ignore_errors=True)
