"""Ingest probe: write synthetic FASTA files (plain and
gzip) to a scratch directory, then time gg_pack_files (host: read, gunzip,
parse, 2-bit pack) and the whole gg_precluster_files path on them.

    python scripts/ingest_probe.py [--files 256] [--len 3000000] [--threads 16]
"""
import argparse
import gzip
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import galah_amd as ga  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=256)
    ap.add_argument("--len", type=int, default=3000000)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--dir", default=None)
    a = ap.parse_args()
    d = a.dir or tempfile.mkdtemp(prefix="gg_ingest_")
    os.makedirs(d, exist_ok=True)
    rng = np.random.default_rng(5)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    paths = {"plain": [], "gz": []}
    t0 = time.perf_counter()
    root = acgt[rng.integers(0, 4, a.len)]
    for i in range(a.files):
        seq = root.copy()
        mut = rng.random(a.len) < 0.02 * (i % 4)
        seq[mut] = acgt[rng.integers(0, 4, int(mut.sum()))]
        lines = seq[: a.len // 80 * 80].reshape(-1, 80)
        body = b"\n".join(bytes(x) for x in lines)
        data = b">genome_%d synthetic\n" % i + body + b"\n"
        for kind in ("plain", "gz"):
            p = os.path.join(d, "g%05d.fna%s" % (i, ".gz" if kind == "gz" else ""))
            if kind == "gz":
                with gzip.open(p, "wb", compresslevel=6) as f:
                    f.write(data)
            else:
                with open(p, "wb") as f:
                    f.write(data)
            paths[kind].append(p)
    gen_s = time.perf_counter() - t0
    out = {"files": a.files, "genome_len": a.len, "threads": a.threads, "generate_s": round(gen_s, 2)}
    bases = a.files * (a.len // 80 * 80)
    for kind in ("plain", "gz"):
        t0 = time.perf_counter()
        pk = ga.pack_files(paths[kind], threads=a.threads)
        t = time.perf_counter() - t0
        out["pack_%s_s" % kind] = round(t, 3)
        out["pack_%s_gbases_per_s" % kind] = round(bases / t / 1e9, 3)
        pk.free()
    with ga.Context(k=21, sketch_size=1000) as ctx:
        ctx.precluster_files(paths["gz"][:8], ga.parse_percentage(95))  # warm
        t0 = time.perf_counter()
        pairs, ani = ctx.precluster_files(paths["gz"], ga.parse_percentage(95))
        out["precluster_files_gz_s"] = round(time.perf_counter() - t0, 3)
        out["pairs_found"] = int(len(pairs))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
