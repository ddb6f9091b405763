"""Ingest probe: write synthetic FASTA files (plain and
gzip) to a scratch directory, then time gg_pack_files (host: read, gunzip,
parse, 2-bit pack) and the whole gg_precluster_files path on them (streamed:
bounded batches of packed files overlap decode with H2D and K1).  Each
gg_precluster_files run happens in a fresh process so its peak RSS can be
read; --repeat lists path-list multiplicities (the same files listed R
times: galah sketches duplicate paths twice) to show that peak RSS does not
grow with the number of genomes.

    python scripts/ingest_probe.py [--files 256] [--len 3000000] [--threads 16] [--repeat 1,4]
"""
import argparse
import gzip
import json
import os
import subprocess
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
    ap.add_argument("--repeat", default="1,4")
    ap.add_argument("--line", type=int, default=80, help="FASTA line width")
    ap.add_argument("--reuse", action="store_true", help="keep files already in --dir")
    ap.add_argument("--child", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--cache", action="store_true", help=argparse.SUPPRESS)
    a = ap.parse_args()
    if a.child:
        return child(a)
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
        lines = seq[: a.len // a.line * a.line].reshape(-1, a.line)
        body = b"\n".join(bytes(x) for x in lines)
        data = b">genome_%d synthetic\n" % i + body + b"\n"
        for kind in ("plain", "gz"):
            p = os.path.join(d, "g%05d.fna%s" % (i, ".gz" if kind == "gz" else ""))
            paths[kind].append(p)
            if a.reuse and os.path.exists(p):  # (the same seeded files from an earlier run)
                continue
            if kind == "gz":
                with gzip.open(p, "wb", compresslevel=6) as f:
                    f.write(data)
            else:
                with open(p, "wb") as f:
                    f.write(data)
    gen_s = time.perf_counter() - t0
    out = {"files": a.files, "genome_len": a.len, "line": a.line, "threads": a.threads, "generate_s": round(gen_s, 2)}
    bases = a.files * (a.len // a.line * a.line)
    for kind in ("plain", "gz"):
        t0 = time.perf_counter()
        pk = ga.pack_files(paths[kind], threads=a.threads)
        t = time.perf_counter() - t0
        out["pack_%s_s" % kind] = round(t, 3)
        out["pack_%s_gbases_per_s" % kind] = round(bases / t / 1e9, 3)
        pk.free()
    listing = os.path.join(d, "gz_paths.txt")
    with open(listing, "w") as f:
        f.write("\n".join(paths["gz"]))
    runs = []
    for rep in [int(x) for x in a.repeat.split(",")]:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", listing, "--repeat", str(rep),
                            "--threads", str(a.threads)], capture_output=True, text=True, timeout=900)
        if r.returncode != 0:
            raise SystemExit(r.stderr)
        runs.append(json.loads(r.stdout.strip().splitlines()[-1]))
    out["precluster_files_gz"] = runs
    # the sketch cache: a cold call (sketches and stores
    # every genome) then a warm one (every genome read from the cache)
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", listing, "--repeat", "1",
                        "--threads", str(a.threads), "--cache"], capture_output=True, text=True, timeout=900)
    if r.returncode != 0:
        raise SystemExit(r.stderr)
    out["precluster_files_gz_cache"] = json.loads(r.stdout.strip().splitlines()[-1])
    out["precluster_files_gz_s"] = runs[0]["s"]
    out["pairs_found"] = runs[0]["pairs"]
    out["precluster_over_pack_gz"] = round(runs[0]["s"] / out["pack_gz_s"], 3)
    print(json.dumps(out), flush=True)


def child(a):
    """One gg_precluster_files call over the listed paths x repeat (after a
    small warm-up call), in its own process: time and peak RSS."""
    import resource
    with open(a.child) as f:
        paths = [x for x in f.read().split("\n") if x] * int(a.repeat)
    rss0 = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss
    if a.cache:
        cache = tempfile.mkdtemp(prefix="gg_cache_")
        with ga.Context(k=21, sketch_size=1000, host_threads=a.threads) as ctx:
            ctx.precluster_files(paths[:8], ga.parse_percentage(95))  # warm-up, no cache
            res = {"genomes": len(paths)}
            for leg in ("cold", "warm"):
                t0 = time.perf_counter()
                pairs, ani = ctx.precluster_files(paths, ga.parse_percentage(95), cache_dir=cache)
                res[leg + "_s"] = round(time.perf_counter() - t0, 3)
                res[leg + "_cached"] = int(ctx.last_cached)
                res[leg + "_pairs"] = int(len(pairs))
        print(json.dumps(res), flush=True)
        return
    with ga.Context(k=21, sketch_size=1000, host_threads=a.threads) as ctx:
        ctx.precluster_files(paths[:8], ga.parse_percentage(95))  # device and library warm-up
        rss1 = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss
        t0 = time.perf_counter()
        pairs, ani = ctx.precluster_files(paths, ga.parse_percentage(95))
        t = time.perf_counter() - t0
    rss2 = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss
    print(json.dumps({"genomes": len(paths), "repeat": int(a.repeat), "s": round(t, 3), "pairs": int(len(pairs)),
                      "peak_rss_mib_before": round(rss1 / 1024, 1), "peak_rss_mib": round(rss2 / 1024, 1),
                      "rss_mib_at_start": round(rss0 / 1024, 1)}), flush=True)


if __name__ == "__main__":
    main()
