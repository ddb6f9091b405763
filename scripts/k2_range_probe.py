"""K2 latency of each member of an M-device call, measured one part at a time
on one GPU: sketch a synthetic set once (C3: 10k x 3 Mbp, or C4-shaped with
--genomes 100000), then time gg_pairs_device over tile part d of M
(gg_pair_partition, as multi.cpp deals them) for M in 1, 2, 4, 8.  On a node
the parts run concurrently on M GPUs, so max over d is the pairs phase's
device time there.  Run it twice, with GALAHGPU_INDEX_RANGE=0 (every device
indexes every entry) and unset (each device indexes the entries its rows may
share: pairs_index.hip's row-range index).

    python scripts/k2_range_probe.py [--genomes 10000] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import galah_amd as ga  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--genomes", type=int, default=10000)
    ap.add_argument("--genome-len", type=int, default=3000000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--parts", default="1,2,4,8")
    ap.add_argument("--by-pairs", action="store_true")
    a = ap.parse_args()
    N, glen, s = a.genomes, a.genome_len, 1000
    ctx = ga.Context(k=21, sketch_size=s)
    d_sk = torch.empty((N, s), dtype=torch.int64, device="cuda")
    d_len = torch.empty(N, dtype=torch.int32, device="cuda")
    chunk = 10000  # genomes synthesised and sketched per pass (HBM for the packed words)
    for g0 in range(0, N, chunk):
        g1 = min(N, g0 + chunk)
        d_words = torch.empty((g1 - g0) * glen // 16, dtype=torch.int32, device="cuda")
        runs = ctx.synth_device(g1 - g0, glen, 10, 0.07, 3, d_words, first_genome=g0)
        ctx.sketch_device(d_words, runs, g1 - g0, d_sk[g0:g1], d_len[g0:g1])
        torch.cuda.synchronize()
        del d_words
    cap = 1 << 24
    d_out = torch.empty(cap * 4, dtype=torch.int32, device="cuda")
    d_cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    mn = ga.parse_percentage(95)
    out = {"genomes": N, "index_range": os.environ.get("GALAHGPU_INDEX_RANGE", "1"),
           "partition": "pairs" if a.by_pairs else "rows", "parts": {}}
    for M in [int(x) for x in a.parts.split(",")]:
        per, found = [], 0
        for d in range(M):
            if a.by_pairs:
                tb, te = ga.pair_partition(N, M, d)
            else:
                nb = (N + 63) // 64  # GG_PAIR_TILE

                def row_tile(I):
                    return I * nb - I * (I - 1) // 2
                tb, te = row_tile(nb * d // M), row_tile(nb * (d + 1) // M)
            best = 1e9
            for r in range(a.reps + 1):
                d_cnt.zero_()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                ctx.pairs_device(d_sk, d_len, N, tb, te, mn, d_out, cap, d_cnt)
                torch.cuda.synchronize()
                if r:
                    best = min(best, time.perf_counter() - t0)
            found += int(d_cnt.item())
            per.append(round(best * 1e3, 3))
        out["parts"][M] = {"ms_per_part": per, "max_ms": max(per), "pairs": found}
        print(json.dumps({"M": M, "max_ms": max(per), "ms_per_part": per, "pairs": found}), flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
