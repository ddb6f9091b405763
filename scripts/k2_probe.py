"""Pair-kernel probe: sketch a synthetic C3-shaped set once, then time the
pair kernel alone (per-launch HIP events on its stream).  For rocprofv3 /
PMC runs on the pair kernel and quick A/B of kernel variants.

    python scripts/k2_probe.py [--genomes 10000] [--genome-len 3000000] [--reps 3]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import galah_amd as ga  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--genomes", type=int, default=10000)
    ap.add_argument("--genome-len", type=int, default=3000000)
    ap.add_argument("--cluster", type=int, default=10)
    ap.add_argument("--sketch", type=int, default=1000)
    ap.add_argument("--min-ani", type=float, default=95.0)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    N, glen, s = a.genomes, a.genome_len, a.sketch
    ctx = ga.Context(k=21, sketch_size=s)
    d_words = torch.empty(N * glen // 16, dtype=torch.int32, device="cuda")
    runs = ctx.synth_device(N, glen, a.cluster, 0.07, 3, d_words)
    d_sk = torch.empty((N, s), dtype=torch.int64, device="cuda")
    d_len = torch.empty(N, dtype=torch.int32, device="cuda")
    ctx.sketch_device(d_words, runs, N, d_sk, d_len)
    del d_words
    torch.cuda.synchronize()
    cap = 1 << 24
    d_out = torch.empty(cap * 4, dtype=torch.int32, device="cuda")
    d_cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    tb, te = 0, ga.pair_tiles(N)
    mn = ga.parse_percentage(a.min_ani)
    ctx.pairs_device(d_sk, d_len, N, tb, te, mn, d_out, cap, d_cnt)  # warm
    torch.cuda.synchronize()
    ctx.timing_enable(True)
    for _ in range(a.reps):
        d_cnt.zero_()
        ctx.pairs_device(d_sk, d_len, N, tb, te, mn, d_out, cap, d_cnt)
    torch.cuda.synchronize()
    st = ctx.timing_read(ga.KERNEL_PAIRS)
    ms = st["ms"] / st["launches"]
    print(json.dumps({"genomes": N, "pairs_per_launch": st["work"] / st["launches"], "ms": round(ms, 3),
                      "pairs_per_s": st["work"] / st["launches"] / (ms * 1e-3), "found": int(d_cnt.item()),
                      "kernel": os.environ.get("GALAHGPU_PAIRS_KERNEL", "gate")}))
    ctx.close()


if __name__ == "__main__":
    main()
