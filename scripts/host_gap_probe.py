"""Where the host time of a C3 step goes (one device): the Python call of
precluster_shards against the library's phase timers, and the Python work
around the call (result arrays, phase_times).  Prints one JSON line.

  python3 scripts/host_gap_probe.py [--genomes 10000] [--steps 20]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import galah_amd as ga  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--genomes", type=int, default=10000)
    ap.add_argument("--genome-len", type=int, default=3_000_000)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    ctx = ga.Context(k=21, sketch_size=1000, seed=0, device=0)
    d_words = torch.empty(a.genomes * a.genome_len // 16, dtype=torch.int32, device="cuda:0")
    runs = ctx.synth_device(a.genomes, a.genome_len, 10, 0.07, 42, d_words, first_genome=0)
    shards = [(d_words, ga.device_runs(runs, "cuda:0"), a.genomes)]
    min_ani = ga.parse_percentage(95)
    for _ in range(3):
        ctx.precluster_shards(shards, min_ani)
    torch.cuda.synchronize()
    call, phases, loop = [], [], []
    for _ in range(a.steps):
        t0 = time.perf_counter()
        pairs, ani = ctx.precluster_shards(shards, min_ani)
        t1 = time.perf_counter()
        ph = ctx.phase_times()
        n = len(pairs)
        t2 = time.perf_counter()
        call.append((t1 - t0) * 1e3)
        phases.append(sum(ph.values()))
        loop.append((t2 - t0) * 1e3)
    call, phases, loop = np.array(call), np.array(phases), np.array(loop)
    print(json.dumps({
        "genomes": a.genomes, "pairs": n,
        "call_ms": round(float(np.median(call)), 4),
        "phases_ms": round(float(np.median(phases)), 4),
        "in_call_outside_phases_ms": round(float(np.median(call - phases)), 4),
        "after_call_ms": round(float(np.median(loop - call)), 4),
        "phase_ms": {k: round(v, 4) for k, v in ph.items()},
    }))
    ctx.close()


if __name__ == "__main__":
    main()
