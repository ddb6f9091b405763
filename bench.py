"""Benchmark: galah finch precluster path on MI355X.

Metric (BASELINE.json): precluster genome-pairs/sec at 10k genomes (s=1000)
+ sketch Gbases/s.  Workload = config C3: 10,000 synthetic
3 Mbp genomes in clusters of 10 (member substitution rate ~ U(0, 0.07)),
k=21, s=1000, min_ani = 0.95 (f32, as parse_percentage(95) yields).

One step = the whole precluster hot path over inputs already resident in
HBM (2-bit packed genomes):
  K1 sketch this rank's genome shard  ->  RCCL all_gather of the sketches
  (N > 1)  ->  K2 all-pairs over this rank's share of the upper-triangle
  tiles  ->  D2H of the passing (i, j, common, total) tuples.
value = N(N-1)/2 genome pairs / step time (max over ranks).  Total work is
fixed as the GPU count grows, so scaling is "strong".

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       multi-GPU: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import galah_amd as ga  # noqa: E402
from galah_amd import sharding  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
CLK_GHZ = 2.4          # max engine clock
N_SIMD = 256 * 4       # 256 CUs x 4 SIMDs
# K1 (sketch) is VALU-issue bound.  A SIMD issues one wave64 integer VALU
# instruction per 4 cycles (16 lanes x 4 passes; multiplies included --
# scripts/ubench_valu.hip, profiles/r01_ubench_valu.txt).  K1's VALU count per
# k-mer (all of the kernel: hashing, windows, segment setup, candidate
# inserts) is SQ_INSTS_VALU / (k-mers / 64) from the PMC pass over the C3
# launch (profiles/r01_pmc_k1_grid112.txt).  Ceiling = 1024 SIMDs x 2.4 GHz x 64
# lanes / (4 cycles x VALU per k-mer).  Since the K1 grid went to 112
# workgroups per CU the kernel reads at ~1.0 of this ceiling (52.1 ms against
# 53.4 ms): it is at the VALU issue limit to within the accuracy of this
# model (PMC instruction count, nominal clock, 4 cycles for every VALU op).
K1_CYCLES_PER_VALU = 4
K1_VALU_PER_KMER = 3.282e10 / (29999800000 / 64)
K1_PEAK_GKMER = N_SIMD * CLK_GHZ * 64 / (K1_CYCLES_PER_VALU * K1_VALU_PER_KMER)  # Gkmer/s
# K2 (pairs: gate_lo32 + gate_build + pairs_gate kernels) is also priced
# against VALU issue: SQ_INSTS_VALU of the three kernels per evaluated pair
# from the PMC pass over the C3 launch (profiles/r01_pmc_k1_k2gate.txt).  It
# runs well under that ceiling: the queued table walks wait on L2/HBM.
K2_VALU_PER_PAIR = (6.706e8 + 3.076e7 + 7.888e5) / 49995000
K2_PEAK_GPAIR = N_SIMD * CLK_GHZ / (K1_CYCLES_PER_VALU * K2_VALU_PER_PAIR)  # Gpair/s
K2_PMC_HBM_BYTES_C3 = (5.586e6 + 7.706e4 + 3.907e4) * 1024 * 2
# SURVEY 8(d)'s merge pricing (8 B x (|A| + |B|) per pair against 256 B/clk/CU
# of LDS), reported for reference: the gate kernel does not merge.
LDS_PEAK_GBS = 256 * 256 * CLK_GHZ
# HBM bytes per K1 launch on this workload from the PMC pass (FETCH_SIZE x 2,
# the gfx950 correction of MI355X_MICROARCH.md), profiles/r01_pmc_k1_grid112.txt
K1_PMC_HBM_BYTES_C3 = 3.871e6 * 1024 * 2


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3", choices=["c2", "c3", "c5"],
                    help="c3 (default, the headline): 10k x 3 Mbp, s=1000; c2: 1k x 3 Mbp; "
                         "c5: 10k genomes of 0.5-12 Mbp (log-uniform) with N runs, s=10000")
    ap.add_argument("--genomes", type=int, default=None)
    ap.add_argument("--genome-len", type=int, default=3000000, help="c2/c3 genome length")
    ap.add_argument("--cluster", type=int, default=10)
    ap.add_argument("--max-sub", type=float, default=0.07)
    ap.add_argument("--min-ani", type=float, default=95.0, help="--precluster-ani (percent)")
    ap.add_argument("--sketch", type=int, default=None)
    ap.add_argument("--k", type=int, default=21)
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget-s", type=float, default=20.0)
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo stages collectives through host memory (testing ranks that share one GPU)")
    a = ap.parse_args()
    if a.genomes is None:
        a.genomes = 1000 if a.config == "c2" else 10000
    if a.sketch is None:
        a.sketch = 10000 if a.config == "c5" else 1000
    return a


def cpu_baseline(words_dev, runs, glen, sk_all, lens_all, k, s, min_ani, n_total, budget_s):
    """The CPU oracle (oracle/, a C restatement of finch as galah calls it)
    timed on this host on a bounded sample, extrapolated to the workload:
    sketching parallel over genomes on T threads (finch sketch_files is a
    rayon par_iter over files), the pair loop serial as src/finch.rs:53."""
    import concurrent.futures as cf

    import oracle
    T = max(1, min(16, os.cpu_count() or 1))
    # -- sketch sample: T genomes, one per thread
    n_s = min(T, len(runs))
    words = words_dev[: (n_s * glen) // 16].cpu().numpy().view(np.uint32)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    seqs = []
    for g in range(n_s):
        w = words[g * glen // 16:(g + 1) * glen // 16]
        codes = (w[:, None] >> (np.uint32(30) - 2 * np.arange(16, dtype=np.uint32))[None, :]) & np.uint32(3)
        seqs.append(acgt[codes.reshape(-1)].tobytes())
    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(T) as ex:
        outs = list(ex.map(lambda q: oracle.sketch_sequence(q, k=k, s=s), seqs))
    t_sk = time.perf_counter() - t0
    for g in range(n_s):  # the sample doubles as a parity spot check
        assert (outs[g] == sk_all[g][:lens_all[g]]).all()
    sketch_bases_per_s = n_s * glen / t_sk
    # -- pair sample: the serial loop over the first m genomes' sketches
    m = 200
    while True:
        t0 = time.perf_counter()
        oracle.pairs(sk_all[:m], lens_all[:m].astype(np.int32), min_ani, k=k, cap=m * m)
        t_p = time.perf_counter() - t0
        if t_p > budget_s / 4 or m >= min(2000, n_total):
            break
        m = min(min(2000, n_total), int(m * max(1.5, (budget_s / 4 / max(t_p, 1e-3)) ** 0.5)))
    pair_rate = m * (m - 1) / 2 / t_p
    npairs = n_total * (n_total - 1) / 2
    t_total = n_total * glen / sketch_bases_per_s + npairs / pair_rate
    return {
        "value": npairs / t_total, "unit": "genome-pairs/s", "cores": T, "kind": "port",
        "sample": ("oracle/ C restatement of finch on %d host threads: sketched %d x %d bp synthetic genomes "
                   "(%.1f Mbases/s), serial pair loop (1 core, src/finch.rs:53) over %d genomes' sketches "
                   "(%.0f pairs/s); extrapolated to %d genomes = %.0f s"
                   % (T, n_s, glen, sketch_bases_per_s / 1e6, m, pair_rate, n_total, t_total)),
        "sketch_mbases_per_s": sketch_bases_per_s / 1e6,
        "pair_rate_1core": pair_rate,
    }


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    gloo = a.dist_backend == "gloo"
    if gloo:
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        if gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    N, glen, s = a.genomes, a.genome_len, a.sketch
    g0, g1 = sharding.shard_range(N, world, rank)
    n_loc = g1 - g0
    even = N % world == 0
    min_ani = ga.parse_percentage(a.min_ani)
    ctx = ga.Context(k=a.k, sketch_size=s, seed=0, device=local)
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream

    # inputs resident in HBM: this rank's genome shard, 2-bit packed
    if a.config == "c5":
        lens_bp = ga.synth_mixed_lengths(n_loc, 500000, 12000000, a.cluster, 7, first_genome=g0)
        d_words = torch.empty(int(lens_bp.sum()) // 16, dtype=torch.int32, device="cuda")
        runs = ctx.synth_mixed_device(lens_bp, a.cluster, a.max_sub, 1e-4, 8, d_words, stream=sh, first_genome=g0)
        bases_loc = int(lens_bp.sum())
    else:
        d_words = torch.empty(n_loc * glen // 16, dtype=torch.int32, device="cuda")
        runs = ctx.synth_device(n_loc, glen, a.cluster, a.max_sub, a.seed, d_words, stream=sh, first_genome=g0)
        bases_loc = n_loc * glen
    d_sk_loc = torch.empty((n_loc, s), dtype=torch.int64, device="cuda")
    d_len_loc = torch.empty(n_loc, dtype=torch.int32, device="cuda")
    if world > 1:
        d_sk = torch.empty((N, s), dtype=torch.int64, device="cuda")
        d_len = torch.empty(N, dtype=torch.int32, device="cuda")
    else:
        d_sk, d_len = d_sk_loc, d_len_loc
    tb, te = sharding.rank_tiles(N, world, rank)
    cap = max(1 << 22, N * 64)
    d_out = torch.empty(cap * 4, dtype=torch.int32, device="cuda")
    d_cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()

    ev = {k: (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for k in ("sketch", "gather", "pairs")}

    def step():
        ev["sketch"][0].record(stream)
        ctx.sketch_device(d_words, runs, n_loc, d_sk_loc, d_len_loc, stream=sh)
        ev["sketch"][1].record(stream)
        ev["gather"][0].record(stream)
        if world > 1 and gloo:
            gsk, gln = sharding.all_gather_sketches(d_sk_loc.cpu(), d_len_loc.cpu(), N, world, rank, dist)
            d_sk.copy_(gsk)
            d_len.copy_(gln)
        elif world > 1 and even:
            dist.all_gather_into_tensor(d_sk, d_sk_loc)
            dist.all_gather_into_tensor(d_len, d_len_loc)
        elif world > 1:
            gsk, gln = sharding.all_gather_sketches(d_sk_loc, d_len_loc, N, world, rank, dist)
            d_sk.copy_(gsk)
            d_len.copy_(gln)
        ev["gather"][1].record(stream)
        d_cnt.zero_()
        ev["pairs"][0].record(stream)
        ctx.pairs_device(d_sk, d_len, N, tb, te, min_ani, d_out, cap, d_cnt, stream=sh)
        ev["pairs"][1].record(stream)
        cnt = int(d_cnt.item())
        if cnt > cap:
            raise RuntimeError("pair buffer too small: %d > %d" % (cnt, cap))
        host = d_out[: cnt * 4].cpu()  # sparse results to host
        return cnt, host

    for _ in range(a.warmup):
        step()
    phase = {k: 0.0 for k in ev}
    ctx.timing_enable(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    found = 0
    for _ in range(a.steps):
        found, _host = step()
        torch.cuda.synchronize()
        for k, (e0, e1) in ev.items():
            phase[k] += e0.elapsed_time(e1)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kst = {name: ctx.timing_read(kid) for name, kid in
           (("sketch", ga.KERNEL_SKETCH), ("finalize", ga.KERNEL_FINALIZE), ("pairs", ga.KERNEL_PAIRS))}
    ctx.timing_enable(False)
    t = torch.tensor([elapsed, phase["sketch"], phase["pairs"], phase["gather"], float(found), float(bases_loc)],
                     dtype=torch.float64, device="cuda")
    if world > 1:
        if gloo:
            t = t.cpu()
        tmax = t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tsum = t.clone()
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
    else:
        tmax = tsum = t
    elapsed_max = float(tmax[0])
    ms_step = elapsed_max / a.steps * 1e3
    npairs = N * (N - 1) // 2
    value = npairs / (elapsed_max / a.steps)
    total_bases = float(tsum[5])

    # roofline of the dominant kernel, from this rank's per-launch events
    sk_ms = kst["sketch"]["ms"] / max(1, kst["sketch"]["launches"])
    pr_ms = kst["pairs"]["ms"] / max(1, kst["pairs"]["launches"])
    kmers_per_launch = kst["sketch"]["work"] / max(1, kst["sketch"]["launches"])
    pairs_per_launch = kst["pairs"]["work"] / max(1, kst["pairs"]["launches"])
    k1_gkmer = kmers_per_launch / (sk_ms * 1e-3) / 1e9
    k1 = {"kernel": "sketch_candidates_kernel<21>", "bound": "valu", "unit": "Gkmer/s",
          "achieved": k1_gkmer, "peak": K1_PEAK_GKMER, "avg_ms": sk_ms, "work_per_launch": kmers_per_launch,
          "hbm_achieved_GBps": kmers_per_launch * 0.25 / (sk_ms * 1e-3) / 1e9, "hbm_peak_GBps": HBM_PEAK_GBS,
          "traffic": (K1_PMC_HBM_BYTES_C3 if (a.config == "c3" and N == 10000 and glen == 3000000 and world == 1)
                      else None),
          "valu_per_kmer": K1_VALU_PER_KMER,
          "note": ("VALU-issue ceiling: %.1f VALU per wave64 k-mer (PMC) x %d cycles each, 1024 SIMDs at "
                   "%.1f GHz; input is 0.25 B/k-mer, so the HBM fraction is small by design; a frac of ~1.0 or "
                   "slightly above means the kernel is at the issue limit and the PMC count or the 4-cycle/nominal-"
                   "clock model is a few percent off, not that the limit is exceeded"
                   % (K1_VALU_PER_KMER, K1_CYCLES_PER_VALU, CLK_GHZ))}
    c3 = a.config == "c3" and N == 10000 and glen == 3000000 and world == 1 and s == 1000
    k2 = {"kernel": "pairs_gate_kernel (+ gate_build_kernel, gate_lo32_kernel)", "bound": "valu", "unit": "Gpair/s",
          "achieved": pairs_per_launch / (pr_ms * 1e-3) / 1e9, "peak": K2_PEAK_GPAIR,
          "avg_ms": pr_ms, "work_per_launch": pairs_per_launch,
          "traffic": (K2_PMC_HBM_BYTES_C3 if c3 else None), "valu_per_pair": K2_VALU_PER_PAIR,
          "merge_priced_GBps": pairs_per_launch * 16.0 * s / (pr_ms * 1e-3) / 1e9, "lds_peak_GBps": LDS_PEAK_GBS,
          "note": ("VALU-issue ceiling: %.2f VALU per pair (PMC, all three kernels) x %d cycles, 1024 SIMDs at %.1f GHz; "
                   "latency of the queued table walks keeps it below; merge_priced_GBps = SURVEY 8(d) pricing "
                   "(16 KB per pair at s=1000) for reference" % (K2_VALU_PER_PAIR, K1_CYCLES_PER_VALU, CLK_GHZ))}
    dom = k1 if sk_ms * kst["sketch"]["launches"] >= pr_ms * kst["pairs"]["launches"] else k2
    roof = {"bound": dom["bound"], "achieved": round(dom["achieved"], 3), "peak": round(dom["peak"], 3),
            "unit": dom["unit"], "frac": round(dom["achieved"] / dom["peak"], 4), "traffic": dom["traffic"],
            "kernel": dom["kernel"], "avg_launch_ms": round(dom["avg_ms"], 4), "note": dom["note"],
            "kernels": [{kk: (round(v, 5) if isinstance(v, float) else v) for kk, v in x.items()}
                        for x in (k1, k2)]}

    # SURVEY 8(f) row 1, downstream of the timed step: single-linkage
    # preclusters of the passing pairs (host C++, union-find), and
    # transform_ids for every precluster at once
    downstream = None
    if rank == 0 and world == 1:
        pairs_h = _host.numpy().view(np.uint32).reshape(-1, 4)
        pa = np.zeros(len(pairs_h), dtype=ga.PAIR_DTYPE)
        for k_, f_ in enumerate(("i", "j", "common", "total")):
            pa[f_] = pairs_h[:, k_]
        t0 = time.perf_counter()
        members, offsets = ga.partition_preclusters(N, pa)
        t_part = time.perf_counter() - t0
        t0 = time.perf_counter()
        ga.precluster_pairs(N, pa, members, offsets)
        t_tr = time.perf_counter() - t0
        downstream = {"partition_preclusters_ms": round(t_part * 1e3, 3), "precluster_pairs_ms": round(t_tr * 1e3, 3),
                      "preclusters": int(len(offsets) - 1), "largest": int(np.diff(offsets).max()) if N else 0}

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline and a.config != "c5":
        sk_h = d_sk.cpu().numpy().view(np.uint64)
        ln_h = d_len.cpu().numpy().view(np.uint32)
        cpu = cpu_baseline(d_words, runs, glen, sk_h, ln_h, a.k, s, min_ani, N, a.cpu_budget_s)

    if rank == 0:
        line = {
            "metric": "precluster genome-pairs/sec at 10k genomes (s=1000) + sketch Gbases/s",
            "value": round(value, 1), "unit": "genome-pairs/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "u64",
            "data": "synthetic clustered genomes generated on device (no network)",
            "config": {"workload": (("C5: %d synthetic genomes of 0.5-12 Mbp (log-uniform, %.0f bp total) with N runs"
                                     % (N, total_bases)) if a.config == "c5" else
                                    ("%s: %d synthetic genomes x %d bp" % (a.config.upper(), N, glen)))
                                   + ", clusters of %d, sub rate U(0,%.2f), k=%d, s=%d, min_ani=%s"
                                   % (a.cluster, a.max_sub, a.k, s, min_ani),
                       "genomes": N, "genome_len": (None if a.config == "c5" else glen), "sketch_size": s, "k": a.k,
                       "min_ani": float(min_ani), "parallelism": "dp%d" % world},
            "sketch_gbases_per_s": round(total_bases / (float(tmax[1]) / a.steps * 1e-3) / 1e9, 3),
            "pairs_kernel_pairs_per_s": round(npairs / (float(tmax[2]) / a.steps * 1e-3), 1),
            "phase_ms": {"sketch": round(float(tmax[1]) / a.steps, 3), "allgather": round(float(tmax[3]) / a.steps, 3),
                         "pairs": round(float(tmax[2]) / a.steps, 3)},
            "pairs_found": int(tsum[4]) if world > 1 else found,
            "roofline": roof,
            "cpu_baseline": cpu,
            "downstream": downstream,
        }
        print(json.dumps(line), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
