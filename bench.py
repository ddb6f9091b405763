"""Benchmark: galah finch precluster path on MI355X.

Metric (BASELINE.json): precluster genome-pairs/sec at 10k genomes (s=1000)
+ sketch Gbases/s.  Workload = config C3: 10,000 synthetic
3 Mbp genomes in clusters of 10 (member substitution rate ~ U(0, 0.07)),
k=21, s=1000, min_ani = 0.95 (f32, as parse_percentage(95) yields).

One step = the whole precluster hot path over inputs already resident in
HBM (2-bit packed genomes), i.e. FinchPreclusterer::distances after ingest
(src/finch.rs:47-73), as ONE library call (gg_precluster_shards):
  K1 sketch every device's genome shard  ->  replicate the sketches to every
  device (peer copies over xGMI)  ->  K2 over each device's share of the
  upper-triangle tiles  ->  D2H of the passing (i, j, common, total)  ->
  host merge sorted by (i, j) with the f32 ANI of src/finch.rs:70.
value = N(N-1)/2 genome pairs / step time.  Total work is fixed as the GPU
count grows, so scaling is "strong".

Multi-GPU: `--gpus N` drives N devices from one process through the library
(galah calls distances() once, from one process: src/clusterer.rs:36).  Under
the driver's `torch.distributed.run --nproc-per-node N`, rank 0 runs that
call over all N GPUs and the other ranks only join the CPU (gloo) barriers
around the timed region.  `--mode dist` keeps the one-process-per-GPU layout
(RCCL all-gather of the sketches, galah_amd/sharding.py) for comparison.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c5]
"""
import argparse
import json
import os
import platform
import subprocess
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
CLK_GHZ = 2.4          # max engine clock (MI355X_MICROARCH.md chip parameters)
N_SIMD = 256 * 4       # 256 CUs x 4 SIMDs
# K1's VALU-issue ceiling (the kernel is bound by VALU issue; its input is
# 0.25 B per k-mer, ~2% of HBM): profiles/r04_k1_issue_model.json, written by
# scripts/k1_issue_model.py from a rocprofv3 PMC pass over K1 at HEAD and the
# per-opcode issue costs measured by scripts/ubench_dual.hip.  The model
# records a fingerprint of K1's machine code; bench.py recomputes it from the
# library it loads and flags the peak as stale when K1 has changed since.
ISSUE_MODEL = os.path.join(ROOT, "profiles", "r04_k1_issue_model.json")
# K2's per-kernel PMC summary (HBM bytes from FETCH_SIZE x 2 and WRITE_SIZE,
# VALU issue share, LDS-array utilisation) of the bucketed inverted index:
# scripts/k2_pmc.sh + scripts/k2_pmc_model.py
K2_PMC = os.path.join(ROOT, "profiles", "r05_k2_pmc.json")
# the device-inflate ingest kernels' counters at C2 (scripts/ingest_pmc.sh + ingest_pmc_model.py)
INGEST_PMC = os.path.join(ROOT, "profiles", "r06", "ingest_pmc.json")
sys.path.insert(0, os.path.join(ROOT, "scripts"))
from host_cpus import host_cpu_info  # noqa: E402


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--mode", default="lib", choices=["lib", "dist"],
                    help="lib (default): one library call drives every GPU; dist: one process per GPU, "
                         "RCCL all-gather (galah_amd/sharding.py)")
    ap.add_argument("--config", default="c3", choices=["c2", "c3", "c4", "c5"],
                    help="c3 (default, the headline): 10k x 3 Mbp, s=1000; c2: 1k x 3 Mbp; c4: 100k x 3 Mbp; "
                         "c5: 10k genomes of 0.5-12 Mbp (log-uniform) with N runs, s=10000")
    ap.add_argument("--genomes", type=int, default=None)
    ap.add_argument("--genome-len", type=int, default=3000000, help="c2/c3/c4 genome length")
    ap.add_argument("--cluster", type=int, default=10)
    ap.add_argument("--max-sub", type=float, default=0.07)
    ap.add_argument("--min-ani", type=float, default=95.0, help="--precluster-ani (percent)")
    ap.add_argument("--sketch", type=int, default=None)
    ap.add_argument("--k", type=int, default=21)
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--devices", default=None,
                    help="lib mode: comma-separated HIP ordinals (repeats allowed, e.g. 0,0 to run the sharded "
                         "path on one GPU); default: 0..gpus-1")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--files", dest="files", action="store_true", default=None,
                    help="add the ingest-inclusive leg (C2's genomes as gzip FASTA files through "
                         "gg_precluster_files); on by default for the one-GPU C3 headline")
    ap.add_argument("--no-files", dest="files", action="store_false")
    ap.add_argument("--files-genomes", type=int, default=1000, help="genomes in the files leg (C2: 1000)")
    ap.add_argument("--c4", dest="c4_leg", action="store_true", default=None,
                    help="add the north-star leg (C4: 100k x 3 Mbp, s=1000 on one GPU, 3 steps); on by default for "
                         "the one-GPU C3 headline")
    ap.add_argument("--no-c4", dest="c4_leg", action="store_false")
    ap.add_argument("--c4-steps", type=int, default=3)
    ap.add_argument("--cpu-budget-s", type=float, default=24.0)
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="dist mode: gloo stages collectives through host memory (ranks sharing one GPU)")
    a = ap.parse_args()
    if a.genomes is None:
        a.genomes = {"c2": 1000, "c4": 100000}.get(a.config, 10000)
    if a.sketch is None:
        a.sketch = 10000 if a.config == "c5" else 1000
    return a


# ---------------------------------------------------------------------------
# inputs: the synthetic workload, generated in HBM
# ---------------------------------------------------------------------------
def make_shard(ctx, a, g0, g1, dev):
    """Genomes [g0, g1) of the workload on device `dev` -> (d_words, runs, bases)."""
    n = g1 - g0
    if a.config == "c5":
        lens_bp = ga.synth_mixed_lengths(n, 500000, 12000000, a.cluster, 7, first_genome=g0)
        d_words = torch.empty(max(1, int(lens_bp.sum()) // 16), dtype=torch.int32, device="cuda:%d" % dev)
        runs = ctx.synth_mixed_device(lens_bp, a.cluster, a.max_sub, 1e-4, 8, d_words, first_genome=g0)
        return d_words, runs, int(lens_bp.sum())
    d_words = torch.empty(max(1, n * a.genome_len // 16), dtype=torch.int32, device="cuda:%d" % dev)
    runs = ctx.synth_device(n, a.genome_len, a.cluster, a.max_sub, a.seed, d_words, first_genome=g0)
    return d_words, runs, n * a.genome_len


def sync_all(devs):
    for d in sorted(set(devs)):
        torch.cuda.synchronize(d)


# ---------------------------------------------------------------------------
# roofline of the dominant kernel
# ---------------------------------------------------------------------------
def k1_fingerprint():
    """sha1 of K1's (k = 21, seed 0) machine code in the loaded library (scripts/k1_isa.py), or None."""
    try:
        sys.path.insert(0, os.path.join(ROOT, "scripts"))
        import k1_isa
        listing = k1_isa.kernel_listing(ga.LIB_PATH)
        return k1_isa.fingerprint(listing) if listing else None
    except Exception:
        return None


def k2_pmc(config):
    """The K2 kernels' PMC summary for this config (one step of the same
    workload, measured by scripts/k2_pmc.sh), or None."""
    if not os.path.exists(K2_PMC):
        return None
    with open(K2_PMC) as f:
        m = json.load(f)
    c = m.get(config)
    if not c:
        return None
    keep = ("dispatches", "ms", "hbm_bytes", "hbm_GBps", "hbm_frac", "valu_frac_guide", "lds_util", "l2_hit",
            "bound", "bound_frac")
    ks = {k: {x: e[x] for x in keep if x in e} for k, e in c["kernels"].items()}
    return {"source": "profiles/r05_k2_pmc.json (%s, one step; raw: %s)" % (config, c.get("source")), "kernels": ks,
            "peaks": "VALU: 2 cycles per wave64 instruction per SIMD (MI355X_MICROARCH.md); LDS: array busy cycles "
                     "per CU; HBM: 8 TB/s, bytes = FETCH_SIZE x 2 + WRITE_SIZE"}


# K2 kernels timed under GG_KERNEL_PAIRS / GG_KERNEL_PAIRS_INDEX (the passing
# pairs' device sort is not: it is output handling, ~0.1 ms at C3)
K2_TIMED = ("index_scan", "bucket_hist", "bucket_base", "index_fill", "index_sort", "bucket_bounds", "split_keys",
            "split_scan", "split_scatter", "superbin_count", "superbin_place", "index_bucket", "index_pairs")


def index_split_on():
    """The split build (default) or GALAHGPU_INDEX_SPLIT=0's fill + 16-bit sort."""
    return os.environ.get("GALAHGPU_INDEX_SPLIT", "1") != "0"


def k2_algorithmic_bytes(d_sk, d_len, n, s):
    """Algorithmic HBM bytes of one K2 launch set (the bucketed inverted index
    over n sketches of stride s) from the sketches themselves:
    E = entries (sum of lengths), S = row slots (n x s: the fill keys every
    slot, unused ones sort last), runs of g >= 2 equal hashes give the pairs
    kernel g member reads per member (sum of g^2).  Member ids are 2 B when
    n <= 65,536 (index_ents16), else 4 B."""
    lens = d_len.to(torch.int64)
    E = int(lens.sum())
    S = n * s
    mask = torch.arange(s, device=d_sk.device)[None, :] < lens[:, None]
    _, cnt = torch.unique(d_sk[mask], return_counts=True)
    cnt = cnt[cnt >= 2].to(torch.float64)
    g2 = float((cnt * cnt).sum())
    runs = int(cnt.numel())
    # member reads of the pairs kernel: a run of g <= 32 is stored in row
    # order and each member reads only the members after it (g (g - 1) / 2
    # per run); a longer run is read whole by every member (g^2)
    short = cnt <= 32
    members = float((cnt[short] * (cnt[short] - 1) / 2).sum() + (cnt[~short] * cnt[~short]).sum())
    del mask
    m = 2 if n <= 65536 else 4
    per = {
        "index_scan": 4.0 * n,                        # row lengths
        "bucket_hist": 8.0 * (E if E < (1 << 26) else E / 8),  # each hash once (past 2^26 entries: 1 line in 8)
    }
    if index_split_on():
        per.update({
            "split_keys": 8.0 * E + 2.0 * S,          # hash read; 16-bit bucket id written per slot
            "split_scan": 2 * 4.0 * 256 * n,           # per-row super-bin counts read, offsets written
            "split_scatter": 2.0 * E + 5.0 * E,        # bucket ids read; low key byte + 32-bit entry written
            "superbin_count": 1.0 * E,                 # key bytes
            "superbin_place": 5.0 * E + 4.0 * E,       # key bytes + entries read, entries written
        })
    else:
        per.update({
            "index_fill": 8.0 * E + 6.0 * S,          # hash read; 16-bit bucket key + 32-bit entry written per slot
            "sort_16bit_2pass": 2.0 * S + 2 * 12.0 * S,  # key histogram; 2 passes reading and writing 6 B per slot
            "bucket_bounds": 2.0 * S,                 # sorted keys
        })
    per.update({
        "index_bucket": (4.0 + 8.0 + m + 8.0) * E,    # entry, its hash, member id and runinfo written
        "index_pairs": 8.0 * E + m * members,         # runinfo of every entry; the members after it in its run
    })
    return {"bytes": sum(per.values()), "per_kernel": per, "entries": E, "slots": S, "shared_runs": runs,
            "sum_g2": g2, "member_reads": members}


def roofline_k2(model, kst_pr, config):
    """K2's own roofline: algorithmic bytes of the index build + pairs kernel
    per launch set over its HIP-event time, against 8 TB/s."""
    sets = max(1, kst_pr["launches_sets"])
    ms = kst_pr["ms"] / sets
    ach = model["bytes"] / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
    out = {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None, "avg_launch_ms": round(ms, 4),
           "algorithmic_bytes": round(model["bytes"]),
           "algorithmic_bytes_per_kernel": {k: round(v) for k, v in model["per_kernel"].items()},
           "entries": model["entries"], "slots": model["slots"], "shared_runs": model["shared_runs"],
           "sum_g2": round(model["sum_g2"]), "member_reads": round(model["member_reads"]),
           "kernel": ("K2: bucketed inverted index (index_scan, bucket_hist, bucket_base, split_keys, scan, "
                      "split_scatter, superbin_count/place, index_bucket) + index_pairs_kernel" if index_split_on() else
                      "K2: bucketed inverted index (index_scan, bucket_hist, bucket_base, index_fill, 16-bit onesweep "
                      "sort, bucket_bounds, index_bucket) + index_pairs_kernel"),
           "note": "achieved = algorithmic bytes (per kernel above, DESIGN §4) / K2's HIP-event time per step (index "
                   "build + pairs kernel, on the stream they run on); traffic = HBM bytes of the same kernels from "
                   "the PMC pass (FETCH_SIZE x 2 + WRITE_SIZE, MI355X_MICROARCH.md), per step"}
    pmc = k2_pmc(config) if config else None
    if pmc:
        out["pmc"] = pmc
        tr = sum(e.get("hbm_bytes", 0.0) for k, e in pmc["kernels"].items() if k in K2_TIMED)
        out["traffic"] = round(tr) if tr else None
        out["pmc_ms"] = round(sum(e.get("ms", 0.0) for k, e in pmc["kernels"].items() if k in K2_TIMED), 4)
    return out


def roofline(kst_sk, kst_pr, s, config_note, config=None):
    model = None
    if os.path.exists(ISSUE_MODEL):
        with open(ISSUE_MODEL) as f:
            model = json.load(f)
    sk_ms = kst_sk["ms"] / max(1, kst_sk["launches"])
    pr_ms = kst_pr["ms"] / max(1, kst_pr["launches"])
    kmers = kst_sk["work"] / max(1, kst_sk["launches"])
    pairs = kst_pr["work"] / max(1, kst_pr["launches"])
    k1_gkmer = kmers / (sk_ms * 1e-3) / 1e9 if sk_ms > 0 else 0.0
    k1 = {"kernel": "sketch_candidates_kernel<21>", "bound": "valu", "unit": "Gkmer/s", "achieved": k1_gkmer,
          "avg_ms": sk_ms, "work_per_launch": kmers,
          "hbm_achieved_GBps": kmers * 0.25 / (sk_ms * 1e-3) / 1e9 if sk_ms > 0 else 0.0,
          "hbm_peak_GBps": HBM_PEAK_GBS, "algorithmic_bytes_per_kmer": 0.25}
    k1["hbm_frac"] = k1["hbm_achieved_GBps"] / HBM_PEAK_GBS
    if model:
        fp = k1_fingerprint()
        k1["peak_model"] = model["note"]
        k1["valu_per_wave_kmer"] = model["valu_per_wave_kmer"]
        k1["floor_cycles_per_wave_kmer"] = model["floor_cycles_per_wave_kmer"]
        k1["traffic_bytes_per_kmer_pmc"] = model.get("hbm_bytes_per_kmer_pmc")
        k1["peak_stale"] = (fp is None or fp != model.get("k1_fingerprint"))
        # three fractions of one kernel:
        #  frac_vs_guide_valu  K1's VALU instructions at MI355X_MICROARCH.md's
        #                      "2 cycles per wave64 VALU" (:54, :473): the
        #                      headline fraction
        #  frac_issue_model    the same instructions at the issue cost of
        #                      their class measured on this chip (2.3 / 4.2 /
        #                      5.0 cycles, scripts/ubench_dual.hip)
        #  hbm_frac            0.25 B per k-mer against 8 TB/s
        guide = N_SIMD * CLK_GHZ * 64 / (model["valu_per_wave_kmer"] * 2.0)
        k1["peak_guide_valu"] = guide
        k1["frac_vs_guide_valu"] = k1_gkmer / guide
        k1["peak_issue_model"] = model["peak_gkmer_per_s"]
        k1["frac_issue_model"] = k1_gkmer / model["peak_gkmer_per_s"]
        k1["peak"] = guide
        k1["frac"] = k1["frac_vs_guide_valu"]
    k2 = {"kernel": "K2: index_pairs_kernel (+ the bucketed index build) or pairs_gate_kernel", "unit": "Gpair/s",
          "achieved": pairs / (pr_ms * 1e-3) / 1e9 if pr_ms > 0 else 0.0, "avg_ms": pr_ms, "work_per_launch": pairs,
          "note": "pairs evaluated per second; K2's HBM roofline is the line's roofline_k2"}
    dom = k1 if sk_ms * kst_sk["launches"] >= pr_ms * kst_pr["launches"] else k2
    roof = {"bound": dom.get("bound", "valu"), "achieved": round(dom["achieved"], 3),
            "peak": round(dom.get("peak", 0.0), 3), "unit": dom["unit"],
            "frac": round(dom.get("frac", 0.0), 4),
            "frac_vs_guide_valu": round(dom["frac_vs_guide_valu"], 4) if "frac_vs_guide_valu" in dom else None,
            "frac_issue_model": round(dom["frac_issue_model"], 4) if "frac_issue_model" in dom else None,
            "hbm_frac": round(dom["hbm_frac"], 4) if "hbm_frac" in dom else None,
            "peak_stale": dom.get("peak_stale"),
            "traffic": (round(2 * model["hbm_bytes_per_kmer_pmc"] * kmers) if (model and dom is k1
                        and model.get("hbm_bytes_per_kmer_pmc")) else None),
            "kernel": dom["kernel"], "avg_launch_ms": round(dom["avg_ms"], 4),
            "note": ("K1 is bound by VALU issue, not HBM (hbm_frac: 0.25 B per k-mer at 8 TB/s). peak = 1024 SIMDs x "
                     "%.1f GHz x 64 k-mers / (K1's VALU instructions per wave-k-mer, PMC at HEAD, x 2 cycles: "
                     "MI355X_MICROARCH.md's wave64 VALU issue); frac_issue_model prices the same instructions at the "
                     "issue cost of their class measured on this chip (simple 32-bit ~2.3 cycles, other 32-bit ~4.2, "
                     "64-bit ~5.0; profiles/r04_k1_issue_model.json, DESIGN §4); traffic = HBM bytes per launch "
                     "from the PMC pass: FETCH_SIZE x 2 (the gfx950 factor, calibrated for 4-, 8- and 16-B loads by "
                     "scripts/ubench_fetch.hip) per k-mer x k-mers; %s"
                     % (CLK_GHZ, config_note)),
            "kernels": [{kk: (round(v, 5) if isinstance(v, float) else v) for kk, v in x.items()} for x in (k1, k2)]}
    return roof


# ---------------------------------------------------------------------------
# CPU baseline: the oracle on the host cores
# ---------------------------------------------------------------------------
def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_threads():
    """Every CPU this process can use (the CPU path on all host
    cores): the affinity mask, capped by the cgroup CPU quota (on the GPU
    box: 16 of the host's 256; scripts/host_cpus.py)."""
    return host_cpu_info()["usable"]


def cpu_baseline(sample_words, glen, sk_all, lens_all, k, s, min_ani, n_total, budget_s):
    """The CPU oracle (oracle/, a C restatement of finch as galah calls it)
    timed on this host on a bounded sample, extrapolated to the workload:
    sketching parallel over genomes on T threads (finch sketch_files is a
    rayon par_iter over files), the pair loop serial as src/finch.rs:53, and
    the pair loop on all T threads as the fairer upper bound."""
    import concurrent.futures as cf

    import oracle
    T = cpu_threads()
    words = sample_words
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    n_s = len(words) * 16 // glen
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
    # serial pair loop (src/finch.rs:53) over the first m genomes' sketches
    m = 200
    while True:
        t0 = time.perf_counter()
        oracle.pairs(sk_all[:m], lens_all[:m].astype(np.int32), min_ani, k=k, cap=m * m)
        t_p = time.perf_counter() - t0
        if t_p > budget_s / 4 or m >= min(3000, n_total):
            break
        m = min(min(3000, n_total), int(m * max(1.5, (budget_s / 4 / max(t_p, 1e-3)) ** 0.5)))
    pair_rate = m * (m - 1) / 2 / t_p
    # all-core pair loop over m2 genomes
    m2 = min(n_total, int(m * T ** 0.5))
    t0 = time.perf_counter()
    oracle.pairs_parallel(sk_all[:m2], lens_all[:m2].astype(np.int32), min_ani, k=k, threads=T)
    t_pp = time.perf_counter() - t0
    pair_rate_all = m2 * (m2 - 1) / 2 / t_pp
    npairs = n_total * (n_total - 1) / 2
    t_total = n_total * glen / sketch_bases_per_s + npairs / pair_rate
    t_total_all = n_total * glen / sketch_bases_per_s + npairs / pair_rate_all
    hi = host_cpu_info()
    # the same CPU path on every logical CPU of the host at the measured
    # per-thread rates (sketching is parallel over genomes, the all-core pair
    # loop over pairs): an upper bound for the CPU, as SMT threads are counted
    # as full cores; used when the quota keeps this process below nproc
    scale = (hi["nproc"] or T) / T
    t_total_host = n_total * glen / (sketch_bases_per_s * scale) + npairs / (pair_rate_all * scale)
    return {
        "value": npairs / t_total, "unit": "genome-pairs/s", "cores": T, "kind": "port",
        "cpu_model": cpu_model(), "nproc": hi["nproc"], "affinity_cpus": hi["affinity"],
        "cgroup_cpu_quota": hi["cgroup_cpu_quota"],
        "sample": ("oracle/ C restatement of finch on %d host threads (%s): sketched %d x %d bp synthetic genomes "
                   "of the workload (%.1f Mbases/s), serial pair loop (1 core, src/finch.rs:53) over %d genomes' "
                   "sketches (%.0f pairs/s), all-core pair loop over %d genomes (%.0f pairs/s); extrapolated to %d "
                   "genomes = %.0f s (serial pairs) / %.0f s (all-core pairs)"
                   % (T, cpu_model(), n_s, glen, sketch_bases_per_s / 1e6, m, pair_rate, m2, pair_rate_all,
                      n_total, t_total, t_total_all)),
        "sketch_mbases_per_s": sketch_bases_per_s / 1e6,
        "pair_rate_1core": pair_rate,
        "pair_rate_all_cores": pair_rate_all,
        "value_all_core_pairs": npairs / t_total_all,
        "value_all_host_cpus_extrapolated": npairs / t_total_host,
        "host_cpus_note": ("this process may use %d CPUs (affinity %s, cgroup quota %s of nproc %s); "
                           "value_all_host_cpus_extrapolated scales the measured per-thread sketch and all-core "
                           "pair rates linearly to all %s logical CPUs (an upper bound for the CPU path)"
                           % (T, hi["affinity"], hi["cgroup_cpu_quota"], hi["nproc"], hi["nproc"])),
    }


# ---------------------------------------------------------------------------
# ingest-inclusive leg: real gzip FASTA files through gg_precluster_files
# ---------------------------------------------------------------------------
def pcie_h2d_gbps(device, nbytes=1 << 30, reps=5):
    """The host-to-device PCIe rate of this box: a pinned host buffer copied
    to device memory by the DMA engine (torch), best of `reps` (the upload
    kernel that moves the ingest's staged batches reads mapped pinned memory
    over the same link, so this is its ceiling, not the 8 TB/s of HBM)."""
    src = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    dst = torch.empty(nbytes, dtype=torch.uint8, device="cuda:%d" % device)
    best = 0.0
    for _ in range(reps):
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize(device)
        best = max(best, nbytes / (time.perf_counter() - t0) / 1e9)
    del src, dst
    return best


def roofline_ingest(ks, wall_s, gz_bytes, text_bytes, pcie_gbps=None):
    """The device-inflate ingest priced kernel by kernel:
    HIP-event ms per call of each kernel class on the stream it ran on (one
    call with one processing lane, so no kernel shares the GPU with
    another), its algorithmic bytes against 8 TB/s HBM, and the PMC pass's
    VALU issue share and HBM bytes (profiles/r06/ingest_pmc.json, 1,000
    C2-like files).  Algorithmic bytes per call (G = gzip bytes, X = text
    bytes, T = tokens the decode wrote):
      upload  G (host -> device over PCIe: priced against the box's measured
              PCIe H2D rate, pcie_h2d_gbps, not HBM; not a candidate for
              the dominant HBM kernel)
      search  G read once
      decode  G read + 4 T (tokens written)
      expand  4 T read + 2 X (sym: u16 per text byte)
      resolve 3 X (sym read, the text written)
      crc     X
      parse   3.25 X (three passes over the text, X / 4 of packed words)"""
    G, X = float(gz_bytes), float(text_bytes)
    T = float(ks["decode"]["work"]) if ks.get("decode") else 0.0
    alg = {"upload": G, "search": G, "decode": G + 4 * T, "expand": 4 * T + 2 * X, "resolve": 3 * X, "crc": X,
           "parse": 3.25 * X}
    pmc = {}
    if os.path.exists(INGEST_PMC):
        with open(INGEST_PMC) as f:
            pk = json.load(f)["kernels"]
        merge = {"decode": ("decode_staged", "decode_global")}
        for name in alg:
            parts = merge.get(name, (name,))
            rows = [pk[p] for p in parts if p in pk]
            if not rows:
                continue
            ms = sum(r["ms_per_call"] for r in rows)
            hb = sum(r.get("hbm_bytes_per_call", 0.0) for r in rows)
            valu = sum(r["valu_frac_guide"] * r["ms_per_call"] for r in rows) / ms if ms else 0.0
            pmc[name] = {"ms_per_call": round(ms, 4), "valu_frac_guide": round(valu, 4),
                         "hbm_bytes_per_call": round(hb), "hbm_frac": round(hb / (ms * 1e-3) / 8e12, 4) if ms else 0.0,
                         "wait_frac": round(max(r["wait_frac"] for r in rows), 3)}
    kern = {}
    tot_ms = tot_alg = 0.0
    for name, b in alg.items():
        k = ks.get(name)
        if not k or not k["launches"]:
            continue
        ms = k["ms"]
        peak = pcie_gbps if (name == "upload" and pcie_gbps) else 8000.0
        e = {"ms_per_call": round(ms, 4), "launches": k["launches"], "algorithmic_bytes": round(b),
             "achieved_GBps": round(b / (ms * 1e-3) / 1e9, 2), "peak_GBps": round(peak, 2),
             "frac": round(b / (ms * 1e-3) / 1e9 / peak, 5), "bound": "pcie" if name == "upload" else "hbm"}
        if name in pmc:
            e["pmc"] = pmc[name]
        kern[name] = e
        tot_ms += ms
        tot_alg += b
    # the HBM-side kernels (upload reads host memory over PCIe: its own line)
    dev = {x: v for x, v in kern.items() if x != "upload"}
    dom = max(dev, key=lambda x: dev[x]["ms_per_call"]) if dev else None
    d_ms = sum(v["ms_per_call"] for v in dev.values())
    d_alg = sum(v["algorithmic_bytes"] for v in dev.values())
    traffic = sum(v.get("pmc", {}).get("hbm_bytes_per_call", 0) for v in dev.values()) or None
    return {"bound": "hbm", "unit": "GB/s", "peak": 8000.0,
            "achieved": round(d_alg / (d_ms * 1e-3) / 1e9, 2) if d_ms else None,
            "frac": round(d_alg / (d_ms * 1e-3) / 8e12, 5) if d_ms else None, "traffic": traffic,
            "algorithmic_bytes": round(d_alg), "traffic_over_algorithmic": round(traffic / d_alg, 3) if (traffic and d_alg) else None,
            "kernels_ms_per_call": round(tot_ms, 3), "device_kernels_ms_per_call": round(d_ms, 3),
            "call_s_one_lane": round(wall_s, 4), "dominant": dom,
            "upload": kern.get("upload"), "pcie_h2d_GBps": round(pcie_gbps, 2) if pcie_gbps else None,
            "kernels": kern,
            "note": "achieved = the device-memory ingest kernels' algorithmic bytes per call (docstring of "
                    "bench.py roofline_ingest) / their summed HIP-event time on their own streams, one call with "
                    "one lane (GALAHGPU_GZ_LANES=1); the default two lanes overlap these kernels; upload (host "
                    "memory over PCIe) is priced against pcie_h2d_GBps, the box's pinned H2D DMA rate; pmc: "
                    "profiles/r06/ingest_pmc.json (valu_frac_guide = VALU wave-instructions / (1024 SIMDs x "
                    "cycles / 2), hbm_bytes = FETCH_SIZE x 2 + WRITE_SIZE)"}


def bgzf_bytes(data, level=6, block=65280):
    """bgzip's output for data (BGZF, SAM/BAM specification 4.1): deflate
    members of <= 64 KB of input, each header carrying its size in the 'BC'
    extra subfield, then the empty end-of-file member."""
    import zlib
    out = []
    for i in range(0, max(len(data), 1), block):
        chunk = data[i:i + block]
        c = zlib.compressobj(level, zlib.DEFLATED, -15)
        body = c.compress(chunk) + c.flush()
        hdr = bytes([0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 66, 67, 2, 0]) + (len(body) + 25).to_bytes(2, "little")
        out.append(hdr + body + zlib.crc32(chunk).to_bytes(4, "little") + len(chunk).to_bytes(4, "little"))
    out.append(bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000"))
    return b"".join(out)


def files_leg(a, device, steps):
    """C2's genomes (1k x 3 Mbp, clusters of 10) written as FASTA files (80
    columns) to local disk OUTSIDE the timed region -- gzip (zlib level 6,
    one member), bgzip (BGZF, level 6) and plain -- then gg_precluster_files
    over each list (what galah's distances() calls: src/finch.rs:47-73) timed
    end to end.  gzip: the default device inflate, and the host inflate
    beside it; bgzip: the default device inflate (members from the headers);
    plain: the default (host threads read and pack) and the device parse
    (GALAHGPU_INFLATE=device).  Files are in the page cache (written just
    before).  Beside them: pure read + libdeflate gunzip of the gzip files
    on the same threads (scripts/gunzip_probe) and a pure read of the plain
    files, the floors any host ingest sits on."""
    import concurrent.futures as cf
    import shutil
    import tempfile
    import zlib

    n, glen, T = a.files_genomes, 3000000, cpu_threads()
    out = {"workload": "C2: %d synthetic genomes x %d bp as gzip FASTA (80 columns, zlib level 6), "
                       "k=21, s=1000, min_ani=%s" % (n, glen, float(ga.parse_percentage(a.min_ani))),
           "host_threads": T}
    plain_out = {}
    d = tempfile.mkdtemp(prefix="gg_files_", dir=os.environ.get("TMPDIR") or "/tmp")
    try:
        t0 = time.perf_counter()
        with ga.Context(k=21, sketch_size=1000, seed=0, device=device) as ctx:
            d_words = torch.empty(n * glen // 16, dtype=torch.int32, device="cuda:%d" % device)
            ctx.synth_device(n, glen, a.cluster, a.max_sub, a.seed, d_words)
            torch.cuda.synchronize(device)
            words = d_words.cpu().numpy().view(np.uint32)
            del d_words
        acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
        shifts = (np.uint32(30) - 2 * np.arange(16, dtype=np.uint32))[None, :]
        nl = np.full((glen // 80, 1), ord("\n"), np.uint8)
        for f in ("gz", "bgzf", "plain"):
            os.makedirs(os.path.join(d, f))

        def write(g):
            w = words[g * glen // 16:(g + 1) * glen // 16]
            seq = acgt[((w[:, None] >> shifts) & np.uint32(3)).reshape(-1)]
            body = np.concatenate([seq[: glen // 80 * 80].reshape(-1, 80), nl], axis=1).tobytes()
            text = b">genome_%d synthetic C2\n" % g + body + (bytes(seq[glen // 80 * 80:]) + b"\n" if glen % 80 else b"")
            c = zlib.compressobj(6, zlib.DEFLATED, 31)
            ps = {f: os.path.join(d, f, "g%05d.fna" % g + ("" if f == "plain" else ".gz")) for f in ("gz", "bgzf", "plain")}
            with open(ps["gz"], "wb") as fh:
                fh.write(c.compress(text) + c.flush())
            with open(ps["bgzf"], "wb") as fh:
                fh.write(bgzf_bytes(text))
            with open(ps["plain"], "wb") as fh:
                fh.write(text)
            return ps

        with cf.ThreadPoolExecutor(T) as ex:
            written = list(ex.map(write, range(n)))
        del words
        lists = {f: [w[f] for w in written] for f in ("gz", "bgzf", "plain")}
        paths = lists["gz"]
        out["write_s"] = round(time.perf_counter() - t0, 2)
        out["gz_bytes"] = int(sum(os.path.getsize(p) for p in paths))
        print("[bench] files leg: wrote %d gzip, bgzip and plain FASTA files (%.2f GB gzip) in %.1f s"
              % (n, out["gz_bytes"] / 1e9, out["write_s"]), file=sys.stderr, flush=True)
        thr = ga.parse_percentage(a.min_ani)
        bases = n * glen
        ingest = []

        def timed(plist, inflate, kernel_timing=False):
            """gg_precluster_files over plist, GALAHGPU_INFLATE=inflate (None: the default)."""
            if inflate:
                os.environ["GALAHGPU_INFLATE"] = inflate
            try:
                with ga.Context(k=21, sketch_size=1000, seed=0, device=device, host_threads=T) as ctx:
                    ctx.precluster_files(plist, thr)  # warm-up: one untimed call (device buffers sized for the batches)
                    times, found, ph = [], 0, {p: 0.0 for p in ga.PHASES}
                    for _ in range(max(1, steps)):
                        t1 = time.perf_counter()
                        pairs, _ani = ctx.precluster_files(plist, thr)
                        times.append(time.perf_counter() - t1)
                        found = len(pairs)
                        for p, v in ctx.phase_times().items():
                            ph[p] += v
                    ctx.timing_enable(True)  # (one more call, untimed: K1's HIP-event time per call)
                    ctx.precluster_files(plist, thr)
                    k1 = ctx.timing_read(ga.KERNEL_SKETCH)
                    ctx.timing_enable(False)
                    fb = ctx.fallbacks()["inflate_host"]
                    info = ctx.info_line()
                    if kernel_timing:  # one more call, timed kernel by kernel (one lane: no overlap)
                        os.environ["GALAHGPU_GZ_LANES"] = "1"
                        try:
                            ctx.timing_enable(True)
                            t1 = time.perf_counter()
                            ctx.precluster_files(plist, thr)
                            w1 = time.perf_counter() - t1
                            kst = {name: ctx.timing_read(k) for name, k in ga.INGEST_KERNELS.items()}
                            kst["k1"] = ctx.timing_read(ga.KERNEL_SKETCH)
                            ctx.timing_enable(False)
                        finally:
                            os.environ.pop("GALAHGPU_GZ_LANES", None)
                        ingest[:] = [kst, w1]
            finally:
                os.environ.pop("GALAHGPU_INFLATE", None)
            t = float(np.median(times))
            return {"steps": len(times), "s_per_call_median": round(t, 4), "s_per_call_max": round(max(times), 4),
                    "max_over_median": round(max(times) / t, 3), "s_per_call": [round(x, 4) for x in times],
                    "gbases_per_s": round(bases / t / 1e9, 3), "genome_pairs_per_s": round(n * (n - 1) / 2 / t, 1),
                    "pairs_found": int(found), "phase_ms": {p: round(v / len(times), 2) for p, v in ph.items()},
                    "k1_ms_per_call": round(k1["ms"], 3),
                    "inflate_host_batches": fb, "info_line": info}, pairs

        # the default path for gzip files: inflated on the GPU (inflate.hip), the host threads only read
        dev, dp = timed(paths, "device", kernel_timing=True)
        out.update(dev)
        if ingest:
            text_bytes = sum(len(b">genome_%d synthetic C2\n" % g) for g in range(n)) + n * (glen + glen // 80)
            try:
                pcie = pcie_h2d_gbps(device)
            except Exception:
                pcie = None
            out["roofline_ingest"] = roofline_ingest(ingest[0], ingest[1], out["gz_bytes"], text_bytes, pcie)
        out["inflate"] = "device"
        t = dev["s_per_call_median"]
        # the same files gunzipped and packed on the host threads (GALAHGPU_INFLATE=host, round 3's path)
        host, hp = timed(paths, "host")
        out["host_inflate"] = host
        out["same_pairs_as_host_inflate"] = bool(np.array_equal(hp, dp))
        out["device_over_host_inflate"] = round(host["s_per_call_median"] / t, 3)
        # bgzip (BGZF members from their headers), the default path
        bg, bp = timed(lists["bgzf"], None)
        bg["bgzf_bytes"] = int(sum(os.path.getsize(p) for p in lists["bgzf"]))
        bg["same_pairs_as_gzip"] = bool(np.array_equal(bp, dp))
        out["bgzip"] = bg
        probe = os.path.join(ROOT, "scripts", "gunzip_probe")
        if os.path.exists(probe):
            r = subprocess.run([probe, str(T)] + paths, capture_output=True, text=True, timeout=300)
            if r.returncode == 0:
                dec = json.loads(r.stdout.strip().splitlines()[-1])
                out["pure_decode_s"] = dec["decode_s"]
                out["pure_decode_gbases_per_s"] = round(bases / dec["decode_s"] / 1e9, 3)
                out["ratio_to_pure_decode"] = round(t / dec["decode_s"], 3)
            else:
                out["pure_decode_error"] = r.stderr[-300:]
        out["note"] = ("kernel-only headline vs this: the same path from gzip files on %d host threads; galah's "
                       "distances() starts from these paths (src/finch.rs:47); top level: the default for gzip "
                       "files, gzip bytes to the GPU, inflated and parsed there (inflate.hip, parse.hip), the host "
                       "threads only read; host_inflate: gunzip + parse + pack on the host threads "
                       "(GALAHGPU_INFLATE=host); bgzip: the same genomes as BGZF files (device inflate, one unit "
                       "per member); pure_decode: read + libdeflate gunzip alone on the same threads" % T)
        # plain FASTA (the reference's own fixtures: tests/data/*.fna): the
        # default (read + parse + 2-bit pack on the host threads, packed words
        # to the device) and the device parse (text to the device)
        pl = lists["plain"]
        text_total = int(sum(os.path.getsize(p) for p in pl))

        def pure_read():
            def rd(p):
                with open(p, "rb", buffering=0) as fh:
                    return len(fh.read())
            t1 = time.perf_counter()
            with cf.ThreadPoolExecutor(T) as ex:
                got = sum(ex.map(rd, pl))
            return time.perf_counter() - t1, got

        pure_read()  # (warm)
        rs = min(pure_read()[0] for _ in range(3))
        dflt, p0 = timed(pl, None)
        devp, p1 = timed(pl, "device")
        plain_out = {"workload": out["workload"].replace("as gzip FASTA (80 columns, zlib level 6)",
                                                           "as plain FASTA (80 columns)"),
                     "text_bytes": text_total, "host_threads": T,
                     "default": dflt, "device_parse": devp,
                     "gbases_per_s": dflt["gbases_per_s"],
                     "pure_read_s": round(rs, 4), "pure_read_GBps": round(text_total / rs / 1e9, 2),
                     "same_pairs_as_gzip": bool(np.array_equal(p0, dp) and np.array_equal(p1, dp)),
                     "split_ms": {"pure_read_floor": round(rs * 1e3, 2),
                                  "sketch_phase": dflt["phase_ms"]["sketch"], "k1_kernel": dflt["k1_ms_per_call"],
                                  "pairs_phase": dflt["phase_ms"]["pairs"], "merge_phase": dflt["phase_ms"]["merge"]},
                     "note": "default: the host threads read, parse and 2-bit pack (pack.cpp), packed words go to "
                             "the device, K1 + K2 there; device_parse (GALAHGPU_INFLATE=device): the text goes to the "
                             "device and parse.hip packs it; split_ms: the pure read of the same files on the same "
                             "threads (page cache), the sketch phase (read + pack + upload + K1, overlapped), K1's "
                             "HIP-event time, K2 + D2H, merge"}
    finally:
        shutil.rmtree(d, ignore_errors=True)
    return out, plain_out


# ---------------------------------------------------------------------------
def workload_note(a, N, total_bases, min_ani, s):
    w = (("C5: %d synthetic genomes of 0.5-12 Mbp (log-uniform, %.0f bp total) with N runs" % (N, total_bases))
         if a.config == "c5" else ("%s: %d synthetic genomes x %d bp" % (a.config.upper(), N, a.genome_len)))
    return w + ", clusters of %d, sub rate U(0,%.2f), k=%d, s=%d, min_ani=%s" % (a.cluster, a.max_sub, a.k, s,
                                                                                 min_ani)


def c4_leg(a, device):
    """The north-star workload on one GPU (BASELINE.json configs[3]: 100k
    synthetic 3 Mbp genomes, s=1000, min_ani f32(0.95); src/finch.rs:53-73
    over all 5e9 pairs): one warm-up and a.c4_steps timed steps of the same
    gg_precluster_shards call as the headline, inputs resident in HBM (75 GB
    of packed words), K1 / K2 HIP-event times and both rooflines.  The
    node's 8-GPU curve extends this N=1 point."""
    import copy
    b = copy.copy(a)
    b.config, b.genomes = "c4", 100000
    N, s = b.genomes, 1000
    min_ani = ga.parse_percentage(b.min_ani)
    t0 = time.perf_counter()
    ctx = ga.Context(k=b.k, sketch_size=s, seed=0, device=device)
    try:
        d_words, runs, bases = make_shard(ctx, b, 0, N, device)
        d_runs = ga.device_runs(runs, "cuda:%d" % device)
        shards = [(d_words, d_runs, N)]
        torch.cuda.synchronize(device)
        synth_s = time.perf_counter() - t0
        ctx.precluster_shards(shards, min_ani)  # warm-up
        ctx.timing_enable(True)
        torch.cuda.synchronize(device)
        times, ph = [], {p: 0.0 for p in ga.PHASES}
        found = 0
        for _ in range(max(1, b.c4_steps)):
            t1 = time.perf_counter()
            pairs, _ani = ctx.precluster_shards(shards, min_ani)
            torch.cuda.synchronize(device)
            times.append(time.perf_counter() - t1)
            found = len(pairs)
            for p, v in ctx.phase_times().items():
                ph[p] += v
        kst = {name: ctx.timing_read(kid) for name, kid in
               (("sketch", ga.KERNEL_SKETCH), ("finalize", ga.KERNEL_FINALIZE), ("pairs", ga.KERNEL_PAIRS),
                ("index", ga.KERNEL_PAIRS_INDEX))}
        kst["pairs"]["ms"] += kst["index"]["ms"]
        ctx.timing_enable(False)
        steps = len(times)
        roof = roofline(kst["sketch"], kst["pairs"], s, "C4 on one GPU")
        d_sk = torch.zeros((N, s), dtype=torch.int64, device="cuda:%d" % device)
        d_len = torch.zeros(N, dtype=torch.int32, device="cuda:%d" % device)
        ctx.sketch_device(d_words, d_runs, N, d_sk, d_len)
        torch.cuda.synchronize(device)
        kp = dict(kst["pairs"])
        kp["launches_sets"] = kst["pairs"]["launches"]
        roof_k2 = roofline_k2(k2_algorithmic_bytes(d_sk, d_len, N, s), kp, None)
        paths = ctx.pair_paths()
        fb = ctx.fallbacks()
        del d_sk, d_len, shards, d_words, d_runs
    finally:
        ctx.close()
        torch.cuda.empty_cache()
    ms = float(np.mean(times)) * 1e3
    npairs = N * (N - 1) // 2
    return {"workload": workload_note(b, N, bases, min_ani, s), "genomes": N, "steps": steps, "warmup": 1,
            "ms_per_step": round(ms, 3), "ms_per_step_all": [round(x * 1e3, 3) for x in times],
            "genome_pairs_per_s": round(npairs / (ms * 1e-3), 1), "pairs_found": found,
            "sketch_gbases_per_s": round(bases / (ph["sketch"] / steps * 1e-3) / 1e9, 3),
            "phase_ms": {p: round(v / steps, 3) for p, v in ph.items()},
            "kernel_ms_per_step": {"k1": round(kst["sketch"]["ms"] / steps, 3),
                                   "finalize": round(kst["finalize"]["ms"] / steps, 3),
                                   "k2": round(kst["pairs"]["ms"] / steps, 3)},
            "roofline": roof, "roofline_k2": roof_k2, "pair_paths": paths,
            "fallbacks": fb, "synth_s": round(synth_s, 2),
            "note": "the north-star scale (100k genomes, s=1000) on ONE MI355X, inputs resident in HBM; "
                    "BASELINE's target is >= 1e9 genome-pairs/s node-wide"}


def run_lib(a, world, rank):
    """One process drives every device through gg_precluster_shards."""
    if world > 1:
        dist.init_process_group("gloo")
    N, s = a.genomes, a.sketch
    min_ani = ga.parse_percentage(a.min_ani)
    n_dev = a.gpus if world == 1 else world
    line = None
    if rank == 0:
        devs = [int(x) for x in a.devices.split(",")] if a.devices else list(range(n_dev))
        ctx = ga.Context(k=a.k, sketch_size=s, seed=0, devices=devs) if len(devs) > 1 else \
            ga.Context(k=a.k, sketch_size=s, seed=0, device=devs[0])
        M = ctx.device_count
        shards, total_bases, keep = [], 0, []
        for m in range(M):
            g0, g1 = sharding.shard_range(N, M, m)
            torch.cuda.set_device(devs[m])
            d_words, runs, bases = make_shard(ctx.member(m), a, g0, g1, devs[m])
            # the run table is input too: resident on the member's device like the words
            shards.append((d_words, ga.device_runs(runs, "cuda:%d" % devs[m]), g1 - g0))
            keep.append(d_words)
            total_bases += bases
        sync_all(devs)
        for _ in range(a.warmup):
            ctx.precluster_shards(shards, min_ani)
        phase = {p: 0.0 for p in ga.PHASES}
        m0 = ctx.member(0)
        m0.timing_enable(True)
    if world > 1:
        dist.barrier()
    if rank == 0:
        sync_all(devs)
    t0 = time.perf_counter()
    found = 0
    if rank == 0:
        for _ in range(a.steps):
            pairs, ani = ctx.precluster_shards(shards, min_ani)
            found = len(pairs)
            for p, v in ctx.phase_times().items():
                phase[p] += v
        sync_all(devs)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed_max = float(t[0])
    if rank == 0:
        kst = {name: m0.timing_read(kid) for name, kid in
               (("sketch", ga.KERNEL_SKETCH), ("finalize", ga.KERNEL_FINALIZE), ("pairs", ga.KERNEL_PAIRS),
                ("index", ga.KERNEL_PAIRS_INDEX))}
        kst["pairs"]["ms"] += kst["index"]["ms"]  # the index kernel's sort + run pass belong to K2
        m0.timing_enable(False)
        ms_step = elapsed_max / a.steps * 1e3
        npairs = N * (N - 1) // 2
        note = ("per-launch figures are device 0's (%d of %d genomes)" % (shards[0][2], N)) if M > 1 else ""
        roof = roofline(kst["sketch"], kst["pairs"], s, note)
        pmc_config = a.config if M == 1 and N == {"c3": 10000, "c5": 10000}.get(a.config) else None
        downstream = None
        if M == 1 and found:
            t1 = time.perf_counter()
            members, offsets = ga.partition_preclusters(N, pairs)
            t_part = time.perf_counter() - t1
            t1 = time.perf_counter()
            ga.precluster_pairs(N, pairs, members, offsets)
            t_tr = time.perf_counter() - t1
            downstream = {"partition_preclusters_ms": round(t_part * 1e3, 3), "precluster_pairs_ms":
                          round(t_tr * 1e3, 3), "preclusters": int(len(offsets) - 1),
                          "largest": int(np.diff(offsets).max()) if N else 0}
        cpu = None
        roof_k2 = None
        d_sk = d_len = None
        if M == 1:  # the step's sketches, for K2's byte model and the CPU baseline's parity spot check
            d_words, runs, _ = shards[0]
            d_sk = torch.zeros((N, s), dtype=torch.int64, device="cuda:%d" % devs[0])
            d_len = torch.zeros(N, dtype=torch.int32, device="cuda:%d" % devs[0])
            ctx.sketch_device(d_words, runs, N, d_sk, d_len)
            torch.cuda.synchronize()
            kp = dict(kst["pairs"])
            kp["launches_sets"] = kst["pairs"]["launches"]
            roof_k2 = roofline_k2(k2_algorithmic_bytes(d_sk, d_len, N, s), kp, pmc_config)
        if world == 1 and M == 1 and not a.no_cpu_baseline and a.config in ("c2", "c3", "c4"):
            n_sample = cpu_threads()
            sample = d_words[: n_sample * a.genome_len // 16].cpu().numpy().view(np.uint32)
            cpu = cpu_baseline(sample, a.genome_len, d_sk.cpu().numpy().view(np.uint64),
                               d_len.cpu().numpy().view(np.uint32), a.k, s, min_ani, N, a.cpu_budget_s)
        del d_sk, d_len
        pair_paths, fallbacks = ctx.pair_paths(), ctx.fallbacks()
        # the headline workload's context and inputs are released before the
        # files leg, which is a separate call as galah makes it in a fresh
        # process (with the C3 context and its ~10 GB of inputs still held, the
        # same calls measured 0.073 s against 0.061-0.065 in a fresh process:
        # scripts/files_data_ab.py, gpurun_out r6e/r6f)
        ctx.close()
        ctx = None
        del shards, keep, d_words, runs
        torch.cuda.empty_cache()
        files = files_plain = c4 = None
        want_files = a.files if a.files is not None else (a.config == "c3")
        if world == 1 and M == 1 and want_files:
            try:
                files, files_plain = files_leg(a, devs[0], 9)
            except Exception as e:  # the headline stands without it
                files = {"error": "%s: %s" % (type(e).__name__, e)}
        want_c4 = a.c4_leg if a.c4_leg is not None else (a.config == "c3")
        if world == 1 and M == 1 and want_c4:
            try:
                c4 = c4_leg(a, devs[0])
            except Exception as e:  # the headline stands without it
                c4 = {"error": "%s: %s" % (type(e).__name__, e)}
        line = {
            "metric": "precluster genome-pairs/sec at 10k genomes (s=1000) + sketch Gbases/s",
            "value": round(npairs / (elapsed_max / a.steps), 1), "unit": "genome-pairs/s", "n_gpus": n_dev,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "u64",
            "data": "synthetic clustered genomes generated on device (no network)",
            "config": {"workload": workload_note(a, N, total_bases, min_ani, s), "genomes": N,
                       "genome_len": (None if a.config == "c5" else a.genome_len), "sketch_size": s, "k": a.k,
                       "min_ani": float(min_ani), "parallelism": "dp%d" % M, "mode": "lib",
                       "devices": devs},
            "sketch_gbases_per_s": round(total_bases / (phase["sketch"] / a.steps * 1e-3) / 1e9, 3),
            "phase_ms": {p: round(v / a.steps, 3) for p, v in phase.items()},
            # device time per step of K1, its finalize and K2 (index build + pairs kernel), device 0
            "kernel_ms_per_step": {"k1": round(kst["sketch"]["ms"] / a.steps, 3),
                                   "finalize": round(kst["finalize"]["ms"] / a.steps, 3),
                                   "k2": round(kst["pairs"]["ms"] / a.steps, 3)},
            "pairs_found": found,
            "pair_paths": pair_paths,
            "fallbacks": fallbacks,
            "roofline": roof,
            "roofline_k2": roof_k2,
            "cpu_baseline": cpu,
            "downstream": downstream,
            "files": files,
            "files_plain": files_plain,
            "c4_one_gpu": c4,
        }
    if world > 1:
        dist.destroy_process_group()
    return line


def run_dist(a, world, rank, local):
    """One process per GPU; RCCL all-gather of the sketches (galah_amd/sharding.py)."""
    gloo = a.dist_backend == "gloo"
    if gloo:
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        if gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    N, s = a.genomes, a.sketch
    g0, g1 = sharding.shard_range(N, world, rank)
    n_loc = g1 - g0
    even = N % world == 0
    min_ani = ga.parse_percentage(a.min_ani)
    ctx = ga.Context(k=a.k, sketch_size=s, seed=0, device=local)
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    d_words, runs, bases_loc = make_shard(ctx, a, g0, g1, local)
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

    def step():
        ctx.sketch_device(d_words, runs, n_loc, d_sk_loc, d_len_loc, stream=sh)
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
        d_cnt.zero_()
        ctx.pairs_device(d_sk, d_len, N, tb, te, min_ani, d_out, cap, d_cnt, stream=sh)
        cnt = int(d_cnt.item())
        if cnt > cap:
            raise RuntimeError("pair buffer too small: %d > %d" % (cnt, cap))
        return cnt, d_out[: cnt * 4].cpu()

    for _ in range(a.warmup):
        step()
    ctx.timing_enable(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    found = 0
    for _ in range(a.steps):
        found, _h = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kst = {name: ctx.timing_read(kid) for name, kid in
           (("sketch", ga.KERNEL_SKETCH), ("pairs", ga.KERNEL_PAIRS), ("index", ga.KERNEL_PAIRS_INDEX))}
    kst["pairs"]["ms"] += kst["index"]["ms"]
    ctx.timing_enable(False)
    t = torch.tensor([elapsed, float(found), float(bases_loc)], dtype=torch.float64,
                     device="cpu" if gloo else "cuda")
    tmax, tsum = t.clone(), t.clone()
    if world > 1:
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
    line = None
    if rank == 0:
        elapsed_max = float(tmax[0])
        npairs = N * (N - 1) // 2
        line = {
            "metric": "precluster genome-pairs/sec at 10k genomes (s=1000) + sketch Gbases/s",
            "value": round(npairs / (elapsed_max / a.steps), 1), "unit": "genome-pairs/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(elapsed_max / a.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u64",
            "data": "synthetic clustered genomes generated on device (no network)",
            "config": {"workload": workload_note(a, N, float(tsum[2]), min_ani, s), "genomes": N,
                       "sketch_size": s, "k": a.k, "min_ani": float(min_ani), "parallelism": "dp%d" % world,
                       "mode": "dist"},
            "pairs_found": int(tsum[1]),
            "roofline": roofline(kst["sketch"], kst["pairs"], s, "rank 0's launches"),
            "cpu_baseline": None,
        }
    ctx.close()
    if world > 1:
        dist.destroy_process_group()
    return line


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    mode = a.mode
    if mode == "lib" and world > 1 and not a.devices and torch.cuda.device_count() < world:
        # a launcher that shows each rank only its own GPU: one process per
        # GPU with the RCCL all-gather instead of one process driving all
        mode = "dist"
    line = run_lib(a, world, rank) if mode == "lib" else run_dist(a, world, rank, local)
    if rank == 0 and line is not None:
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
