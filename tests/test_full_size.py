"""Parity at the BASELINE.json configs, at full size, on one MI355X.

  C3  10,000 x 3 Mbp genomes, s = 1000, min_ani = f32(0.95)   (the headline)
  C4  100,000 x 3 Mbp genomes, s = 1000, min_ani = f32(0.95)  (one-GPU shape of the 8-GPU config)
  C5  10,000 genomes of 0.5-12 Mbp (log-uniform) with N runs, s = 10000

Each config is generated on the device (galah_amd synthetic clustered genomes,
clusters of 10, member substitution rate ~ U(0, 0.07)), sketched by K1 and
paired by K2 through the C ABI, then checked (src/finch.rs:47 and :53-73 are
the reference loops; the oracle restates them):

  * sketch properties: every row full (len = s) and strictly ascending;
  * sketches bit-exact with the oracle on 8+ genomes, including the smallest
    and the largest;
  * (common, total) bit-exact and the pass decision equal for EVERY pair
    inside a cluster (45 per cluster: these are all the pairs whose ANI is
    near the cutoff; every one within +-3 of cmin[total] is among them and
    counted), and for 2,000 random pairs across clusters;
  * the default pair kernel's (the inverted index at these sizes) pair set
    equal to the gate kernel's and to the independent merge kernel's
    (GALAHGPU_PAIRS_KERNEL=merge, one lane per pair, the literal merge) over
    a band of 1,024 rows against all columns.
"""
import concurrent.futures as cf
import os

import numpy as np
import pytest

import galah_amd as ga
import oracle
from conftest import xcheck_module
from test_host import ACGT

pytestmark = pytest.mark.gpu

CLUSTER = 10
MAX_SUB = 0.07


def torch_dev():
    import torch
    assert torch.cuda.is_available()
    return torch


def unpack_device_run(d_words, base, length):
    """ASCII bases [base, base + length) of a device-resident 2-bit stream."""
    w0 = base // 16
    w1 = (base + length + 15) // 16
    words = d_words[w0:w1].cpu().numpy().view(np.uint32)
    idx = np.arange(base - 16 * w0, base - 16 * w0 + length, dtype=np.uint64)
    w = words[(idx >> np.uint64(4)).astype(np.int64)]
    sh = np.uint32(30) - np.uint32(2) * (idx & np.uint64(15)).astype(np.uint32)
    return ACGT[(w >> sh) & np.uint32(3)].tobytes()


def smallest_passing_common(t, cmax, thr64):
    """Smallest common c <= cmax with oracle ani(c, t) >= thr (ani rises with c), or None."""
    if t == 0 or oracle.ani(cmax, t) < thr64:
        return None
    lo, hi = -1, cmax
    while hi - lo > 1:
        mid = (lo + hi) // 2
        if oracle.ani(mid, t) >= thr64:
            hi = mid
        else:
            lo = mid
    return hi


def tile_row_range(n, row0, rows):
    """Tile range [tb, te) covering the tile rows of rows [row0, row0 + rows)."""
    nb = (n + ga.GG_PAIR_TILE - 1) // ga.GG_PAIR_TILE
    I0 = row0 // ga.GG_PAIR_TILE
    I1 = min(nb, (row0 + rows + ga.GG_PAIR_TILE - 1) // ga.GG_PAIR_TILE)
    tb = sum(nb - I for I in range(I0))
    te = tb + sum(nb - I for I in range(I0, I1))
    return tb, te


def device_pairs(ctx, d_sk, d_len, n, tb, te, thr):
    torch = torch_dev()
    cap = max(1 << 20, 64 * n)
    d_out = torch.empty(cap * 4, dtype=torch.int32, device="cuda")
    d_cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    ctx.pairs_device(d_sk, d_len, n, tb, te, thr, d_out, cap, d_cnt)
    torch.cuda.synchronize()
    c = int(d_cnt.item())
    assert c <= cap
    p = d_out[:c * 4].cpu().numpy().view(np.uint32).reshape(-1, 4)
    return p[np.lexsort((p[:, 1], p[:, 0]))]


def check_config(ctx, d_words, runs, n, s, thr, genome_bases, spot):
    torch = torch_dev()
    d_sk = torch.zeros((n, s), dtype=torch.int64, device="cuda")
    d_len = torch.zeros(n, dtype=torch.int32, device="cuda")
    ctx.sketch_device(d_words, runs, n, d_sk, d_len)
    torch.cuda.synchronize()
    sk = d_sk.cpu().numpy().view(np.uint64)
    ln = d_len.cpu().numpy().view(np.uint32)
    # properties
    assert (ln == s).all()
    assert (sk[:, 1:] > sk[:, :-1]).all()
    # oracle sketches: smallest, largest and a spread of others
    order = np.argsort(genome_bases, kind="stable")
    picks = sorted(set([int(order[0]), int(order[-1])] + [int(x) for x in spot]))
    assert len(picks) >= 8
    g_of_run = runs["genome"]

    def oracle_sketch(g):
        recs = [unpack_device_run(d_words, int(r["base"]), int(r["len"])) for r in runs[g_of_run == g]]
        return g, oracle.sketch_records(recs, s=s)

    with cf.ThreadPoolExecutor(8) as ex:
        outs = list(ex.map(oracle_sketch, picks))
    for g, exp in outs:
        assert len(exp) == ln[g] and (sk[g][:ln[g]] == exp).all(), g

    # all pairs on the device, through the inverted index to completion (the
    # default at these sizes; an abandoned index would fall back to the gate
    # kernel with the same pairs, hiding a broken index)
    before = ctx.pair_paths()
    P = device_pairs(ctx, d_sk, d_len, n, 0, ga.pair_tiles(n), thr)
    after = ctx.pair_paths()
    assert after["index"] == before["index"] + 1 and after["index_abandoned"] == before["index_abandoned"]
    assert after["gate"] == before["gate"]
    assert after["index_full_sort"] == before["index_full_sort"]  # the bucketed build
    got = {(int(a), int(b)): (int(c), int(t)) for a, b, c, t in P}
    assert len(got) == len(P)
    # every within-cluster pair against the oracle
    ii, jj = [], []
    for c0 in range(0, n, CLUSTER):
        m = min(CLUSTER, n - c0)
        a, b = np.triu_indices(m, 1)
        ii.append(a + c0)
        jj.append(b + c0)
    ii = np.concatenate(ii).astype(np.uint32)
    jj = np.concatenate(jj).astype(np.uint32)
    oc, ot = oracle.pair_list(sk, ln.astype(np.int32), ii, jj)
    thr64 = np.float64(np.float32(thr))
    opass = oracle.ani_array(oc, ot) >= thr64
    cmin = {}
    near = 0
    for x in range(len(ii)):
        key = (int(ii[x]), int(jj[x]))
        if opass[x]:
            assert got.get(key) == (int(oc[x]), int(ot[x])), key
        else:
            assert key not in got, key
        t = int(ot[x])
        if t not in cmin:
            cmin[t] = smallest_passing_common(t, min(t, s), thr64)
        if cmin[t] is not None and abs(int(oc[x]) - cmin[t]) <= 3:
            near += 1
    assert opass.any() and not opass.all()
    # random pairs across clusters
    rng = np.random.default_rng(n + s)
    ri = rng.integers(0, n, 4000).astype(np.uint32)
    rj = rng.integers(0, n, 4000).astype(np.uint32)
    keep = (ri // CLUSTER) != (rj // CLUSTER)
    ri, rj = np.minimum(ri, rj)[keep][:2000], np.maximum(ri, rj)[keep][:2000]
    xc, xt = oracle.pair_list(sk, ln.astype(np.int32), ri, rj)
    xpass = oracle.ani_array(xc, xt) >= thr64
    for x in range(len(ri)):
        key = (int(ri[x]), int(rj[x]))
        assert (key in got) == bool(xpass[x]), key
        if xpass[x]:
            assert got[key] == (int(xc[x]), int(xt[x]))
    # the gate kernel vs the merge kernel over a 1,024-row band
    row0 = (n // 2) // ga.GG_PAIR_TILE * ga.GG_PAIR_TILE
    tb, te = tile_row_range(n, row0, 1024)
    band_gate = device_pairs(ctx, d_sk, d_len, n, tb, te, thr)
    old = os.environ.get("GALAHGPU_PAIRS_KERNEL")
    bands = {}
    try:
        for kern in ("merge", "gate", "index"):
            os.environ["GALAHGPU_PAIRS_KERNEL"] = kern
            # (merge: the cross-check kernel of the test build)
            with (xcheck_module() if kern == "merge" else ga).Context(k=21, sketch_size=s) as mctx:
                bands[kern] = device_pairs(mctx, d_sk, d_len, n, tb, te, thr)
                if kern == "index":
                    assert mctx.pair_paths() == {"index": 1, "index_abandoned": 0, "gate": 0, "other": 0,
                                                 "index_full_sort": 0}
    finally:
        if old is None:
            os.environ.pop("GALAHGPU_PAIRS_KERNEL")
        else:
            os.environ["GALAHGPU_PAIRS_KERNEL"] = old
    for kern in bands:
        assert np.array_equal(band_gate, bands[kern]), kern
    in_band = (P[:, 0] >= row0) & (P[:, 0] < row0 + 1024)
    assert np.array_equal(P[in_band], band_gate)
    print("\n%d genomes, s=%d: %d passing pairs, %d within-cluster pairs checked (%d pass, %d within +-3 of "
          "cmin), %d cross-cluster pairs, band of 1024 rows: %d pairs default == gate == index == merge"
          % (n, s, len(P), len(ii), int(opass.sum()), near, len(ri), len(band_gate)))
    assert near > 0
    del d_sk, d_len
    return P


def synth_uniform(ctx, n, glen, seed):
    torch = torch_dev()
    d_words = torch.empty(n * glen // 16, dtype=torch.int32, device="cuda")
    runs = ctx.synth_device(n, glen, CLUSTER, MAX_SUB, seed, d_words)
    torch.cuda.synchronize()
    return d_words, runs


def test_c3_full_size(gpu_ctx):
    """C3: 10k x 3 Mbp at parse_percentage(95) (BASELINE.json configs[2], bench.py's workload)."""
    n, glen = 10000, 3000000
    d_words, runs = synth_uniform(gpu_ctx, n, glen, 3)
    spot = [1, 2, 4999, 5000, 7777, 9998]
    check_config(gpu_ctx, d_words, runs, n, 1000, ga.parse_percentage(95), np.full(n, glen), spot)


def test_c4_shape_one_gpu():
    """C4 shape on one GPU: 100k x 3 Mbp, s = 1000, parse_percentage(95)
    (75 GB of packed genomes in HBM)."""
    torch = torch_dev()
    n, glen = 100000, 3000000
    with ga.Context(k=21, sketch_size=1000) as ctx:
        d_words, runs = synth_uniform(ctx, n, glen, 5)
        spot = [1, 12345, 49999, 50000, 77777, 99990]
        check_config(ctx, d_words, runs, n, 1000, ga.parse_percentage(95), np.full(n, glen), spot)
        del d_words
    torch.cuda.empty_cache()


def test_c5_full_size():
    """C5: 10k genomes of 0.5-12 Mbp (log-uniform per cluster) with N runs
    (0.01% per base, 1-64 long), s = 10000, parse_percentage(95)."""
    torch = torch_dev()
    n, s = 10000, 10000
    lens_bp = ga.synth_mixed_lengths(n, 500000, 12000000, CLUSTER, 7)
    d_words = torch.empty(int(lens_bp.sum()) // 16, dtype=torch.int32, device="cuda")
    with ga.Context(k=21, sketch_size=s) as ctx:
        runs = ctx.synth_mixed_device(lens_bp, CLUSTER, MAX_SUB, 1e-4, 8, d_words)
        torch.cuda.synchronize()
        assert len(runs) > n
        spot = [3, 1234, 5000, 6789, 9999, 4321]
        check_config(ctx, d_words, runs, n, s, ga.parse_percentage(95), lens_bp, spot)
    del d_words
    torch.cuda.empty_cache()


def test_sampled_histogram_missing_a_heavy_bin():
    """Past 2^26 entries the coarse histogram samples one 128-B line (16
    entries) in 8 of every row (row i: lines i % 8, i % 8 + 8, ...;
    pairs_index.hip bucket_hist_kernel).  Here 70,000 rows of 1,000 hashes
    (7.0e7 entries) put 96 hashes each into one coarse bin (top 12 bits
    0x800) at row positions the sample never reads -- 6.7M entries the
    histogram does not see, so that bin gets one bucket of millions of
    entries.  The build must notice (bucket over kBucketCap: the full-sort
    rebuild, counted in index_full_sort) and the result must be exact: rows
    2t and 2t + 1 share 990 hashes (every other pair shares none), so the
    passing pairs are exactly those 35,000, each with the oracle's (common,
    total).  Round 5's C5 failure (a missed bin's entries sent to bucket
    `nbuckets`) is this failure class; this pins it without relying on C5's
    natural hash distribution."""
    rng = np.random.default_rng(61)
    n, s, shared, heavy = 70000, 1000, 990, 96
    B = np.uint64(0x800 << 52)
    lo_span, hi_start = int(B), int(B) + (1 << 52)  # bin 0x800 is [B, B + 2^52)
    sk = np.empty((n, s), np.uint64)
    for t in range(n // 2):
        e = (2 * t) & 7
        c = 16 * (e + 2) + 256  # hashes below the bin: the bin's run starts in line e + 2 (mod 8) for rows 2t and 2t+1
        below = rng.integers(1, lo_span, c, dtype=np.uint64)
        binv = B + rng.integers(0, 1 << 52, heavy, dtype=np.uint64)
        above = rng.integers(hi_start, (1 << 64) - 1, s - c - heavy + 10, dtype=np.uint64)
        common = np.concatenate([below, binv, above[:s - c - heavy - 10]])
        for r, extra in ((2 * t, above[-20:-10]), (2 * t + 1, above[-10:])):
            sk[r] = np.sort(np.concatenate([common, extra]))
    assert all(len(np.unique(sk[i])) == s for i in (0, 1, 12345, n - 1))  # (distinct with near certainty; checked on a few)
    # the construction: no sampled line of any row holds a bin-0x800 hash
    bins = (sk >> np.uint64(52)).astype(np.uint32)
    line = np.arange(s) // 16
    rows = np.arange(n)
    sampled = (line[None, :] % 8) == (rows[:, None] % 8)
    assert not (sampled & (bins == 0x800)).any() and (bins == 0x800).sum() == heavy * n
    lens = np.full(n, s, np.uint32)
    thr = ga.parse_percentage(95)
    with ga.Context(k=21, sketch_size=s) as ctx:
        p = ctx.pairs(sk, lens, thr)
        paths = ctx.pair_paths()
    assert paths["index"] >= 1 and paths["index_full_sort"] >= 1 and paths["index_abandoned"] == 0, paths
    got = [(int(r["i"]), int(r["j"])) for r in p]
    assert got == [(2 * t, 2 * t + 1) for t in range(n // 2)]
    for r in p[::97]:  # (the oracle's merge on a spread of them)
        i, j = int(r["i"]), int(r["j"])
        assert (int(r["common"]), int(r["total"])) == oracle.raw_distance(sk[i], sk[j])


@pytest.mark.parametrize("cluster,s,max_sub,pct", [(1000, 1000, MAX_SUB, 95), (5000, 1000, MAX_SUB, 95),
                                                   (1000, 10000, MAX_SUB, 95), (10000, 1000, 0.01, 99.9)])
def test_large_clusters(cluster, s, max_sub, pct):
    """Dereplicating many strains of one species: 10k x 3 Mbp genomes in
    clusters of 1,000 and 5,000 (s = 1000), of 1,000 at s = 10000, and one
    cluster of 10,000 near-identical genomes (substitution rate <= 1%, so a
    hash is held by up to ~9,000 sketches: runs past a bucket and past the
    old 4,096 / 8,191 run limits, at 99.9% so that few pairs pass).  Runs of
    hundreds to thousands of members overflow the bucketed build's buckets:
    the full-sort build keeps each run in row order and each member reads
    only the members after it; rows with thousands of partners take the
    large partner map.  The index runs to completion (no
    abandon), its pairs equal the gate kernel's over every pair, and
    (common, total) and the pass decision equal the oracle's on 6,000
    sampled within-cluster pairs and 2,000 across clusters."""
    torch = torch_dev()
    n, glen = 10000, 3000000
    thr = ga.parse_percentage(pct)
    with ga.Context(k=21, sketch_size=s) as ctx:
        d_words = torch.empty(n * glen // 16, dtype=torch.int32, device="cuda")
        runs = ctx.synth_device(n, glen, cluster, max_sub, 11, d_words)
        d_sk = torch.zeros((n, s), dtype=torch.int64, device="cuda")
        d_len = torch.zeros(n, dtype=torch.int32, device="cuda")
        ctx.sketch_device(d_words, runs, n, d_sk, d_len)
        torch.cuda.synchronize()
        del d_words
        sk = d_sk.cpu().numpy().view(np.uint64)
        ln = d_len.cpu().numpy().view(np.uint32)
        assert (ln == s).all()

        def all_pairs(c):
            cap = 1 << 24
            d_out = torch.empty(cap * 4, dtype=torch.int32, device="cuda")
            d_cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
            c.pairs_device(d_sk, d_len, n, 0, ga.pair_tiles(n), thr, d_out, cap, d_cnt)
            torch.cuda.synchronize()
            k = int(d_cnt.item())
            assert k <= cap
            p = d_out[:k * 4].cpu().numpy().view(np.uint32).reshape(-1, 4)
            return p[np.lexsort((p[:, 1], p[:, 0]))]

        P = all_pairs(ctx)
        paths = ctx.pair_paths()
        assert paths["index"] == 1 and paths["index_abandoned"] == 0 and paths["gate"] == 0, paths
    old = os.environ.get("GALAHGPU_PAIRS_KERNEL")
    os.environ["GALAHGPU_PAIRS_KERNEL"] = "gate"
    try:
        with ga.Context(k=21, sketch_size=s) as gctx:
            PG = all_pairs(gctx)
            assert gctx.pair_paths()["gate"] == 1
    finally:
        if old is None:
            os.environ.pop("GALAHGPU_PAIRS_KERNEL")
        else:
            os.environ["GALAHGPU_PAIRS_KERNEL"] = old
    assert np.array_equal(P, PG)
    got = {(int(a), int(b)): (int(c), int(t)) for a, b, c, t in P}
    rng = np.random.default_rng(cluster + s)
    cl = rng.integers(0, n // cluster, 6000)
    a = rng.integers(0, cluster, 6000)
    b = rng.integers(0, cluster, 6000)
    keep = a != b
    ii = (cl * cluster + np.minimum(a, b))[keep].astype(np.uint32)
    jj = (cl * cluster + np.maximum(a, b))[keep].astype(np.uint32)
    if n // cluster > 1:
        ri = rng.integers(0, n, 4000).astype(np.uint32)
        rj = rng.integers(0, n, 4000).astype(np.uint32)
        x = (ri // cluster) != (rj // cluster)
        ii = np.concatenate([ii, np.minimum(ri, rj)[x][:2000]])
        jj = np.concatenate([jj, np.maximum(ri, rj)[x][:2000]])
    oc, ot = oracle.pair_list(sk, ln.astype(np.int32), ii, jj)
    opass = oracle.ani_array(oc, ot) >= np.float64(np.float32(thr))
    for q in range(len(ii)):
        key = (int(ii[q]), int(jj[q]))
        if opass[q]:
            assert got.get(key) == (int(oc[q]), int(ot[q])), key
        else:
            assert key not in got, key
    assert len(P) > 0 and not opass.all()
    print("\nclusters of %d, s=%d: %d passing pairs; index (full sort, row-ordered runs) == gate" % (cluster, s, len(P)))
    del d_sk, d_len
    torch.cuda.empty_cache()
