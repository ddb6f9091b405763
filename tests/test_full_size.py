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
