"""Parity of the HIP path (through the C ABI) with the CPU oracle and the
committed golden fixtures.  Needs an MI355X.

Bar: sketches and (common, total) bit-exact; ANI f32 identical (computed
from (common, total) by the same f64 expression); pair sets identical.
"""
import numpy as np
import pytest

import galah_amd as ga
import oracle
from conftest import xcheck_module
from test_host import EDGE_RECORDS, packed_records, unpack_run

pytestmark = pytest.mark.gpu


def torch_dev():
    import torch
    assert torch.cuda.is_available()
    return torch


def expected_pairs_from_table(golden, min_ani):
    thr = np.float64(np.float32(min_ani))
    return [(i, j, c, t) for (i, j, c, t, a) in golden["pairs"] if oracle.ani(c, t) >= thr]


def as_tuples(p):
    return [(int(r["i"]), int(r["j"]), int(r["common"]), int(r["total"])) for r in p]


def test_golden_sketches_bit_exact(gpu_ctx, golden):
    pk = ga.pack_files(golden["paths"])
    sk, lens = gpu_ctx.sketch(pk)
    assert (lens == golden["lens"]).all()
    for g in range(len(lens)):
        n = lens[g]
        assert (sk[g][:n] == golden["sketches"][g][:n]).all(), golden["names"][g]


@pytest.mark.parametrize("min_ani", [0.0, 0.5, 0.9, 0.95, 0.97, 0.98, 0.99, 1.0])
def test_golden_pairs_exact(gpu_ctx, golden, min_ani):
    p = gpu_ctx.pairs(golden["sketches"], golden["lens"], np.float32(min_ani))
    assert as_tuples(p) == expected_pairs_from_table(golden, min_ani)


def test_finch_rs_hello_world(golden, caplog):
    # src/finch.rs:85-107 through the reference-interface mirror
    paths = [golden["paths"][golden["names"].index(n)] for n in ("set1/1mbp.fna", "set1/500kb.fna")]
    with caplog.at_level("INFO", logger="galah"):
        d1 = ga.distances(paths, 0.9, 1000, 21)
    # src/finch.rs:46,48 and the library's one line (devices, phases, fallbacks)
    msgs = [r.getMessage() for r in caplog.records if r.name == "galah"]
    assert msgs[:2] == ["Sketching MinHash representations of each genome with finch ..",
                        "Finished sketching genomes"]
    assert msgs[2].startswith("galahgpu: ") and "index->gate 0, index full sort 0" in msgs[2]
    e1 = ga.SortedPairGenomeDistanceCache()
    e1.insert((0, 1), np.float32(0.9808188))
    assert d1 == e1
    assert repr(d1) == "SortedPairGenomeDistanceCache { internal: {(0, 1): Some(0.9808188)} }"
    d2 = ga.FinchPreclusterer(0.99, 1000, 21).distances(paths)
    assert d2 == ga.SortedPairGenomeDistanceCache()


def test_debug_logs_every_compared_pair(golden, caplog):
    """src/finch.rs:65-68: at debug level every pair i < j is logged with its
    f64 distance (Rust's `{}` formatting); the cache is the INFO-level one."""
    paths = golden["paths"]
    n = len(paths)
    with caplog.at_level("INFO", logger="galah"):
        d_info = ga.distances(paths, np.float32(0.9), 1000, 21)
    caplog.clear()
    with caplog.at_level("DEBUG", logger="galah"):
        d_dbg = ga.distances(paths, np.float32(0.9), 1000, 21)
    assert d_dbg == d_info and len(d_info.internal) == 161
    lines = [r.getMessage() for r in caplog.records if r.name == "galah" and r.levelname == "DEBUG"]
    assert len(lines) == n * (n - 1) // 2
    table = {(int(i), int(j)): (int(c), int(t)) for (i, j, c, t, _a) in golden["pairs"]}
    assert len(table) == len(lines)
    want = [(i, j) for i in range(n) for j in range(i + 1, n)]  # (the reference's loop order)
    for line, (i, j) in zip(lines, want):
        c, t = table[(i, j)]
        assert line == "Comparing %s and %s, distance %s" % (paths[i], paths[j], ga.rust_f64(oracle.ani(c, t))), line


@pytest.mark.parametrize("block_pairs", ["1", "10000"])
def test_each_streams_every_pair_in_blocks(gpu_ctx, golden, block_pairs, monkeypatch):
    """gg_precluster_files_each (the debug level's every-pair stream,
    src/finch.rs:53-68) over 162 genomes (the 27 golden files six times:
    three tile rows): every i < j exactly once, in (i, j) order across the
    blocks, each with the oracle's (common, total); the returned pairs are
    precluster_files' own.  GALAHGPU_EACH_PAIRS=1 makes every tile row a
    block of its own; 10000 puts two rows in the first block."""
    monkeypatch.setenv("GALAHGPU_EACH_PAIRS", block_pairs)
    n0 = len(golden["paths"])
    paths = golden["paths"] * 6
    n = len(paths)
    table = {(int(i), int(j)): (int(c), int(t)) for (i, j, c, t, _a) in golden["pairs"]}
    lens = golden["lens"]
    blocks = []
    min_ani = ga.parse_percentage(95)
    pairs, ani = gpu_ctx.precluster_files_each(paths, min_ani, lambda b: blocks.append(b.copy()))
    want_pairs, want_ani = gpu_ctx.precluster_files(paths, min_ani)
    assert as_tuples(pairs) == as_tuples(want_pairs) and (ani == want_ani).all()
    assert len(blocks) == (3 if block_pairs == "1" else 2)
    got = np.concatenate(blocks)
    assert len(got) == n * (n - 1) // 2
    ij = [(i, j) for i in range(n) for j in range(i + 1, n)]
    assert [(int(r["i"]), int(r["j"])) for r in got] == ij
    for r in got:
        a, b = int(r["i"]) % n0, int(r["j"]) % n0
        exp = (int(lens[a]), int(lens[a])) if a == b else table[(min(a, b), max(a, b))]
        assert (int(r["common"]), int(r["total"])) == exp


def test_each_sink_can_stop_the_call(gpu_ctx, golden):
    with pytest.raises(ga.GalahGpuError) as e:
        gpu_ctx.precluster_files_each(golden["paths"], np.float32(0.9), lambda b: True)
    assert e.value.status == 9


def test_precluster_files_matches_oracle(gpu_ctx, golden):
    min_ani = ga.parse_percentage(90)
    pairs, ani = gpu_ctx.precluster_files(golden["paths"], min_ani)
    exp = expected_pairs_from_table(golden, min_ani)
    assert as_tuples(pairs) == exp and len(exp) == 161
    for r, a in zip(pairs, ani):
        assert a == np.float32(oracle.ani(int(r["common"]), int(r["total"])))


def test_edge_records_and_retry_paths(gpu_ctx):
    rng = np.random.default_rng(11)
    rnd = lambda n: np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, n)].tobytes()
    half = rnd(40000)
    genomes = [[r] for r in EDGE_RECORDS]
    genomes += [
        [half, half],            # every k-mer twice: exercises tau retries
        [half + half],
        [b"A" * 300000],         # one distinct k-mer
        [rnd(900)],              # fewer k-mers than s
        [rnd(1100)],
        [rnd(30) for _ in range(50)],
        [],                      # genome without records
        [rnd(250000)],
        [(b"ACGTTGCAAT" * 2000)],  # low-complexity
    ]
    # part of a genome repeated (10-30% of its k-mers twice): the candidate
    # list repeats those values and still fits the finalize's sort, which
    # keeps the first copy of each (append mode, no set-mode retry)
    for frac in (0.1, 0.3):
        r = rnd(100000)
        genomes.append([r, r[:int(len(r) * frac)]])
        genomes.append([r + r[20000:20000 + int(len(r) * frac)]])
    pk = ga.pack_records(genomes)
    sk, lens = gpu_ctx.sketch(pk)
    for g, recs in enumerate(genomes):
        exp = oracle.sketch_records(recs) if recs else np.zeros(0, np.uint64)
        assert lens[g] == len(exp), g
        assert (sk[g][:lens[g]] == exp).all(), g


def test_repeated_kmers_dedup_in_candidate_list():
    """Genomes with 10-30% of their k-mers twice: each candidate list holds
    those values twice, fits the finalize's sort and keeps one copy (the
    first pass succeeds: no retry pass, no set mode), equal to the oracle."""
    rng = np.random.default_rng(12)
    rnd = lambda n: np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, n)].tobytes()
    genomes = []
    for frac in (0.1, 0.2, 0.3):
        r = rnd(100000)
        genomes += [[r, r[:int(len(r) * frac)]], [r + r[30000:30000 + int(len(r) * frac)]]]
    with ga.Context(k=21, sketch_size=1000) as ctx:
        sk, lens = ctx.sketch(ga.pack_records(genomes))
        assert ctx.fallbacks()["sketch_retry"] == 0
    for g, recs in enumerate(genomes):
        exp = oracle.sketch_records(recs)
        assert lens[g] == len(exp) == 1000 and (sk[g][:lens[g]] == exp).all(), g


@pytest.mark.parametrize("max_batch", ["0", "2"])
def test_tandem_repeats_switch_to_set_mode(monkeypatch, max_batch):
    """Tandem repeats (a 20-60 kb stretch 8-40 times over): every distinct
    candidate is appended once per copy, so once tau admits s distinct values
    the append-mode list outgrows its region and the finalize re-runs the
    genome at the same tau in set mode (kSketchRetrySet: one atomicCAS insert
    per distinct value, finch's insert-if-new).  The sketches equal the
    oracle's, through one batch and through batches of 2 genomes
    (GALAHGPU_K1_MAX_BATCH), next to genomes that need no retry."""
    rng = np.random.default_rng(13)
    rnd = lambda n: np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, n)].tobytes()
    genomes = [[rnd(20000) * 10], [rnd(120000)], [rnd(5000) * 40], [rnd(60000) * 8, rnd(3000)], [rnd(90000)]]
    monkeypatch.setenv("GALAHGPU_K1_MAX_BATCH", max_batch)
    with ga.Context(k=21, sketch_size=1000) as ctx:
        sk, lens = ctx.sketch(ga.pack_records(genomes))
        fb = ctx.fallbacks()
        assert fb["sketch_set"] >= 3 and fb["sketch_retry"] > 0, fb
        assert "set-mode genomes %d" % fb["sketch_set"] in ctx.info_line()
    for g, recs in enumerate(genomes):
        exp = oracle.sketch_records(recs)
        assert lens[g] == len(exp) == 1000 and (sk[g][:lens[g]] == exp).all(), g


def test_other_k_and_s():
    rng = np.random.default_rng(5)
    recs = [[np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, 20000)].tobytes()] for _ in range(3)]
    for k, s in [(21, 10), (16, 500), (31, 2000), (32, 64), (11, 100), (5, 50), (21, 10000)]:
        with ga.Context(k=k, sketch_size=s) as ctx:
            pk = ga.pack_records(recs, k=k)
            sk, lens = ctx.sketch(pk)
            for g in range(3):
                exp = oracle.sketch_records(recs[g], k=k, s=s)
                assert lens[g] == len(exp) and (sk[g][:lens[g]] == exp).all(), (k, s, g)


def random_sketch_set(rng, n, s, n_clusters):
    """Sketch-like rows: clustered shared hashes, some short and empty rows."""
    sk = np.zeros((n, s), np.uint64)
    lens = np.zeros(n, np.uint32)
    pools = [np.unique(rng.integers(0, 2**52, 3 * s, dtype=np.uint64)) for _ in range(n_clusters)]
    for i in range(n):
        pool = pools[i % n_clusters]
        m = s if i % 17 else int(rng.integers(0, s))
        if i % 29 == 0:
            m = 0
        share = rng.random()
        a = pool[rng.random(len(pool)) < share]
        b = rng.integers(0, 2**52, s, dtype=np.uint64)
        v = np.unique(np.concatenate([a, b]))[:m]
        sk[i, :len(v)] = v
        lens[i] = len(v)
    return sk, lens


@pytest.mark.parametrize("min_ani", [0.0, 0.9, 0.95, 0.99])
def test_random_pairs_vs_oracle(gpu_ctx, min_ani):
    rng = np.random.default_rng(3)
    sk, lens = random_sketch_set(rng, 300, 1000, 7)
    p = gpu_ctx.pairs(sk, lens, np.float32(min_ani))
    o = oracle.pairs(sk, lens.astype(np.int32), np.float32(min_ani))
    assert as_tuples(p) == [(int(r["i"]), int(r["j"]), int(r["common"]), int(r["total"])) for r in o]


def test_pairs_device_partition_union(gpu_ctx):
    torch = torch_dev()
    rng = np.random.default_rng(9)
    n = 333
    sk, lens = random_sketch_set(rng, n, 1000, 5)
    d_sk = torch.from_numpy(sk.view(np.int64)).cuda()
    d_lens = torch.from_numpy(lens.view(np.int32)).cuda()
    cap = n * n
    full = None
    for parts in (1, 2, 3, 5):
        got = []
        for part in range(parts):
            b, e = ga.pair_partition(n, parts, part)
            d_out = torch.zeros(cap * 4, dtype=torch.int32, device="cuda")
            d_cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
            gpu_ctx.pairs_device(d_sk, d_lens, n, b, e, np.float32(0.9), d_out, cap, d_cnt)
            torch.cuda.synchronize()
            c = int(d_cnt.item())
            assert c <= cap
            arr = d_out[:c * 4].cpu().numpy().view(np.uint32).reshape(-1, 4)
            got += [tuple(map(int, r)) for r in arr]
        got.sort()
        if full is None:
            full = got
            o = oracle.pairs(sk, lens.astype(np.int32), np.float32(0.9))
            assert full == [(int(r["i"]), int(r["j"]), int(r["common"]), int(r["total"])) for r in o]
        assert got == full


def synth_packed(ctx, n, glen, cl, rate, seed):
    torch = torch_dev()
    d_words = torch.empty(n * glen // 16, dtype=torch.int32, device="cuda")
    runs = ctx.synth_device(n, glen, cl, rate, seed, d_words)
    torch.cuda.synchronize()
    return d_words, runs


def test_synthetic_genomes_sketch_and_pairs_vs_oracle(gpu_ctx):
    torch = torch_dev()
    n, glen = 24, 200000
    d_words, runs = synth_packed(gpu_ctx, n, glen, 4, 0.07, 1234)
    d_out = torch.zeros((n, 1000), dtype=torch.int64, device="cuda")
    d_lens = torch.zeros(n, dtype=torch.int32, device="cuda")
    gpu_ctx.sketch_device(d_words, runs, n, d_out, d_lens)
    torch.cuda.synchronize()
    words = d_words.cpu().numpy().view(np.uint32)
    sk = d_out.cpu().numpy().view(np.uint64)
    lens = d_lens.cpu().numpy().view(np.uint32)
    osk = np.zeros((n, 1000), np.uint64)
    for g in range(n):
        seq = unpack_run(words, int(runs[g]["base"]), glen)
        exp = oracle.sketch_sequence(seq)
        assert lens[g] == len(exp) and (sk[g][:lens[g]] == exp).all(), g
        osk[g] = exp
    # clusters: members of a cluster are related, clusters are not
    o = oracle.pairs(osk, lens.astype(np.int32), np.float32(0.9))
    p = gpu_ctx.pairs(sk, lens, np.float32(0.9))
    assert as_tuples(p) == [(int(r["i"]), int(r["j"]), int(r["common"]), int(r["total"])) for r in o]
    assert all(r["i"] // 4 == r["j"] // 4 for r in p)
    assert len(p) > 0


def test_full_size_properties_c2(gpu_ctx):
    """C2 shape (1k x 3 Mbp): size-independent properties + oracle spot checks."""
    torch = torch_dev()
    n, glen, cl = 1000, 3000000, 10
    d_words, runs = synth_packed(gpu_ctx, n, glen, cl, 0.07, 2)
    d_out = torch.zeros((n, 1000), dtype=torch.int64, device="cuda")
    d_lens = torch.zeros(n, dtype=torch.int32, device="cuda")
    gpu_ctx.sketch_device(d_words, runs, n, d_out, d_lens)
    torch.cuda.synchronize()
    sk = d_out.cpu().numpy().view(np.uint64)
    lens = d_lens.cpu().numpy().view(np.uint32)
    assert (lens == 1000).all()
    assert (np.diff(sk, axis=1) > 0).all()  # ascending, distinct
    words = None
    for g in (0, 1, 517, 999):
        if words is None:
            words = d_words.cpu().numpy().view(np.uint32)
        exp = oracle.sketch_sequence(unpack_run(words, int(runs[g]["base"]), glen))
        assert (sk[g] == exp).all(), g
    p = gpu_ctx.pairs(sk, lens, np.float32(0.95))
    assert all(r["i"] // cl == r["j"] // cl for r in p)
    # spot-check (common, total) of 200 random pairs against the oracle merge
    rng = np.random.default_rng(0)
    passing = {(int(r["i"]), int(r["j"])): (int(r["common"]), int(r["total"])) for r in p}
    for _ in range(200):
        i, j = sorted(rng.choice(n, 2, replace=False))
        if rng.random() < 0.5:
            j = min(n - 1, (i // cl) * cl + int(rng.integers(0, cl)))
            if j == i:
                continue
            i, j = min(i, j), max(i, j)
        c, t = oracle.raw_distance(sk[i], sk[j])
        passes = oracle.ani(c, t) >= np.float64(np.float32(0.95))
        assert ((i, j) in passing) == passes
        if passes:
            assert passing[(i, j)] == (c, t)


def adversarial_sketches(rng, n, s):
    """Identical rows, prefix rows, extreme values (0 and 2^64-1), equal
    last elements, empty and singleton rows, a spread of genome-size-like
    value ranges."""
    rows = []
    base = np.unique(rng.integers(0, 2**63, 4 * s, dtype=np.uint64))
    for i in range(n):
        kind = i % 9
        if kind == 0:
            v = base[:s]
        elif kind == 1:
            v = base[: s // 2]                       # prefix of kind 0
        elif kind == 2:
            v = np.unique(np.concatenate([base[:s - 1], [np.uint64(2**64 - 1)]]))
        elif kind == 3:
            v = np.unique(np.concatenate([[np.uint64(0)], base[1:s]]))
        elif kind == 4:
            v = np.zeros(0, np.uint64)
        elif kind == 5:
            v = base[s // 3: s // 3 + 1]
        elif kind == 6:                              # small "genome": large hash range
            v = np.unique(rng.integers(0, 2**64 - 1, s, dtype=np.uint64))
        elif kind == 7:                              # shares the last element with kind 0
            mid = base[s // 2: s - 1]
            v = np.unique(np.concatenate([mid[rng.random(len(mid)) < 0.7], [base[s - 1]]]))
        else:
            scale = np.uint64(2 ** int(rng.integers(40, 63)))
            v = np.unique(np.concatenate([base[:s][rng.random(s) < 0.5],
                                          rng.integers(0, int(scale), s, dtype=np.uint64)]))[:s]
        rows.append(v[:s])
    sk = np.zeros((n, s), np.uint64)
    lens = np.zeros(n, np.uint32)
    for i, v in enumerate(rows):
        sk[i, :len(v)] = v
        lens[i] = len(v)
    return sk, lens


@pytest.mark.parametrize("s", [1000, 2000, 4000, 8000, 10000, 100, 37])
@pytest.mark.parametrize("min_ani", [0.0, 0.9])
def test_gate_table_and_merge_kernels_match_oracle(monkeypatch, s, min_ani):
    rng = np.random.default_rng(s)
    n = 150 if s >= 4000 else 260
    sk, lens = adversarial_sketches(rng, n, s)
    o = oracle.pairs(sk, lens.astype(np.int32), np.float32(min_ani))
    exp = [(int(r["i"]), int(r["j"]), int(r["common"]), int(r["total"])) for r in o]
    got = {}
    for kern in ("gate", "table", "merge", "index", "auto"):
        monkeypatch.setenv("GALAHGPU_PAIRS_KERNEL", kern)
        # (table, merge: the cross-check kernels of the test build)
        lib = xcheck_module() if kern in ("table", "merge") else ga
        with lib.Context(k=21, sketch_size=s) as ctx:
            got[kern] = as_tuples(ctx.pairs(sk, lens, np.float32(min_ani)))
    for kern in got:
        assert got[kern] == exp, kern


def test_product_refuses_cross_check_kernels(monkeypatch):
    """GALAHGPU_PAIRS_KERNEL=table|merge names kernels the product library
    does not carry: the call fails loudly instead of running another form."""
    sk, lens = random_sketch_set(np.random.default_rng(1), 40, 100, 3)
    for kern in ("table", "merge"):
        monkeypatch.setenv("GALAHGPU_PAIRS_KERNEL", kern)
        with ga.Context(k=21, sketch_size=100) as ctx:
            with pytest.raises(ga.GalahGpuError, match="libgalahgpu_xcheck.so"):
                ctx.pairs(sk, lens, np.float32(0.5))


def test_c5_mixed_sizes_s10000(gpu_ctx, monkeypatch):
    """Config C5 shape: s = 10000, genome lengths log-uniform in
    0.5-12 Mbp, N runs breaking k-mers.  Oracle spot checks on sketches (the
    smallest and largest genome and one more) and on 150 pairs; the gate,
    table-free merge and oracle agree on a 200-genome subset; pairs stay
    inside clusters."""
    torch = torch_dev()
    n, s, cl = 3000, 10000, 10
    lens_bp = ga.synth_mixed_lengths(n, 500000, 12000000, cl, 7)
    assert lens_bp.min() >= 500000 - 16 and lens_bp.max() <= 12000000
    d_words = torch.empty(int(lens_bp.sum()) // 16, dtype=torch.int32, device="cuda")
    with ga.Context(k=21, sketch_size=s) as ctx:
        runs = ctx.synth_mixed_device(lens_bp, cl, 0.07, 1e-4, 8, d_words)
        torch.cuda.synchronize()
        assert len(runs) > n  # N runs split the genomes
        d_sk = torch.zeros((n, s), dtype=torch.int64, device="cuda")
        d_len = torch.zeros(n, dtype=torch.int32, device="cuda")
        ctx.sketch_device(d_words, runs, n, d_sk, d_len)
        torch.cuda.synchronize()
        sk = d_sk.cpu().numpy().view(np.uint64)
        ln = d_len.cpu().numpy().view(np.uint32)
        assert (ln == s).all()
        assert (np.diff(sk, axis=1) > 0).all()
        words = d_words.cpu().numpy().view(np.uint32)
        for g in (int(np.argmin(lens_bp)), int(np.argmax(lens_bp)), 1234):
            recs = [unpack_run(words, int(r["base"]), int(r["len"])) for r in runs[runs["genome"] == g]]
            exp = oracle.sketch_records(recs, s=s)
            assert (sk[g] == exp).all(), g
        thr = np.float32(0.95)
        p = ctx.pairs(sk, ln, thr)
        assert len(p) > 0 and all(r["i"] // cl == r["j"] // cl for r in p)
        passing = {(int(r["i"]), int(r["j"])): (int(r["common"]), int(r["total"])) for r in p}
        rng = np.random.default_rng(1)
        for _ in range(150):
            i = int(rng.integers(0, n - 1))
            j = min(n - 1, (i // cl) * cl + int(rng.integers(0, cl))) if rng.random() < 0.7 else int(rng.integers(0, n))
            if i == j:
                continue
            i, j = min(i, j), max(i, j)
            c, t = oracle.raw_distance(sk[i], sk[j])
            assert ((i, j) in passing) == (oracle.ani(c, t) >= np.float64(thr))
            if (i, j) in passing:
                assert passing[(i, j)] == (c, t)
    sub = 200
    o = oracle.pairs(sk[:sub], ln[:sub].astype(np.int32), thr)
    exp = [(int(r["i"]), int(r["j"]), int(r["common"]), int(r["total"])) for r in o]
    assert [x for x in as_tuples(p) if x[1] < sub] == exp
    monkeypatch.setenv("GALAHGPU_PAIRS_KERNEL", "merge")
    with xcheck_module().Context(k=21, sketch_size=s) as ctx:
        assert as_tuples(ctx.pairs(sk[:sub], ln[:sub], thr)) == exp


@pytest.mark.parametrize("s", [200, 3000])
def test_gate_kernel_low_word_collisions(monkeypatch, s):
    """Keys that share their low 32 bits all land in one bucket of the gate
    kernel's table and set a single gate bit: the walks degenerate into
    full-bucket scans but must still count exactly (narrow and wide)."""
    rng = np.random.default_rng(s)
    n = 70
    lo = np.uint64(0x9E3779B9)
    his = np.unique(rng.integers(1, 2**31, 3 * s, dtype=np.uint64))
    sk = np.zeros((n, s), np.uint64)
    lens = np.zeros(n, np.uint32)
    for i in range(n):
        m = s if i % 5 else s // 3
        pick = np.sort(rng.choice(len(his) // (1 + i % 3), m, replace=False))
        v = (his[pick] << np.uint64(32)) | lo
        if i % 7 == 0:  # a few keys with their own low words
            v = np.unique(np.concatenate([v[: m - 5], rng.integers(0, 2**63, 5, dtype=np.uint64)]))[:m]
        sk[i, :len(v)] = v
        lens[i] = len(v)
    for thr in (0.0, 0.5, 0.9):
        o = oracle.pairs(sk, lens.astype(np.int32), np.float32(thr))
        exp = [(int(r["i"]), int(r["j"]), int(r["common"]), int(r["total"])) for r in o]
        for kern in ("gate", "index"):
            monkeypatch.setenv("GALAHGPU_PAIRS_KERNEL", kern)
            with ga.Context(k=21, sketch_size=s) as ctx:
                assert as_tuples(ctx.pairs(sk, lens, np.float32(thr))) == exp, (thr, kern)


@pytest.mark.parametrize("n", [1, 2, 3, 31, 33, 65, 129])
def test_gate_kernel_small_and_ragged_n(gpu_ctx, n):
    rng = np.random.default_rng(n)
    sk, lens = random_sketch_set(rng, n, 1000, 3)
    for thr in (0.0, 0.9):
        p = gpu_ctx.pairs(sk, lens, np.float32(thr))
        o = oracle.pairs(sk, lens.astype(np.int32), np.float32(thr))
        assert as_tuples(p) == [(int(r["i"]), int(r["j"]), int(r["common"]), int(r["total"])) for r in o]


def test_index_kernel_tile_ranges_and_partition(monkeypatch):
    """The inverted-index kernel over explicit tile ranges (multi-GPU parts):
    the union over 1, 2, 3 and 7 parts equals the oracle."""
    torch = torch_dev()
    monkeypatch.setenv("GALAHGPU_PAIRS_KERNEL", "index")
    rng = np.random.default_rng(23)
    n = 701
    sk, lens = random_sketch_set(rng, n, 1000, 9)
    o = oracle.pairs(sk, lens.astype(np.int32), np.float32(0.9))
    exp = [(int(r["i"]), int(r["j"]), int(r["common"]), int(r["total"])) for r in o]
    d_sk = torch.from_numpy(sk.view(np.int64)).cuda()
    d_lens = torch.from_numpy(lens.view(np.int32)).cuda()
    cap = n * n
    with ga.Context(k=21, sketch_size=1000) as ctx:
        for parts in (1, 2, 3, 7):
            got = []
            for part in range(parts):
                b, e = ga.pair_partition(n, parts, part)
                d_out = torch.zeros(cap * 4, dtype=torch.int32, device="cuda")
                d_cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
                ctx.pairs_device(d_sk, d_lens, n, b, e, np.float32(0.9), d_out, cap, d_cnt)
                torch.cuda.synchronize()
                c = int(d_cnt.item())
                arr = d_out[:c * 4].cpu().numpy().view(np.uint32).reshape(-1, 4)
                got += [tuple(map(int, r)) for r in arr]
            assert sorted(got) == exp, parts


def test_index_kernel_many_partners_and_long_runs(monkeypatch):
    """Row 0 shares one hash with each of 2,999 other rows (more partners
    than one LDS map holds: the row is counted in several passes), and a hash
    shared by more sketches than the index kernel's run limit (the call falls
    back to the gate kernel before emitting anything): both equal the oracle."""
    rng = np.random.default_rng(29)
    s = 1000
    n = 3000
    base = np.unique(rng.integers(1, 2**62, 4 * s, dtype=np.uint64))[:s]
    sk = np.zeros((n, s), np.uint64)
    lens = np.zeros(n, np.uint32)
    sk[0] = base
    lens[0] = s
    for i in range(1, n):
        v = np.unique(np.concatenate([[base[i % s]], rng.integers(2**62, 2**63, 40, dtype=np.uint64)]))
        sk[i, :len(v)] = v
        lens[i] = len(v)
    for thr in (0.001, 0.5):
        o = oracle.pairs(sk, lens.astype(np.int32), np.float32(thr))
        exp = [(int(r["i"]), int(r["j"]), int(r["common"]), int(r["total"])) for r in o]
        for kern in ("index", "gate"):
            monkeypatch.setenv("GALAHGPU_PAIRS_KERNEL", kern)
            with ga.Context(k=21, sketch_size=s) as ctx:
                assert as_tuples(ctx.pairs(sk, lens, np.float32(thr))) == exp, (thr, kern)
        # row 0's partners still overflowing the map at the last split: the
        # index launch's output is dropped and the gate kernel runs instead
        monkeypatch.setenv("GALAHGPU_PAIRS_KERNEL", "index")
        for split in ("0", "1"):
            monkeypatch.setenv("GALAHGPU_INDEX_MAX_SPLIT", split)
            with ga.Context(k=21, sketch_size=s) as ctx:
                assert as_tuples(ctx.pairs(sk, lens, np.float32(thr))) == exp, (thr, split)
                if split == "0":  # 2,999 partners never fit one map: abandoned for the gate kernel
                    assert ctx.pair_paths() == {"index": 0, "index_abandoned": 1, "gate": 1, "other": 0,
                                                "index_full_sort": 0}
                    assert ctx.fallbacks()["index_to_gate"] == 1
                    assert "index->gate 1," in ctx.info_line()
        monkeypatch.delenv("GALAHGPU_INDEX_MAX_SPLIT")
    # 5,000 sketches that all hold one hash: a run of 5,000 (over one bucket
    # of the bucketed build and over the old 4,096 run limit): the full-sort
    # build keeps the run in row order, each member reads the members after
    # it, and rows with thousands of partners take the large partner map
    n = 5000
    s = 40
    shared = np.uint64(12345)
    sk = np.zeros((n, s), np.uint64)
    lens = np.zeros(n, np.uint32)
    for i in range(n):
        v = np.unique(np.concatenate([[shared], rng.integers(2**40, 2**63, s - 1, dtype=np.uint64)]))[:s]
        sk[i, :len(v)] = v
        lens[i] = len(v)
    o = oracle.pairs(sk, lens.astype(np.int32), np.float32(0.01))
    exp = [(int(r["i"]), int(r["j"]), int(r["common"]), int(r["total"])) for r in o]
    assert len(exp) > 0
    monkeypatch.setenv("GALAHGPU_PAIRS_KERNEL", "index")
    with ga.Context(k=21, sketch_size=s) as ctx:
        assert as_tuples(ctx.pairs(sk, lens, np.float32(0.01))) == exp
        # (one index call per output-buffer pass, none abandoned)
        paths = ctx.pair_paths()
        assert paths["index"] >= 1 and paths["index_abandoned"] == 0 and paths["gate"] == 0, paths
        assert paths["index_full_sort"] == paths["index"]


def _part_of(j, plog2):
    # pairs_index.hip part_of: the top plog2 bits of j * 0x9E3779B1 (mod 2^32)
    return ((j * 0x9E3779B1) & 0xFFFFFFFF) >> (32 - plog2) if plog2 else 0


def test_index_kernel_later_partner_class_overflows(monkeypatch):
    """Row 0's partners split into 2 classes where class 0 fits the LDS map
    and class 1 (2,000 partners > the map's 1,536) does not: the row goes on
    at classes 2 and 3 of 4 without counting class 0 again (it
    restarted at class 0 and emitted those pairs twice)."""
    rng = np.random.default_rng(41)
    s = 1000
    n = 4400
    c1 = [j for j in range(1, n) if _part_of(j, 1) == 1][:2000]
    c0 = [j for j in range(1, n) if _part_of(j, 1) == 0][:200]
    assert len(c1) == 2000 and len(c0) == 200
    partners = set(c0) | set(c1)
    base = np.unique(rng.integers(1, 2**62, 4 * s, dtype=np.uint64))[:s]
    sk = np.zeros((n, s), np.uint64)
    lens = np.zeros(n, np.uint32)
    sk[0] = base
    lens[0] = s
    for i in range(1, n):
        own = rng.integers(2**62, 2**63, 40, dtype=np.uint64)
        v = np.unique(np.concatenate([[base[i % s]], own]) if i in partners else own)
        sk[i, :len(v)] = v
        lens[i] = len(v)
    monkeypatch.setenv("GALAHGPU_PAIRS_KERNEL", "index")
    for thr in (0.001, 0.5):
        o = oracle.pairs(sk, lens.astype(np.int32), np.float32(thr))
        exp = [(int(r["i"]), int(r["j"]), int(r["common"]), int(r["total"])) for r in o]
        assert sum(1 for p in exp if p[0] == 0) == len(partners)
        with ga.Context(k=21, sketch_size=s) as ctx:
            got = as_tuples(ctx.pairs(sk, lens, np.float32(thr)))
            assert len({(p[0], p[1]) for p in got}) == len(got), "duplicate (i, j)"
            assert got == exp, thr
            assert ctx.pair_paths()["index"] == 1 and ctx.pair_paths()["index_abandoned"] == 0


def test_many_runs_index_and_run_table_errors(gpu_ctx):
    """> 2^18 runs (the host run index runs in parallel chunks), ragged run
    lengths around one K1 segment (44 k-mers), genomes without runs between
    others, and every run-table error, through gg_sketch_device."""
    torch = torch_dev()
    rng = np.random.default_rng(77)
    n_words = 1 << 21
    words = rng.integers(0, 2**32, n_words, dtype=np.uint64).astype(np.uint32)
    d_words = torch.from_numpy(words.view(np.int32)).cuda()
    n_runs, n_genomes = 300000, 64
    lens = rng.integers(21, 160, n_runs).astype(np.uint32)
    lens[::7] = rng.integers(21, 66, len(lens[::7]))   # around one segment (k-mers 1..45)
    gaps = rng.integers(1, 40, n_runs).astype(np.uint64)
    base = np.cumsum(lens.astype(np.uint64) + gaps) - lens.astype(np.uint64)
    assert base[-1] + lens[-1] <= n_words * 16
    # genomes 5, 6 and 40 get no runs
    owners = np.array([g for g in range(n_genomes) if g not in (5, 6, 40)], np.uint32)
    genome = owners[np.sort(rng.integers(0, len(owners), n_runs))]
    runs = np.zeros(n_runs, ga.RUN_DTYPE)
    runs["genome"], runs["len"], runs["base"] = genome, lens, base
    d_out = torch.zeros((n_genomes, 1000), dtype=torch.int64, device="cuda")
    d_lens = torch.zeros(n_genomes, dtype=torch.int32, device="cuda")
    gpu_ctx.sketch_device(d_words, runs, n_genomes, d_out, d_lens)
    torch.cuda.synchronize()
    sk = d_out.cpu().numpy().view(np.uint64)
    gl = d_lens.cpu().numpy().view(np.uint32)
    for g in list(range(0, n_genomes, 9)) + [5, 6, 40, n_genomes - 1]:
        sel = runs[runs["genome"] == g]
        recs = [unpack_run(words, int(r["base"]), int(r["len"])) for r in sel]
        exp = oracle.sketch_records(recs) if recs else np.zeros(0, np.uint64)
        assert gl[g] == len(exp) and (sk[g][:gl[g]] == exp).all(), g
    bad = []
    r1 = runs.copy()
    r1["genome"][1000], r1["genome"][1001] = r1["genome"][1001] + 1, r1["genome"][1000]
    bad.append((r1, "non-decreasing genome"))
    r2 = runs.copy()
    r2["len"][250000] = 20
    bad.append((r2, "shorter than k"))
    r3 = runs.copy()
    r3["base"][-1] = n_words * 16 - 10
    bad.append((r3, "past the packed words"))
    r4 = runs.copy()
    r4["genome"][-1] = n_genomes
    bad.append((r4, "non-decreasing genome"))
    # a rejected table leaves the caller's rows and lengths as they were
    # (the one-batch path's finalize used to write them first)
    d_out.fill_(7)
    d_lens.fill_(9)
    for r, msg in bad:
        with pytest.raises(ga.GalahGpuError, match=msg):
            gpu_ctx.sketch_device(d_words, r, n_genomes, d_out, d_lens)
        torch.cuda.synchronize()
        assert bool((d_out == 7).all()) and bool((d_lens == 9).all()), msg
    # and the context still sketches correctly afterwards
    gpu_ctx.sketch_device(d_words, runs, n_genomes, d_out, d_lens)
    torch.cuda.synchronize()
    sk2 = d_out.cpu().numpy().view(np.uint64)
    assert (d_lens.cpu().numpy().view(np.uint32) == gl).all()
    assert all((sk2[g][:gl[g]] == sk[g][:gl[g]]).all() for g in range(n_genomes))


class HostPacked:
    """A caller-built gg_packed (host words + run table) for Context.sketch."""

    def __init__(self, words, runs, n_genomes):
        self.words = np.ascontiguousarray(words, dtype=np.uint32)
        self.runs = np.ascontiguousarray(runs, dtype=ga.RUN_DTYPE)
        self.kmers = np.zeros(max(n_genomes, 1), np.uint64)
        p = ga._Packed()
        p.words = self.words.ctypes.data_as(ga.ctypes.POINTER(ga.ctypes.c_uint32))
        p.n_words = len(self.words)
        p.n_bases = len(self.words) * 16
        p.runs = self.runs.ctypes.data_as(ga.ctypes.POINTER(ga._Run))
        p.n_runs = len(self.runs)
        p.n_genomes = n_genomes
        p.genome_kmers = self.kmers.ctypes.data_as(ga.ctypes.POINTER(ga.ctypes.c_uint64))
        self._struct = p
        self._p = ga.ctypes.pointer(p)
        self.n_genomes = n_genomes


def test_host_sketch_run_table_checked_before_split():
    """gg_sketch (host buffers) splits the run table by genome among the
    members before K1 sees it: every bad table fails with the run-table error
    on 1 and 2 members, and a valid table whose bases do not rise with the
    genome (genome 0 packed after genome 1) gives the oracle's sketches."""
    rng = np.random.default_rng(78)
    n_words = 1 << 14
    words = rng.integers(0, 2**32, n_words, dtype=np.uint64).astype(np.uint32)
    n_genomes = 6
    runs = np.zeros(12, ga.RUN_DTYPE)
    runs["genome"] = np.repeat(np.arange(n_genomes), 2)
    runs["len"] = rng.integers(21, 5000, 12)
    # genome g's two runs inside block (n_genomes - 1 - g): bases fall as g rises
    blk = n_words * 16 // n_genomes
    for r in range(12):
        g = r // 2
        runs["base"][r] = (n_genomes - 1 - g) * blk + (r % 2) * 6000
    bad = []
    r1 = runs.copy()
    r1["genome"][3] = n_genomes + 5
    bad.append((r1, "non-decreasing genome"))
    r2 = runs.copy()
    r2["genome"][4], r2["genome"][5] = 3, 1
    bad.append((r2, "non-decreasing genome"))
    r3 = runs.copy()
    r3["len"][7] = 20
    bad.append((r3, "shorter than k"))
    r4 = runs.copy()
    r4["base"][11] = n_words * 16 - 10
    bad.append((r4, "past the packed words"))
    for devs in ([0], [0, 0]):
        with ga.Context(k=21, sketch_size=1000, devices=devs) as ctx:
            for r, msg in bad:
                with pytest.raises(ga.GalahGpuError, match=msg):
                    ctx.sketch(HostPacked(words, r, n_genomes))
            sk, lens = ctx.sketch(HostPacked(words, runs, n_genomes))
            for g in range(n_genomes):
                sel = runs[runs["genome"] == g]
                recs = [unpack_run(words, int(x["base"]), int(x["len"])) for x in sel]
                exp = oracle.sketch_records(recs)
                assert lens[g] == len(exp) and (sk[g][:lens[g]] == exp).all(), (devs, g)


@pytest.mark.parametrize("buckets", ["1", "0"])
@pytest.mark.parametrize("top", [2**50, 2**64 - 1, 2**31])
def test_index_kernel_shared_top_bits(monkeypatch, top, buckets):
    """The index sorts by the top 32 significant bits of each hash and carries
    the low word: hashes that differ only below those bits share a key and
    must be split into their own runs (clusters of values within 2^12 of
    each other, rows mixing them, the largest hash setting the key shift;
    top = 2^31 leaves whole hashes as keys).  Equal to the oracle, with the
    bucketed build (default: ~2,000 entries of one cluster in one bucket)
    and with the full sort and run pass (GALAHGPU_INDEX_BUCKETS=0)."""
    rng = np.random.default_rng(31)
    n, s = 400, 300
    anchors = rng.integers(0, top // 2, 60, dtype=np.uint64)
    pool = np.unique((anchors[:, None] + rng.integers(0, 4096, (60, 40)).astype(np.uint64)).reshape(-1))
    sk = np.zeros((n, s), np.uint64)
    lens = np.zeros(n, np.uint32)
    for i in range(n):
        take = pool[rng.random(len(pool)) < 0.12]
        extra = rng.integers(0, top // 2, 30, dtype=np.uint64)
        v = np.unique(np.concatenate([take, extra, [np.uint64(top)]] if i == 7 else [take, extra]))[:s]
        sk[i, :len(v)] = v
        lens[i] = len(v)
    monkeypatch.setenv("GALAHGPU_PAIRS_KERNEL", "index")
    monkeypatch.setenv("GALAHGPU_INDEX_BUCKETS", buckets)
    for thr in (0.5, 0.9):
        o = oracle.pairs(sk, lens.astype(np.int32), np.float32(thr))
        exp = [(int(r["i"]), int(r["j"]), int(r["common"]), int(r["total"])) for r in o]
        with ga.Context(k=21, sketch_size=s) as ctx:
            assert as_tuples(ctx.pairs(sk, lens, np.float32(thr))) == exp, thr
            # the mixed runs are split by the index itself (no gate fallback)
            assert ctx.pair_paths() == {"index": 1, "index_abandoned": 0, "gate": 0, "other": 0,
                                        "index_full_sort": int(buckets == "0")}
        assert thr > 0.5 or len(exp) > 0


def test_index_bucket_overflow_falls_back_to_full_sort(monkeypatch):
    """One hash held by 3,500 sketches: its bucket of the bucketed build holds
    more entries than one workgroup groups in LDS (3,072), while the run
    (3,500) is within the run limit (4,096).  The host rebuilds the index
    with the full sort and the run pass: same pairs as the oracle (every pair
    of the 300 sketches that also share a second hash passes at 0.87, not
    every pair of the others), the index still used (not the gate kernel)."""
    rng = np.random.default_rng(44)
    n, s = 3500, 20
    sk = np.zeros((n, s), np.uint64)
    lens = np.zeros(n, np.uint32)
    a, b = np.uint64(2**40 + 5), np.uint64(2**50 + 11)
    for i in range(n):
        shared = [a, b] if i < 300 else [a]
        v = np.unique(np.concatenate([shared, rng.integers(2**52, 2**63, s, dtype=np.uint64)]))[:s]
        sk[i, :len(v)] = v
        lens[i] = len(v)
    monkeypatch.setenv("GALAHGPU_PAIRS_KERNEL", "index")
    o = oracle.pairs(sk, lens.astype(np.int32), np.float32(0.87))
    exp = [(int(r["i"]), int(r["j"]), int(r["common"]), int(r["total"])) for r in o]
    assert 300 * 299 // 2 <= len(exp) < n * (n - 1) // 2
    with ga.Context(k=21, sketch_size=s) as ctx:
        assert as_tuples(ctx.pairs(sk, lens, np.float32(0.87))) == exp
        assert ctx.pair_paths() == {"index": 1, "index_abandoned": 0, "gate": 0, "other": 0, "index_full_sort": 1}
        # the slow path is reported at galah's log level (gg_fallbacks, gg_info_line)
        assert ctx.fallbacks()["index_full_sort"] == 1 and ctx.fallbacks()["index_to_gate"] == 0
        assert "index full sort 1" in ctx.info_line()


def test_device_run_table_same_as_host(gpu_ctx):
    """A run table in device memory (gg_sketch_device / gg_precluster_shards
    read it in place) gives the host table's sketches, through the retry
    pass (genome 3's 300 runs repeat one stretch: its k-mer count
    overestimates its distinct k-mers 300 times, so the first threshold is
    too small and the genome is sketched again from the host mirror of the
    table) and the run-table errors (the message names the same fault)."""
    torch = torch_dev()
    rng = np.random.default_rng(91)
    n_words = 1 << 16
    words = rng.integers(0, 2**32, n_words, dtype=np.uint64).astype(np.uint32)
    d_words = torch.from_numpy(words.view(np.int32)).cuda()
    n_genomes = 8
    rows = []
    base = 0
    for g in range(n_genomes):
        if g == 3:
            rows += [(g, 400, 5000)] * 300
            continue
        for _ in range(20):
            ln = int(rng.integers(30, 3000))
            rows.append((g, ln, base))
            base += ln + 7
    assert base < n_words * 16
    runs = np.array(rows, dtype=ga.RUN_DTYPE)
    outs = []
    for table in (runs, ga.device_runs(runs, "cuda")):
        d_out = torch.zeros((n_genomes, 1000), dtype=torch.int64, device="cuda")
        d_lens = torch.zeros(n_genomes, dtype=torch.int32, device="cuda")
        gpu_ctx.sketch_device(d_words, table, n_genomes, d_out, d_lens)
        torch.cuda.synchronize()
        outs.append((d_out.cpu().numpy().view(np.uint64).copy(), d_lens.cpu().numpy().view(np.uint32).copy()))
    (sk_h, ln_h), (sk_d, ln_d) = outs
    assert (ln_h == ln_d).all() and (sk_h == sk_d).all()
    for g in (0, 3, n_genomes - 1):
        sel = runs[runs["genome"] == g]
        exp = oracle.sketch_records([unpack_run(words, int(r["base"]), int(r["len"])) for r in sel])
        assert ln_d[g] == len(exp) and (sk_d[g][:ln_d[g]] == exp).all(), g
    assert ln_d[3] < 1000  # (one 400-base stretch: fewer distinct k-mers than s)
    r = runs.copy()
    r["len"][5] = 20
    with pytest.raises(ga.GalahGpuError, match="shorter than k"):
        gpu_ctx.sketch_device(d_words, ga.device_runs(r, "cuda"), n_genomes, d_out, d_lens)


@pytest.mark.parametrize("max_batch", ["7", "1"])
def test_sketch_in_several_batches(monkeypatch, max_batch):
    """More genomes than one K1 batch (GALAHGPU_K1_MAX_BATCH forces batches
    of 7 or 1 genome: the host-planned passes, candidate sets reused from
    batch to batch): the same sketches as one batch, through the retry
    passes (genome 3 repeats one stretch) and on the device run table."""
    torch = torch_dev()
    rng = np.random.default_rng(92)
    n_words = 1 << 16
    words = rng.integers(0, 2**32, n_words, dtype=np.uint64).astype(np.uint32)
    d_words = torch.from_numpy(words.view(np.int32)).cuda()
    n_genomes = 23
    rows, base = [], 0
    for g in range(n_genomes):
        if g == 3:
            rows += [(g, 400, 5000)] * 300
            continue
        for _ in range(8):
            ln = int(rng.integers(30, 4000))
            rows.append((g, ln, base))
            base += ln + 5
    assert base < n_words * 16
    runs = np.array(rows, dtype=ga.RUN_DTYPE)
    outs = []
    for mb in ("0", max_batch):
        monkeypatch.setenv("GALAHGPU_K1_MAX_BATCH", mb)
        for table in (runs, ga.device_runs(runs, "cuda")):
            with ga.Context(k=21, sketch_size=1000) as ctx:
                d_out = torch.zeros((n_genomes, 1000), dtype=torch.int64, device="cuda")
                d_lens = torch.zeros(n_genomes, dtype=torch.int32, device="cuda")
                for _ in range(2):  # (the second call reuses the emptied candidate sets)
                    ctx.sketch_device(d_words, table, n_genomes, d_out, d_lens)
                torch.cuda.synchronize()
                outs.append((d_out.cpu().numpy().view(np.uint64).copy(), d_lens.cpu().numpy().view(np.uint32).copy()))
    sk0, ln0 = outs[0]
    for sk, ln in outs[1:]:
        assert (ln == ln0).all() and (sk == sk0).all()
    for g in (0, 3, 7, n_genomes - 1):
        sel = runs[runs["genome"] == g]
        exp = oracle.sketch_records([unpack_run(words, int(r["base"]), int(r["len"])) for r in sel])
        assert ln0[g] == len(exp) and (sk0[g][:ln0[g]] == exp).all(), g
