"""Host-side logic of libgalahgpu.so, CPU only: the C ABI loads and exports
every declared symbol, the FASTA -> 2-bit packer is checked against the
oracle, and the host arithmetic (ANI, parse_percentage, tile partition) and
the SortedPairGenomeDistanceCache mirror behave as the reference's."""
import gzip
import os
import re

import numpy as np
import pytest

import galah_amd as ga
import oracle
from conftest import ROOT, golden_path

ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)


def unpack_run(words, base, length):
    """2-bit words (first base in bits 31..30) -> ASCII bytes of one run."""
    idx = np.arange(base, base + length, dtype=np.uint64)
    w = words[(idx >> np.uint64(4)).astype(np.int64)]
    sh = (np.uint32(30) - np.uint32(2) * (idx & np.uint64(15)).astype(np.uint32))
    codes = (w >> sh) & np.uint32(3)
    return ACGT[codes].tobytes()


def packed_records(pk):
    """Per genome, the list of ASCII runs."""
    out = [[] for _ in range(pk.n_genomes)]
    for r in pk.runs:
        out[int(r["genome"])].append(unpack_run(pk.words, int(r["base"]), int(r["len"])))
    return out


# ---------------------------------------------------------------- ABI ----
def header_functions():
    with open(os.path.join(ROOT, "include", "galahgpu.h")) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = set(re.findall(r"\b(gg_[a-z0-9_]+)\s*\(", text))
    return names


def test_abi_exports_every_declared_symbol():
    declared = header_functions()
    assert declared == set(ga.EXPORTED_SYMBOLS)
    L = ga.lib()
    for name in declared:
        assert hasattr(L, name), name
    assert ga.abi_version() == 7


def test_no_oracle_in_product_library():
    # the product must not link or embed the CPU oracle
    import subprocess
    syms = subprocess.run(["nm", "-D", ga.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle_" not in syms
    with open(ga.LIB_PATH, "rb") as f:
        assert b"oracle_sketch" not in f.read()


def test_cross_check_kernels_only_in_test_library():
    """pairs.hip's table / merge kernels (independent K2 forms the parity
    tests compare against) are built into libgalahgpu_xcheck.so only: the
    product carries the default index and gate kernels, and the test library
    exports the same C ABI."""
    import subprocess
    from conftest import xcheck_module
    with open(ga.LIB_PATH, "rb") as f:
        prod = f.read()
    assert b"pairs_merge_kernel" not in prod and b"pairs_table_kernel" not in prod
    assert b"index_pairs_kernel" in prod and b"pairs_gate_kernel" in prod
    gx = xcheck_module()
    with open(gx.LIB_PATH, "rb") as f:
        assert b"pairs_merge_kernel" in f.read()
    a = subprocess.run(["nm", "-D", "--defined-only", ga.LIB_PATH], capture_output=True, text=True).stdout
    b = subprocess.run(["nm", "-D", "--defined-only", gx.LIB_PATH], capture_output=True, text=True).stdout
    exported = lambda t: sorted(x.split()[-1] for x in t.splitlines() if " T gg_" in x)
    assert exported(a) == exported(b) and len(exported(a)) >= len(ga.EXPORTED_SYMBOLS)


def test_create_without_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(ga.GalahGpuError) as e:
        ga.Context()
    assert e.value.status == ga.GG_ERR_NO_DEVICE


def test_create_multi_without_device_fails_loudly(monkeypatch):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    for devs in ("all", [0, 0], [0]):
        with pytest.raises(ga.GalahGpuError) as e:
            ga.Context(devices=devs)
        assert e.value.status == ga.GG_ERR_NO_DEVICE
    monkeypatch.setenv("GALAHGPU_DEVICES", "0,0")
    with pytest.raises(ga.GalahGpuError):
        ga.Context(devices="all")


# ------------------------------------------------------------- packer ----
def test_pack_files_thread_count_does_not_change_packing(golden):
    """galah --threads (CAP:1327-1332) bounds ingest; the packed bases and
    runs are the same for 1 thread and for many."""
    one = ga.pack_files(golden["paths"], threads=1)
    many = ga.pack_files(golden["paths"], threads=7)
    assert (one.words == many.words).all()
    assert (one.runs == many.runs).all()
    assert (one.genome_kmers == many.genome_kmers).all()


def test_packer_matches_oracle_on_golden_genomes(golden):
    pk = ga.pack_files(golden["paths"], k=21)
    assert pk.n_genomes == len(golden["paths"])
    recs = packed_records(pk)
    for g, path in enumerate(golden["paths"]):
        assert (pk.runs["genome"] == g).sum() == len(recs[g])
        nk = sum(len(r) - 20 for r in recs[g])
        assert pk.genome_kmers[g] == nk
        sk = oracle.sketch_records(recs[g])
        n = golden["lens"][g]
        assert len(sk) == n and (sk == golden["sketches"][g][:n]).all(), path
    pk.free()


def test_packer_plain_equals_gzip(tmp_path):
    src = golden_path("abisko4/73.20110600_S2D.10.fna")
    plain = tmp_path / "g.fna"
    plain.write_bytes(gzip.open(src).read())
    a = ga.pack_files([str(plain)])
    b = ga.pack_files([src])
    assert (a.words == b.words).all() and (a.runs == b.runs).all()


EDGE_RECORDS = [
    # lower case, U/u, whitespace, CRLF: no break
    b"acgtacgtacgtacgtacgtacguuUUacgtnACGTACGTACGTACGTACGTAC\r\nACGTACGTAC GTACGTA\tCGTACGTA",
    # IUPAC, '-', '.', '*' break k-mers
    b"ACGTRYACGTACGTACGTACGTACGTACGTAC-ACGTACGTACGTACGTACGTACGT.ACGTACGTACGTACGTACGTACGTA*CCCC",
    # short runs (< k) between breaks
    b"ACGTACGTACNACGTACGTACGTACGTACGTANNNNNACGT",
    b"",
    b"NNNNNNNNNNNNNNNNNNNNNNNNNNNNNN",
    b"A" * 20,
    b"A" * 21,
    b"ACGT" * 400,
]


def test_packer_edge_records_match_oracle():
    pk = ga.pack_records([[r] for r in EDGE_RECORDS] + [EDGE_RECORDS])
    recs = packed_records(pk)
    for g, r in enumerate(EDGE_RECORDS):
        assert (oracle.sketch_records(recs[g]) == oracle.sketch_sequence(r)).all(), r
        for run in recs[g]:
            assert len(run) >= 21
    last = len(EDGE_RECORDS)
    assert (oracle.sketch_records(recs[last]) == oracle.sketch_records(EDGE_RECORDS)).all()


def test_packer_fasta_parsing(tmp_path):
    # multi-record FASTA, k-mers never span records; FASTQ; bad format
    seqs = [b"ACGTTGCA" * 10, b"GGGCCCAT" * 12, b"TTAGGCAC" * 9]
    fa = tmp_path / "m.fa"
    fa.write_bytes(b"".join(b">r%d desc\n%s\n%s\n" % (i, s[:30], s[30:]) for i, s in enumerate(seqs)))
    fq = tmp_path / "m.fq"
    fq.write_bytes(b"".join(b"@r%d\n%s\n+\n%s\n" % (i, s, b"I" * len(s)) for i, s in enumerate(seqs)))
    for p in (fa, fq):
        pk = ga.pack_files([str(p)])
        recs = packed_records(pk)
        assert len(recs[0]) == 3
        assert (oracle.sketch_records(recs[0]) == oracle.sketch_file(str(p))).all()
        assert (oracle.sketch_records(recs[0]) == oracle.sketch_records(seqs)).all()
    bad = tmp_path / "bad.fa"
    bad.write_bytes(b"ACGT\n")
    with pytest.raises(ga.GalahGpuError) as e:
        ga.pack_files([str(bad)])
    assert e.value.status == 3
    with pytest.raises(ga.GalahGpuError) as e:
        ga.pack_files([str(tmp_path / "missing.fa")])
    assert e.value.status == 2


def test_packer_random_fuzz_matches_oracle():
    rng = np.random.default_rng(7)
    alphabet = np.frombuffer(b"ACGTACGTACGTacgtNnRYU- \n", dtype=np.uint8)
    genomes = []
    for g in range(12):
        recs = []
        for r in range(rng.integers(1, 5)):
            n = int(rng.integers(0, 3000))
            p = np.where(rng.random(len(alphabet)) < 0.5, 1.0, 0.05)
            p = p / p.sum()
            recs.append(rng.choice(alphabet, size=n, p=p).tobytes())
        genomes.append(recs)
    pk = ga.pack_records(genomes)
    recs = packed_records(pk)
    for g, rs in enumerate(genomes):
        assert (oracle.sketch_records(recs[g], s=200) == oracle.sketch_records(rs, s=200)).all()


# ----------------------------------------------------------- arithmetic ----
def test_ani_matches_oracle_formula():
    for c, t in [(502, 1000), (0, 1000), (0, 0), (1000, 1000), (932, 1039), (460, 1155), (1, 2000),
                 (281, 1325), (418, 1971)]:
        assert ga.ani_f64(c, t) == oracle.ani(c, t)
        assert ga.ani_f32(c, t) == np.float32(oracle.ani(c, t))
    assert ga.ani_f32(502, 1000) == np.float32(0.9808188)
    assert ga.ani_f64(0, 0) == 0.0  # NaN Jaccard -> Rust min/max clamp -> ani 0


def test_parse_percentage_cap_1160():
    assert ga.parse_percentage(90.0) == np.float32(90.0) / np.float32(100.0)
    assert ga.parse_percentage(95) == np.float32(0.95)
    assert ga.parse_percentage(1.0) == np.float32(0.01)
    assert ga.parse_percentage(0.9) == np.float32(0.9)
    assert ga.parse_percentage(0.0) == np.float32(0.0)
    assert float(ga.parse_percentage(90.0)) == 0.8999999761581421
    for bad in (-1.0, 100.5, float("nan")):
        with pytest.raises(ValueError):
            ga.parse_percentage(bad)


@pytest.mark.parametrize("n", [0, 1, 2, 63, 64, 65, 200, 1000, 4097])
@pytest.mark.parametrize("parts", [1, 2, 3, 8])
def test_pair_partition_covers_every_tile_once(n, parts):
    nt = ga.pair_tiles(n)
    nb = (n + 63) // 64
    assert nt == nb * (nb + 1) // 2
    prev = 0
    sizes = []
    for p in range(parts):
        b, e = ga.pair_partition(n, parts, p)
        assert b == prev and e >= b
        prev = e
        pairs = 0
        t = 0
        for I in range(nb):
            for J in range(I, nb):
                if b <= t < e:
                    ri = min(64, n - 64 * I)
                    cj = min(64, n - 64 * J)
                    pairs += ri * (ri - 1) // 2 if I == J else ri * cj
                t += 1
        sizes.append(pairs)
    assert prev == nt
    assert sum(sizes) == n * (n - 1) // 2 if n else True
    if n >= 1000:
        assert max(sizes) - min(sizes) <= 2 * 64 * 64


# --------------------------------------------- reference-interface mirror ----
def test_transform_hello_world():
    # src/sorted_pair_genome_distance_cache.rs:78-96
    cache = ga.SortedPairGenomeDistanceCache()
    cache.insert((1, 2), 0.99)
    assert repr(cache.transform_ids([0, 3])) == "SortedPairGenomeDistanceCache { internal: {} }"
    assert repr(cache.transform_ids([1, 2])) == "SortedPairGenomeDistanceCache { internal: {(0, 1): Some(0.99)} }"
    assert repr(cache.transform_ids([1, 3])) == "SortedPairGenomeDistanceCache { internal: {} }"


def test_transform_multiple():
    # src/sorted_pair_genome_distance_cache.rs:98-113
    cache = ga.SortedPairGenomeDistanceCache()
    cache.insert((1, 2), 0.99)
    cache.insert((1, 4), 0.98)
    assert repr(cache.transform_ids([0, 3])) == "SortedPairGenomeDistanceCache { internal: {} }"
    assert repr(cache.transform_ids([1, 2])) == "SortedPairGenomeDistanceCache { internal: {(0, 1): Some(0.99)} }"
    assert repr(cache.transform_ids([1, 4])) == "SortedPairGenomeDistanceCache { internal: {(0, 1): Some(0.98)} }"
    assert repr(cache.transform_ids([1, 2, 4])) == \
        "SortedPairGenomeDistanceCache { internal: {(0, 1): Some(0.99), (0, 2): Some(0.98)} }"


def test_cache_key_normalisation():
    c = ga.SortedPairGenomeDistanceCache()
    c.insert((5, 3), np.float32(0.9808188))
    assert c.contains_key((3, 5)) and c.contains_key((5, 3))
    assert c.get((3, 5)) == np.float32(0.9808188)
    assert repr(c) == "SortedPairGenomeDistanceCache { internal: {(3, 5): Some(0.9808188)} }"
    d = ga.SortedPairGenomeDistanceCache()
    d.insert((3, 5), np.float32(0.9808188))
    assert c == d


def test_finch_preclusterer_method_name():
    assert ga.FinchPreclusterer(0.9, 1000, 21).method_name() == "finch"


def test_packer_multi_member_gzip_and_decoders(tmp_path, monkeypatch):
    # bgzip-style concatenated gzip members decode to the whole file, with
    # libdeflate (when installed) and with the zlib fallback alike
    recs = [b">a\n" + b"ACGTTGCAAC" * 500 + b"\n", b">b\n" + b"ggcatTTACU" * 700 + b"\nNNNN\nACGT" * 30 + b"\n"]
    gz = tmp_path / "m.fa.gz"
    gz.write_bytes(gzip.compress(recs[0]) + gzip.compress(recs[1]))
    plain = tmp_path / "m.fa"
    plain.write_bytes(recs[0] + recs[1])
    a = ga.pack_files([str(plain)])
    b = ga.pack_files([str(gz)])
    assert (a.words == b.words).all() and (a.runs == b.runs).all()
    assert (oracle.sketch_records(packed_records(a)[0]) == oracle.sketch_file(str(plain))).all()
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); import galah_amd as ga, numpy as np; "
            "a = ga.pack_files([%r]); b = ga.pack_files([%r]); "
            "assert (a.words == b.words).all() and (a.runs == b.runs).all()" % (ROOT, str(plain), str(gz)))
    env = dict(os.environ, GALAHGPU_NO_LIBDEFLATE="1")
    subprocess.run([sys.executable, "-c", code], check=True, env=env)


def reference_runs(seq, k=21):
    """needletail normalize(false) + the "all k bytes in ACGT" window test,
    restated: the maximal A/C/G/T stretches of length >= k (upper case, U as
    T, whitespace dropped without breaking)."""
    out, cur = [], bytearray()
    for ch in seq:
        c = chr(ch)
        if c in " \t\r\n":
            continue
        c = c.upper().replace("U", "T")
        if c in "ACGT":
            cur.append(ord(c))
            continue
        if len(cur) >= k:
            out.append(bytes(cur))
        cur = bytearray()
    if len(cur) >= k:
        out.append(bytes(cur))
    return out


@pytest.mark.parametrize("width", [1, 7, 15, 16, 17, 31, 33, 59, 60, 61, 64, 70, 79, 80, 81, 127])
def test_packer_line_widths_exact_runs(tmp_path, width):
    """Wrapped FASTA at every line width around the packer's 16-byte steps
    (LF and CRLF, lower case, U, IUPAC and N breaks): the packed runs are
    exactly the reference's A/C/G/T stretches, base for base."""
    rng = np.random.default_rng(width)
    body = bytearray(rng.choice(np.frombuffer(b"ACGTacgtU", np.uint8), size=4000,
                                p=[.24, .24, .24, .24, .01, .01, .01, .004, .006]).tobytes())
    for x in rng.integers(0, len(body), 6):
        body[x] = ord("N") if x % 2 else ord("R")
    eol = b"\r\n" if width % 2 else b"\n"
    text = b">r1 test\n" + eol.join(bytes(body[i:i + width]) for i in range(0, len(body), width)) + eol
    p = tmp_path / ("w%d.fa" % width)
    p.write_bytes(text)
    pk = ga.pack_files([str(p)], k=21)
    assert packed_records(pk)[0] == reference_runs(bytes(body))
    pk.free()
