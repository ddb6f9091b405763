"""The CPU oracle against the reference's own known answers, then the
committed golden fixtures against the oracle.  CPU only."""
import json
import os

import numpy as np
import pytest

import oracle
from conftest import GOLD, golden_path


def test_finch_rs_hello_world_known_answer():
    # src/finch.rs:89-97: distances([set1/1mbp, set1/500kb], 0.9, 1000, 21)
    # == {(0,1): Some(0.9808188)}
    a = oracle.sketch_file(golden_path("set1/1mbp.fna"))
    b = oracle.sketch_file(golden_path("set1/500kb.fna"))
    c, t = oracle.raw_distance(a, b)
    ani = oracle.ani(c, t)
    assert np.float32(ani) == np.float32(0.9808188)
    assert ani >= np.float64(np.float32(0.9))
    # src/finch.rs:99-106: empty at 0.99
    assert not ani >= np.float64(np.float32(0.99))
    p = oracle.pairs(np.stack([np.pad(a, (0, 1000 - len(a))), np.pad(b, (0, 1000 - len(b)))]),
                     np.array([len(a), len(b)], np.int32), np.float32(0.9))
    assert len(p) == 1 and p[0]["ani"] == np.float32(0.9808188)
    assert len(oracle.pairs(np.stack([a, np.pad(b, (0, 1000 - len(b)))]), np.array([len(a), len(b)], np.int32),
                            np.float32(0.99))) == 0


def test_published_murmur3_vectors():
    with open(os.path.join(GOLD, "murmur3_kat.json")) as f:
        kat = json.load(f)
    for e in kat["published"]:
        assert oracle.murmur3_x64_128(e["input"].encode()) == (e["h1"], e["h2"])
    for e in kat["kmers21"]:
        assert oracle.murmur3_h1(e["kmer"].encode()) == e["h1"]


def _pair(golden, a, b):
    names = golden["names"]
    ia, ib = names.index(a), names.index(b)
    i, j = min(ia, ib), max(ia, ib)
    for r in golden["pairs"]:
        if r[0] == i and r[1] == j:
            return r
    raise KeyError((a, b))


def test_threshold_facts_from_reference_tests(golden):
    # pass facts at min_ani 0.9 pinned by the reference
    thr = np.float64(np.float32(0.9))
    passing = [
        ("abisko4/73.20120800_S1D.21.fna", "abisko4/73.20110800_S2M.16.fna"),   # test_cmdline.rs:8-57
        ("set1/500kb.fna", "set1/1mbp.fna"),                                    # finch.rs:89-97
        ("set2/1mbp.fna", "set2/1mbp.half_aligned.fna"),                        # test_cmdline.rs:216-255
        ("antonio_mags/BE_RX_R2_MAG52.fna", "antonio_mags/BE_RX_R3_MAG189.fna"),  # test_cmdline.rs:316-338
    ]
    for a, b in passing:
        r = _pair(golden, a, b)
        assert oracle.ani(r[2], r[3]) >= thr, (a, b, r)
    # set1_name_clash/500kb is an unrelated random sequence (test_cmdline.rs:122-155)
    r = _pair(golden, "set1/500kb.fna", "set1_name_clash/500kb.fna")
    assert not oracle.ani(r[2], r[3]) >= thr
    # src/clusterer.rs:482-612: the 4 abisko4 genomes form one connected
    # component at 0.9
    four = ["abisko4/73.20120800_S1X.13.fna", "abisko4/73.20120600_S2D.19.fna",
            "abisko4/73.20120700_S3X.12.fna", "abisko4/73.20110800_S2D.13.fna"]
    parent = {x: x for x in four}

    def find(x):
        while parent[x] != x:
            x = parent[x]
        return x
    for x in range(4):
        for y in range(x + 1, 4):
            r = _pair(golden, four[x], four[y])
            if oracle.ani(r[2], r[3]) >= thr:
                parent[find(four[x])] = find(four[y])
    assert len({find(x) for x in four}) == 1


def test_survey_representative_values(golden):
    # SURVEY.md 8(c) survey-time restatement values (quoted to 7 digits)
    r = _pair(golden, "abisko4/73.20120800_S1X.13.fna", "abisko4/73.20110800_S2D.13.fna")
    assert r[2:4] == (932, 1039) and abs(r[4] - 0.9973421) < 1e-6
    r = _pair(golden, "antonio_mags/BE_RX_R2_MAG52.fna", "antonio_mags/BE_RX_R3_MAG189.fna")
    assert r[2:4] == (460, 1155) and abs(r[4] - 0.9732040) < 1e-6
    r = _pair(golden, "set2/1mbp.fna", "set2/1mbp.half_aligned.fna")
    assert r[2:4] == (502, 1469) and abs(r[4] - 0.9678786) < 1e-6
    assert sum(1 for r in golden["pairs"] if oracle.ani(r[2], r[3]) >= np.float64(np.float32(0.9))) == 161


def test_golden_sketches_match_oracle(golden):
    sk, lens = oracle.sketch_files(golden["paths"], threads=4)
    assert (lens == golden["lens"]).all()
    assert (sk == golden["sketches"]).all()
    n = len(golden["names"])
    full = oracle.pairs(sk, lens, 0.0)
    assert len(full) == n * (n - 1) // 2
    table = {(r[0], r[1]): r[2:] for r in golden["pairs"]}
    for r in full:
        c, t, a = table[(int(r["i"]), int(r["j"]))]
        assert (r["common"], r["total"], r["ani"]) == (c, t, a)


def test_golden_sketch_shape(golden):
    sk, lens = golden["sketches"], golden["lens"]
    assert sk[golden["names"].index("set1/1mbp.fna")][0] == 0x0000032cdc7a8856
    assert sk[golden["names"].index("abisko4/73.20120800_S1X.13.fna")][0] == 0x0000040655b767f9
    assert sk[golden["names"].index("antonio_mags/BE_RX_R2_MAG52.fna")][0] == 0x00000da009708230
    for row, n in zip(sk, lens):
        assert n == 1000
        assert (np.diff(row[:n].astype(np.uint64)) > 0).all()  # strictly ascending => distinct


def test_oracle_plain_and_gzip_agree(tmp_path):
    import gzip
    src = golden_path("fraglen_test/sequence1.fna")
    plain = tmp_path / "s.fna"
    plain.write_bytes(gzip.open(src).read())
    assert (oracle.sketch_file(str(plain)) == oracle.sketch_file(src)).all()


@pytest.mark.parametrize("s,expected", [
    (b"ACGTNACGTACGTACGTACGTACGTA", None),
])
def test_oracle_kmer_breaks(s, expected):
    # a non-ACGT byte breaks k-mers; lower case / U / whitespace do not
    a = oracle.sketch_sequence(b"acgtacgtacgtacgtacgtauuuacg\nacgtacg tacg")
    b = oracle.sketch_sequence(b"ACGTACGTACGTACGTACGTATTTACGACGTACGTACG")
    assert (a == b).all()
    c = oracle.sketch_sequence(s)
    d = oracle.sketch_sequence(s[5:])
    assert (c == d).all()  # the 4 bases before the N form no 21-mer
