"""SURVEY.md 8(f) rows 1 and 3, CPU only: the union-find precluster
partition and the all-at-once transform_ids of libgalahgpu.so against
galah's own loops restated in oracle/ (src/clusterer.rs:409-431, :45-57;
src/sorted_pair_genome_distance_cache.rs:47-58)."""
import numpy as np
import pytest

import galah_amd as ga
import oracle
from conftest import load_golden_pairs


def pair_array(rows):
    p = np.zeros(len(rows), ga.PAIR_DTYPE)
    for k, r in enumerate(rows):
        p[k] = (r[0], r[1], 0, 0)
    return p


def check(n, rows):
    p = pair_array(rows)
    got = ga.preclusters(n, p)
    exp = oracle.partition_sketches(n, [(int(a), int(b)) for a, b, *_ in rows])
    assert got == exp
    members, offsets = ga.partition_preclusters(n, p)
    cache = {(min(int(a), int(b)), max(int(a), int(b))): k for k, (a, b, *_) in enumerate(rows)}
    local, poff = ga.precluster_pairs(n, p, members, offsets)
    for s in range(len(offsets) - 1):
        ids = members[offsets[s]:offsets[s + 1]].tolist()
        want = oracle.transform_ids(cache, ids)
        seg = local[int(poff[s]):int(poff[s + 1])]
        assert (seg["precluster"] == s).all()
        assert [(int(r["i"]), int(r["j"])) for r in seg] == sorted(want)
        assert {(int(r["i"]), int(r["j"])): int(r["src"]) for r in seg} == want


def test_golden_pairs_preclusters():
    # the 27 tests/data genomes at 0.9 (161 pairs), in the reference's order
    rows = [(i, j) for (i, j, c, t, a) in load_golden_pairs() if oracle.ani(c, t) >= np.float64(np.float32(0.9))]
    assert len(rows) == 161
    check(27, rows)


@pytest.mark.parametrize("seed", range(6))
def test_random_graphs(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 300))
    m = int(rng.integers(0, 3 * n))
    rows = set()
    for _ in range(m):
        a, b = rng.integers(0, n, 2)
        if a != b:
            rows.add((int(min(a, b)), int(max(a, b))))
    rows = sorted(rows)
    if seed % 2:
        rows = [(b, a) for a, b in rows[::-1]]  # any order, either orientation
    check(n, rows)


def test_edges():
    check(1, [])
    check(5, [])
    check(4, [(0, 3), (1, 2)])          # equal sizes: smallest member first
    check(6, [(4, 5), (0, 1), (1, 2)])
    members, offsets = ga.partition_preclusters(0, pair_array([]))
    assert len(members) == 0 and list(offsets) == [0]
    with pytest.raises(ga.GalahGpuError):
        ga.partition_preclusters(3, pair_array([(0, 3)]))
    m, o = ga.partition_preclusters(4, pair_array([(0, 1)]))
    with pytest.raises(ga.GalahGpuError):  # pair across preclusters
        ga.precluster_pairs(4, pair_array([(0, 2)]), m, o)


def test_clusterer_rs_abisko4_fact():
    # src/clusterer.rs:482-612: at 0.9 the finch pair graph joins the 4
    # abisko4 genomes S1X.13, S2D.19, S3X.12, S2D.13 into one precluster
    from conftest import load_golden_sketches
    names, _, _ = load_golden_sketches()
    want = ["abisko4/73.20120800_S1X.13.fna", "abisko4/73.20120600_S2D.19.fna",
            "abisko4/73.20120700_S3X.12.fna", "abisko4/73.20110800_S2D.13.fna"]
    idx = [names.index(w) for w in want]
    pos = {g: k for k, g in enumerate(idx)}
    rows = [(pos[i], pos[j]) for (i, j, c, t, a) in load_golden_pairs()
            if i in pos and j in pos and oracle.ani(c, t) >= np.float64(np.float32(0.9))]
    assert ga.preclusters(4, pair_array(rows)) == [[0, 1, 2, 3]]
