"""Sketch cache: per-genome sketches on disk keyed by
the genome file's identity, so a repeated run skips ingest and K1.  galah
itself re-sketches every file on every call (src/finch.rs:47), so the only
parity requirement is that the cache never changes a result: a hit must
return exactly the sketch of the golden fixtures / the GPU path, and any
change to the file or the parameters must miss.

CPU tests drive the host-only store/load entry points with the golden
sketches; the -m gpu tests run gg_sketch_files / gg_precluster_files_cached
with and without the cache."""
import os
import shutil

import numpy as np
import pytest

import galah_amd as ga
from conftest import golden_path, load_golden_sketches


@pytest.fixture()
def genomes(tmp_path):
    """Three golden genomes copied to a scratch directory (their mtimes may be
    changed), with their golden k=21, s=1000 sketches."""
    names, sk, lens = load_golden_sketches()
    pick = [names.index(n) for n in ("set1/1mbp.fna", "set1/500kb.fna", "set1_name_clash/500kb.fna")]
    paths, sketches = [], []
    for n, i in enumerate(pick):
        dst = tmp_path / ("g%d.fna.gz" % n)
        shutil.copyfile(golden_path(names[i]), dst)
        paths.append(str(dst))
        sketches.append(sk[i][:lens[i]].copy())
    return paths, sketches


def test_store_then_load_round_trip(tmp_path, genomes):
    paths, sks = genomes
    cache = str(tmp_path / "cache" / "nested")  # created on first store
    for p, h in zip(paths, sks):
        assert ga.sketch_cache_load(cache, p) is None
        ga.sketch_cache_store(cache, p, h)
    for p, h in zip(paths, sks):
        got = ga.sketch_cache_load(cache, p)
        assert got is not None and got.dtype == np.uint64 and (got == h).all()
    # one file per (genome, k); no temporaries left behind
    assert sorted(os.listdir(cache)) == sorted(f for f in os.listdir(cache) if f.endswith(".k21.ggsk"))
    assert len(os.listdir(cache)) == 3


def test_prefix_serves_smaller_sketch_sizes_only(tmp_path, genomes):
    paths, sks = genomes
    cache = str(tmp_path / "c")
    ga.sketch_cache_store(cache, paths[0], sks[0], s=1000)
    for s in (1, 10, 500, 999, 1000):
        got = ga.sketch_cache_load(cache, paths[0], s=s)
        assert (got == sks[0][:s]).all()
    assert ga.sketch_cache_load(cache, paths[0], s=1001) is None


def test_short_sketch_prefix(tmp_path, genomes):
    # a genome with fewer distinct k-mers than s keeps all of them (no_strict)
    paths, sks = genomes
    cache = str(tmp_path / "c")
    ga.sketch_cache_store(cache, paths[0], sks[0][:37], s=1000)
    assert (ga.sketch_cache_load(cache, paths[0], s=1000) == sks[0][:37]).all()
    assert (ga.sketch_cache_load(cache, paths[0], s=20) == sks[0][:20]).all()
    ga.sketch_cache_store(cache, paths[1], sks[0][:0], s=1000)  # empty sketch
    got = ga.sketch_cache_load(cache, paths[1], s=1000)
    assert got is not None and len(got) == 0


def test_parameters_and_file_identity_invalidate(tmp_path, genomes):
    paths, sks = genomes
    cache = str(tmp_path / "c")
    ga.sketch_cache_store(cache, paths[0], sks[0])
    assert ga.sketch_cache_load(cache, paths[0], k=21, seed=0) is not None
    assert ga.sketch_cache_load(cache, paths[0], k=20) is None
    assert ga.sketch_cache_load(cache, paths[0], seed=1) is None
    assert ga.sketch_cache_load(cache, paths[1]) is None  # other file
    # same path through another spelling resolves to the same entry
    rel = os.path.relpath(paths[0])
    assert (ga.sketch_cache_load(cache, rel) == sks[0]).all()
    # touching the file (mtime) invalidates
    st = os.stat(paths[0])
    os.utime(paths[0], ns=(st.st_atime_ns, st.st_mtime_ns + 1000))
    assert ga.sketch_cache_load(cache, paths[0]) is None
    # rewriting it with other content invalidates too
    ga.sketch_cache_store(cache, paths[0], sks[0])
    with open(paths[0], "ab") as f:
        f.write(b"\n")
    os.utime(paths[0], ns=(st.st_atime_ns, st.st_mtime_ns + 1000))  # same mtime as the entry
    assert ga.sketch_cache_load(cache, paths[0]) is None  # size differs
    # a missing genome file is a miss, not an error
    assert ga.sketch_cache_load(cache, str(tmp_path / "absent.fna")) is None


def test_corrupt_or_truncated_entries_miss(tmp_path, genomes):
    paths, sks = genomes
    cache = tmp_path / "c"
    ga.sketch_cache_store(str(cache), paths[0], sks[0])
    (entry,) = list(cache.iterdir())
    raw = bytearray(entry.read_bytes())
    assert raw[:8] == b"GGSKETCH" and len(raw) == 64 + len(os.path.realpath(paths[0])) + 8 * len(sks[0])
    flipped = bytearray(raw)
    flipped[-3] ^= 0x10  # one hash bit
    entry.write_bytes(bytes(flipped))
    assert ga.sketch_cache_load(str(cache), paths[0]) is None
    entry.write_bytes(bytes(raw[:-8]))  # truncated
    assert ga.sketch_cache_load(str(cache), paths[0]) is None
    entry.write_bytes(b"")
    assert ga.sketch_cache_load(str(cache), paths[0]) is None
    entry.write_bytes(bytes(raw))
    assert (ga.sketch_cache_load(str(cache), paths[0]) == sks[0]).all()


def test_store_rejects_invalid_sketches(tmp_path, genomes):
    paths, sks = genomes
    cache = str(tmp_path / "c")
    with pytest.raises(ga.GalahGpuError):
        ga.sketch_cache_store(cache, paths[0], sks[0][::-1])  # not ascending
    with pytest.raises(ga.GalahGpuError):
        ga.sketch_cache_store(cache, paths[0], np.array([5, 5], np.uint64))  # duplicate
    with pytest.raises(ga.GalahGpuError):
        ga.sketch_cache_store(cache, paths[0], sks[0], s=999)  # longer than s
    with pytest.raises(ga.GalahGpuError):
        ga.sketch_cache_store(cache, str(tmp_path / "absent.fna"), sks[0])
    assert ga.sketch_cache_load(cache, paths[0]) is None


# ----------------------------------------------------------------- GPU ----
@pytest.mark.gpu
def test_gpu_sketch_files_with_cache(tmp_path, genomes, gpu_ctx):
    paths, sks = genomes
    cache = str(tmp_path / "c")
    ref, ref_lens, hits = gpu_ctx.sketch_files(paths)
    assert hits == 0
    for g, h in enumerate(sks):
        assert ref_lens[g] == len(h) and (ref[g][:len(h)] == h).all()
    sk1, ln1, hits1 = gpu_ctx.sketch_files(paths, cache_dir=cache)
    assert hits1 == 0 and (sk1 == ref).all() and (ln1 == ref_lens).all()
    assert len(os.listdir(cache)) == len(paths)
    gpu_ctx.timing_enable(True)
    sk2, ln2, hits2 = gpu_ctx.sketch_files(paths, cache_dir=cache)
    st = gpu_ctx.timing_read(ga.KERNEL_SKETCH)
    gpu_ctx.timing_enable(False)
    assert hits2 == len(paths) and st["launches"] == 0  # K1 skipped
    assert (sk2 == ref).all() and (ln2 == ref_lens).all()
    # one genome changes: only it is re-sketched
    s0 = os.stat(paths[1])
    os.utime(paths[1], ns=(s0.st_atime_ns, s0.st_mtime_ns + 1))
    sk3, ln3, hits3 = gpu_ctx.sketch_files(paths, cache_dir=cache)
    assert hits3 == len(paths) - 1 and (sk3 == ref).all() and (ln3 == ref_lens).all()


@pytest.mark.gpu
def test_gpu_precluster_files_cached_equals_uncached(tmp_path, golden, gpu_ctx):
    paths = golden["paths"]
    cache = str(tmp_path / "c")
    min_ani = ga.parse_percentage(90)
    p0, a0 = gpu_ctx.precluster_files(paths, min_ani)
    p1, a1 = gpu_ctx.precluster_files(paths, min_ani, cache_dir=cache)
    assert gpu_ctx.last_cached == 0
    p2, a2 = gpu_ctx.precluster_files(paths, min_ani, cache_dir=cache)
    assert gpu_ctx.last_cached == len(paths)
    for p, a in ((p1, a1), (p2, a2)):
        assert (p == p0).all() and (a == a0).all()
    exp = {(i, j): (c, t) for i, j, c, t, _ in golden["pairs"] if ga.ani_f64(c, t) >= float(min_ani)}
    got = {(int(r["i"]), int(r["j"])): (int(r["common"]), int(r["total"])) for r in p2}
    assert got == exp
    # the Python mirror of the trait with a cache gives galah's cache
    fp = ga.FinchPreclusterer(min_ani, 1000, 21, sketch_cache_dir=cache)
    assert fp.distances(paths) == ga.FinchPreclusterer(min_ani, 1000, 21).distances(paths)


@pytest.mark.gpu
def test_gpu_cache_serves_smaller_sketch_size(tmp_path, genomes):
    paths, sks = genomes
    cache = str(tmp_path / "c")
    with ga.Context(k=21, sketch_size=1000, seed=0) as big:
        big.sketch_files(paths, cache_dir=cache)
    with ga.Context(k=21, sketch_size=400, seed=0) as small:
        ref, ref_lens, _ = small.sketch_files(paths)
        sk, ln, hits = small.sketch_files(paths, cache_dir=cache)
    assert hits == len(paths) and (sk == ref).all() and (ln == ref_lens).all()
    for g, h in enumerate(sks):
        assert (sk[g][:ln[g]] == h[:400]).all()
