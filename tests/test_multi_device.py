"""Multi-device contexts (gg_create_multi) on one MI355X.

galah calls FinchPreclusterer::distances once, in one process
(src/clusterer.rs:36); with a multi-device context that one call shards
the sketching over the devices, replicates the sketches between them and
partitions the pair tiles (galah_amd/csrc/multi.cpp).  A device ordinal may
repeat in the list -- each entry is then its own shard with its own stream --
so 1, 2 and 3 "devices" are exercised here on the one GPU of the test box:
the results must be identical to the single-device context and to the
oracle, whatever the device count."""
import os

import numpy as np
import pytest

import galah_amd as ga
import oracle
from test_gpu_parity import as_tuples, expected_pairs_from_table, random_sketch_set

pytestmark = pytest.mark.gpu

LISTS = ([0], [0, 0], [0, 0, 0])


def torch_dev():
    import torch
    assert torch.cuda.is_available()
    return torch


def test_precluster_files_same_for_1_2_3_devices(golden):
    min_ani = ga.parse_percentage(90)
    exp = expected_pairs_from_table(golden, min_ani)
    assert len(exp) == 161
    for devs in LISTS:
        with ga.Context(k=21, sketch_size=1000, devices=devs) as ctx:
            assert ctx.device_count == len(devs)
            pairs, ani = ctx.precluster_files(golden["paths"], min_ani)
            assert as_tuples(pairs) == exp, devs
            for r, a in zip(pairs, ani):
                assert a == np.float32(oracle.ani(int(r["common"]), int(r["total"])))
            ph = ctx.phase_times()
            assert ph["sketch"] > 0 and ph["pairs"] > 0
            # every member pair reaches the other directly (one device here;
            # on a node: xGMI peer access), so no copy is staged through host
            assert (ctx.peer_links() == 1).all() and ctx.peer_links().shape == (len(devs), len(devs))
            assert ctx.fallbacks()["peer_staged"] == 0
            line = ctx.info_line()
            assert line.startswith("galahgpu: %d device(s) [%s]" % (len(devs), ",".join(map(str, devs)))), line
            assert "host-staged peer copies 0 (links without peer access 0)" in line


@pytest.mark.parametrize("devs", [[0], [0, 0], [0, 0, 0], [0] * 5])
def test_precluster_files_without_peer_access(golden, monkeypatch, devs):
    """GALAHGPU_TEST_NO_PEER=1 makes every pair of distinct members report no
    peer access (as two GPUs without an xGMI link would): the replication
    takes its host-staged branch (counted in gg_fallbacks) and waits on the
    owners' rows-ready events; pairs and ANI are unchanged."""
    monkeypatch.setenv("GALAHGPU_TEST_NO_PEER", "1")
    min_ani = ga.parse_percentage(90)
    exp = expected_pairs_from_table(golden, min_ani)
    M = len(devs)
    with ga.Context(k=21, sketch_size=1000, devices=devs) as ctx:
        pairs, ani = ctx.precluster_files(golden["paths"], min_ani)
        assert as_tuples(pairs) == exp
        for r, a in zip(pairs, ani):
            assert a == np.float32(oracle.ani(int(r["common"]), int(r["total"])))
        assert (ctx.peer_links() == np.eye(M, dtype=int)).all()
        fb = ctx.fallbacks()
        assert (fb["peer_staged"] > 0) == (M > 1), fb
        assert "links without peer access %d" % (M * M - M if M > 1 else 0) in ctx.info_line()


def test_sketch_and_pairs_host_buffers_multi(golden):
    pk = ga.pack_files(golden["paths"])
    for devs in LISTS[1:]:
        with ga.Context(k=21, sketch_size=1000, devices=devs) as ctx:
            sk, lens = ctx.sketch(pk)
            assert (lens == golden["lens"]).all()
            for g in range(len(lens)):
                assert (sk[g][:lens[g]] == golden["sketches"][g][:lens[g]]).all()
    rng = np.random.default_rng(17)
    sk, lens = random_sketch_set(rng, 257, 1000, 6)
    o = oracle.pairs(sk, lens.astype(np.int32), np.float32(0.9))
    exp = [(int(r["i"]), int(r["j"]), int(r["common"]), int(r["total"])) for r in o]
    for devs in LISTS:
        with ga.Context(k=21, sketch_size=1000, devices=devs) as ctx:
            assert as_tuples(ctx.pairs(sk, lens, np.float32(0.9))) == exp, devs


def test_precluster_shards_2k_synthetic_1_2_3_devices():
    """2,000 synthetic 1 Mbp genomes (clusters of 10) sharded over 1, 2 and 3
    members: identical pairs and ANI, equal to K2 over all tiles on one device
    and to the oracle on the within-cluster pairs."""
    torch = torch_dev()
    n, glen, cl, seed = 2000, 1000000, 10, 21
    thr = ga.parse_percentage(95)
    results = []
    for devs in LISTS:
        with ga.Context(k=21, sketch_size=1000, devices=devs) as ctx:
            M = ctx.device_count
            cuts = [n * m // M for m in range(M + 1)]
            shards, keep = [], []
            for m in range(M):
                g0, g1 = cuts[m], cuts[m + 1]
                mem = ctx.member(m)
                d_words = torch.empty((g1 - g0) * glen // 16, dtype=torch.int32, device="cuda")
                runs = mem.synth_device(g1 - g0, glen, cl, 0.07, seed, d_words, first_genome=g0)
                torch.cuda.synchronize()
                shards.append((d_words, runs, g1 - g0))
                keep.append(d_words)
            pairs, ani = ctx.precluster_shards(shards, thr)
            if M > 1:
                # every member copied the other members' rows with
                # hipMemcpyPeerAsync (multi.cpp replicate: the node's call,
                # here with src == dst device)
                assert ctx.phase_times()["replicate"] > 0
            # at 90% nearly every within-cluster pair passes (> 4096: the
            # host merge's radix sort)
            p90, a90 = ctx.precluster_shards(shards, ga.parse_percentage(90))
            results.append((as_tuples(pairs), ani.tolist(), as_tuples(p90), a90.tolist()))
            t90 = as_tuples(p90)
            assert len(t90) > 4096 and t90 == sorted(t90) and all(i < j for i, j, _, _ in t90)
            if M == 1:
                # the same genomes through the device-resident single-device path
                d_words, runs, _ = shards[0]
                d_sk = torch.zeros((n, 1000), dtype=torch.int64, device="cuda")
                d_len = torch.zeros(n, dtype=torch.int32, device="cuda")
                ctx.sketch_device(d_words, runs, n, d_sk, d_len)
                torch.cuda.synchronize()
                sk = d_sk.cpu().numpy().view(np.uint64)
                ln = d_len.cpu().numpy().view(np.uint32)
                ref = as_tuples(ctx.pairs(sk, ln, thr))
                assert results[0][0] == ref
                ii, jj = [], []
                for c0 in range(0, n, cl):
                    a, b = np.triu_indices(cl, 1)
                    ii.append(a + c0)
                    jj.append(b + c0)
                ii = np.concatenate(ii)
                jj = np.concatenate(jj)
                oc, ot = oracle.pair_list(sk, ln.astype(np.int32), ii, jj)
                opass = oracle.ani_array(oc, ot) >= np.float64(thr)
                exp = sorted((int(i), int(j), int(c), int(t)) for i, j, c, t, p in zip(ii, jj, oc, ot, opass) if p)
                assert [x for x in ref if x[0] // cl == x[1] // cl] == exp
                assert len(exp) > 100
                opass90 = oracle.ani_array(oc, ot) >= np.float64(ga.parse_percentage(90))
                exp90 = sorted((int(i), int(j), int(c), int(t)) for i, j, c, t, p in zip(ii, jj, oc, ot, opass90) if p)
                assert [x for x in t90 if x[0] // cl == x[1] // cl] == exp90
    assert results[1] == results[0] and results[2] == results[0]


def test_file_error_reported_for_lowest_index(golden, tmp_path):
    bad1 = tmp_path / "bad1.fna"
    bad1.write_text("this is not fasta\n")
    bad2 = tmp_path / "bad2.fna"
    bad2.write_text("neither is this\n")
    paths = list(golden["paths"])
    paths.insert(9, str(bad1))
    paths.insert(20, str(bad2))
    paths.insert(24, str(tmp_path / "missing.fna"))
    for devs in LISTS:
        with ga.Context(k=21, sketch_size=1000, devices=devs) as ctx:
            with pytest.raises(ga.GalahGpuError) as e:
                ctx.precluster_files(paths, ga.parse_percentage(90))
            assert "bad1.fna" in str(e.value)
    with pytest.raises(RuntimeError) as e:  # the reference's panic message (src/finch.rs:50)
        ga.distances(paths, 0.9, 1000, 21)
    assert "Failed to sketch genomes with finch" in str(e.value)


def test_host_threads_and_cache_multi(golden, tmp_path):
    min_ani = ga.parse_percentage(90)
    exp = expected_pairs_from_table(golden, min_ani)
    with ga.Context(k=21, sketch_size=1000, devices=[0, 0], host_threads=1) as ctx:
        pairs, _ = ctx.precluster_files(golden["paths"], min_ani)
        assert as_tuples(pairs) == exp
        cache = str(tmp_path / "cache")
        pairs, _ = ctx.precluster_files(golden["paths"], min_ani, cache_dir=cache)
        assert as_tuples(pairs) == exp and ctx.last_cached == 0
        pairs, _ = ctx.precluster_files(golden["paths"], min_ani, cache_dir=cache)
        assert as_tuples(pairs) == exp and ctx.last_cached == len(golden["paths"])
        sk, lens, hits = ctx.sketch_files(golden["paths"], cache_dir=cache)
        assert hits == len(golden["paths"]) and (lens == golden["lens"]).all()
        sk2, lens2, hits2 = ctx.sketch_files(golden["paths"])
        assert hits2 == 0 and (sk2 == sk).all() and (lens2 == lens).all()


def test_devices_env(monkeypatch):
    monkeypatch.setenv("GALAHGPU_DEVICES", "0,0,0")
    with ga.Context(k=21, sketch_size=1000, devices="all") as ctx:
        assert ctx.device_count == 3
        assert ctx.member(2).device == 0
    monkeypatch.delenv("GALAHGPU_DEVICES")
    with ga.Context(k=21, sketch_size=1000, devices="all") as ctx:
        import torch
        assert ctx.device_count == torch.cuda.device_count()


def test_many_small_files_stream_in_batches(tmp_path):
    """More files than one K1 batch (32 genomes) with uneven sizes, some
    without any k-mer: the streamed ingest over 1 and 3 members equals the
    oracle."""
    rng = np.random.default_rng(5)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    paths = []
    for i in range(101):
        L = int(rng.integers(0, 60000)) if i % 13 else 10
        seq = acgt[rng.integers(0, 4, L)].tobytes()
        p = tmp_path / ("g%03d.fna" % i)
        p.write_bytes(b">r\n" + b"\n".join(seq[x:x + 80] for x in range(0, len(seq), 80)) + b"\n")
        paths.append(str(p))
    exp_sk, exp_len = oracle.sketch_files(paths, threads=8)
    for devs in ([0], [0, 0, 0]):
        with ga.Context(k=21, sketch_size=1000, devices=devs, host_threads=3) as ctx:
            sk, lens, _ = ctx.sketch_files(paths)
            assert (lens == exp_len).all()
            for g in range(len(paths)):
                assert (sk[g][:lens[g]] == exp_sk[g][:lens[g]]).all()
                assert (sk[g][lens[g]:] == 0).all()


def test_gzip_list_spread_over_members_in_many_batches(tmp_path, monkeypatch):
    """A gzip list of many more files than one device-inflate batch holds
    (GALAHGPU_GZ_BATCH_FILES=4): files are claimed one at a time across the
    members' lanes, every member inflates batches on its device, none goes
    to the host, and the sketches equal the oracle's for 1 and 3 members."""
    import gzip
    monkeypatch.setenv("GALAHGPU_GZ_BATCH_FILES", "4")
    rng = np.random.default_rng(11)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    paths = []
    for i in range(96):
        seq = acgt[rng.integers(0, 4, int(rng.integers(20000, 80000)))].tobytes()
        p = tmp_path / ("g%03d.fna.gz" % i)
        p.write_bytes(gzip.compress(b">r\n" + b"\n".join(seq[x:x + 80] for x in range(0, len(seq), 80)) + b"\n"))
        paths.append(str(p))
    exp_sk, exp_len = oracle.sketch_files(paths, threads=8)
    for devs in ([0], [0, 0, 0]):
        with ga.Context(k=21, sketch_size=1000, devices=devs) as ctx:
            sk, lens, _ = ctx.sketch_files(paths)
            assert (lens == exp_len).all()
            for g in range(len(paths)):
                assert (sk[g][:lens[g]] == exp_sk[g][:lens[g]]).all()
            assert ctx.fallbacks()["inflate_host"] == 0
            line = ctx.info_line()
            batches = int(line.split("device-inflated ")[1].split(")")[0])
            assert batches >= len(paths) // 4, line
            if len(devs) > 1:  # every member inflated some of them
                per = [int(x) for x in line.rsplit("[", 1)[1].rstrip("]").split(",")]
                assert len(per) == len(devs) and sum(per) == batches and min(per) > 0, line


@pytest.mark.parametrize("min_ani", [0.5, 0.9])
def test_row_range_index_partners_across_members(min_ani):
    """Inverted-index K2 split over 2, 3 and 5 members, each indexing only the
    entries whose hash may occur in its own rows (a Bloom filter of them):
    cluster members are 11 rows apart, so almost every pair's partner row
    belongs to another member's range.  Equal to one device and to the oracle."""
    rng = np.random.default_rng(23)
    n = 800
    sk, lens = random_sketch_set(rng, n, 1000, 11)
    o = oracle.pairs(sk, lens.astype(np.int32), np.float32(min_ani))
    exp = [(int(r["i"]), int(r["j"]), int(r["common"]), int(r["total"])) for r in o]
    assert len(exp) > 1000
    for devs in ([0], [0, 0], [0, 0, 0], [0] * 5):
        with ga.Context(k=21, sketch_size=1000, devices=devs) as ctx:
            assert as_tuples(ctx.pairs(sk, lens, np.float32(min_ani))) == exp, devs
            paths = ctx.pair_paths()  # one index call per member, none abandoned
            assert paths["index"] == len(devs) and paths["index_abandoned"] == 0 and paths["gate"] == 0, paths


def test_precluster_shards_mixed_lengths_s10000_1_vs_3_devices():
    """C5's shape at reduced scale: 900 genomes of 0.2-2 Mbp with N runs,
    s = 10000, sharded over 1 and 3 members (K1 per member, replication of
    80 KB rows, the row-range index at s = 10000): identical pairs and ANI."""
    torch = torch_dev()
    n, cl, s = 900, 10, 10000
    thr = ga.parse_percentage(95)
    results = []
    for devs in ([0], [0, 0, 0]):
        with ga.Context(k=21, sketch_size=s, devices=devs) as ctx:
            M = ctx.device_count
            cuts = [n * m // M for m in range(M + 1)]
            shards, keep = [], []
            for m in range(M):
                g0, g1 = cuts[m], cuts[m + 1]
                lens_bp = ga.synth_mixed_lengths(g1 - g0, 200000, 2000000, cl, 7, first_genome=g0)
                d_words = torch.empty(max(1, int(lens_bp.sum()) // 16), dtype=torch.int32, device="cuda")
                runs = ctx.member(m).synth_mixed_device(lens_bp, cl, 0.07, 1e-4, 8, d_words, first_genome=g0)
                torch.cuda.synchronize()
                shards.append((d_words, runs, g1 - g0))
                keep.append(d_words)
            pairs, ani = ctx.precluster_shards(shards, thr)
            results.append((as_tuples(pairs), ani.tolist()))
    assert len(results[0][0]) > 500
    assert results[1] == results[0]
