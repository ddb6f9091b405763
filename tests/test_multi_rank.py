"""The N > 1 path on CPU: world_size 2 (and 3) with the gloo backend.

Each rank sketches its genome shard, the sketches are all-gathered
(galah_amd.sharding.all_gather_sketches, the step RCCL performs on the GPU
node), each rank evaluates its tile range of the pair space, and the
merged result must equal the single-process result.  The per-rank compute
here is the CPU oracle standing in for kernels K1/K2 (which need a GPU);
what is tested is the sharding, the exchange and the partition."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from galah_amd import sharding

N_GENOMES = 19
GLEN = 12000


def genomes():
    rng = np.random.default_rng(42)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    out = []
    for c in range(0, N_GENOMES, 4):
        root = rng.integers(0, 4, GLEN)
        for m in range(min(4, N_GENOMES - c)):
            g = root.copy()
            mut = rng.random(GLEN) < 0.01 * m
            g[mut] = (g[mut] + rng.integers(1, 4, mut.sum())) % 4
            out.append(acgt[g].tobytes())
    return out


def sketch_all(seqs):
    sk = np.zeros((len(seqs), 1000), np.uint64)
    ln = np.zeros(len(seqs), np.int32)
    for g, q in enumerate(seqs):
        v = oracle.sketch_sequence(q)
        sk[g, :len(v)] = v
        ln[g] = len(v)
    return sk, ln


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    seqs = genomes()
    g0, g1 = sharding.shard_range(N_GENOMES, world, rank)
    sk_loc, ln_loc = sketch_all(seqs[g0:g1])
    sk, ln = sharding.all_gather_sketches(torch.from_numpy(sk_loc.view(np.int64)), torch.from_numpy(ln_loc),
                                          N_GENOMES, world, rank, dist)
    sk = sk.numpy().view(np.uint64)
    ln = ln.numpy()
    b, e = sharding.rank_tiles(N_GENOMES, world, rank)
    rows = []
    for i, j in sharding.tile_pairs(N_GENOMES, b, e):
        c, t = oracle.raw_distance(sk[i][:ln[i]], sk[j][:ln[j]])
        if oracle.ani(c, t) >= np.float64(np.float32(0.9)):
            rows.append((i, j, c, t))
    gathered = [None] * world
    dist.all_gather_object(gathered, rows)
    if rank == 0:
        q.put((sk, ln, gathered))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_precluster_equals_single_process(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    sk, ln, gathered = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ref_sk, ref_ln = sketch_all(genomes())
    assert (sk == ref_sk).all() and (ln == ref_ln).all()
    dt = [("i", np.uint32), ("j", np.uint32), ("common", np.uint32), ("total", np.uint32)]
    parts = [np.array(rows, dtype=dt) for rows in gathered]
    merged = sharding.merge_pair_results(parts)
    ref = oracle.pairs(ref_sk, ref_ln, np.float32(0.9))
    assert [tuple(map(int, r)) for r in merged] == \
        [(int(r["i"]), int(r["j"]), int(r["common"]), int(r["total"])) for r in ref]
    assert len(ref) > 0


@pytest.mark.parametrize("n", [1, 63, 64, 65, 130, 1000])
@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_tile_partition_covers_all_pairs_once(n, world):
    seen = set()
    for r in range(world):
        b, e = sharding.rank_tiles(n, world, r)
        for p in sharding.tile_pairs(n, b, e):
            assert p not in seen
            seen.add(p)
    assert len(seen) == n * (n - 1) // 2


def test_shard_range():
    for n in (0, 1, 7, 10000):
        for w in (1, 2, 3, 8):
            rs = [sharding.shard_range(n, w, r) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
            assert max(b - a for a, b in rs) - min(b - a for a, b in rs) <= 1
