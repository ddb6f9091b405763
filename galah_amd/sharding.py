"""Multi-GPU layout of the precluster path.

One process per GPU.  The path shards naturally:
  1. genomes are split into contiguous shards, one per rank, and each rank
     sketches its shard (kernel K1) -- no communication;
  2. ONE exchange step: the [n_local, s] sketch slabs and their lengths are
     replicated on every rank with an all-gather (RCCL over xGMI on MI355X;
     gloo in the CPU tests);
  3. the upper-triangle pair tiles are split into contiguous ranges with
     equal pair counts (gg_pair_partition); each rank runs kernel K2 on its
     range and keeps its passing pairs;
  4. the sparse results are gathered to the host and concatenated; sorting
     by (i, j) gives the same set for any rank count.
"""
import numpy as np

from . import pair_partition, pair_tiles

TILE = 64


def shard_range(n, world, rank):
    """Genomes [g0, g1) of `rank`: contiguous, sizes differ by at most one."""
    base, extra = divmod(n, world)
    g0 = rank * base + min(rank, extra)
    return g0, g0 + base + (1 if rank < extra else 0)


def tile_pairs(n, tile_begin, tile_end):
    """The (i, j) pairs (i < j < n) of tiles [tile_begin, tile_end), in tile
    order -- the host-side statement of what kernel K2 covers."""
    nb = (n + TILE - 1) // TILE
    t = 0
    for I in range(nb):
        row_tiles = nb - I
        if t + row_tiles <= tile_begin:
            t += row_tiles
            continue
        for J in range(I, nb):
            if tile_begin <= t < tile_end:
                for i in range(I * TILE, min(n, I * TILE + TILE)):
                    for j in range(max(J * TILE, i + 1), min(n, J * TILE + TILE)):
                        yield i, j
            t += 1
            if t >= tile_end:
                return


def rank_tiles(n, world, rank):
    return pair_partition(n, world, rank)


def all_gather_sketches(local_sk, local_len, n_total, world, rank, dist, group=None):
    """Replicate per-rank sketch slabs (torch tensors [n_local, s] int64 and
    [n_local] int32) into [n_total, s] / [n_total] on every rank.  Shards of
    unequal size are padded to the largest for the collective and trimmed."""
    import torch
    sizes = [shard_range(n_total, world, r) for r in range(world)]
    m = max(b - a for a, b in sizes)
    s = local_sk.shape[1]
    pad_sk = torch.zeros((m, s), dtype=local_sk.dtype, device=local_sk.device)
    pad_len = torch.zeros(m, dtype=local_len.dtype, device=local_len.device)
    pad_sk[: local_sk.shape[0]] = local_sk
    pad_len[: local_len.shape[0]] = local_len
    out_sk = [torch.empty_like(pad_sk) for _ in range(world)]
    out_len = [torch.empty_like(pad_len) for _ in range(world)]
    dist.all_gather(out_sk, pad_sk, group=group)
    dist.all_gather(out_len, pad_len, group=group)
    sk = torch.cat([o[: b - a] for o, (a, b) in zip(out_sk, sizes)])
    ln = torch.cat([o[: b - a] for o, (a, b) in zip(out_len, sizes)])
    assert sk.shape[0] == n_total
    return sk, ln


def merge_pair_results(parts):
    """Concatenate per-rank pair arrays and sort by (i, j)."""
    if not parts:
        return np.zeros(0, dtype=[("i", np.uint32), ("j", np.uint32), ("common", np.uint32),
                                  ("total", np.uint32)])
    allp = np.concatenate(parts)
    return allp[np.lexsort((allp["j"], allp["i"]))]


__all__ = ["shard_range", "tile_pairs", "rank_tiles", "all_gather_sketches", "merge_pair_results",
           "pair_tiles", "TILE"]
