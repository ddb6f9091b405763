"""ctypes binding of the CPU oracle (oracle/finch_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package galah_amd/.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libfinch_oracle.so")

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        u64p = ctypes.POINTER(ctypes.c_uint64)
        L.oracle_murmur3_h1.restype = ctypes.c_uint64
        L.oracle_murmur3_h1.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint64]
        L.oracle_murmur3_x64_128.restype = None
        L.oracle_murmur3_x64_128.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint64, u64p]
        L.oracle_sketch_file.restype = ctypes.c_int
        L.oracle_sketch_file.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p]
        L.oracle_sketch_sequence.restype = ctypes.c_int
        L.oracle_sketch_sequence.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_uint64, ctypes.c_void_p]
        L.oracle_sketch_records.restype = ctypes.c_int
        L.oracle_sketch_records.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p]
        L.oracle_sketch_files.restype = ctypes.c_int
        L.oracle_sketch_files.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.c_uint32, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p,
                                          ctypes.c_void_p]
        L.oracle_raw_distance.restype = None
        L.oracle_raw_distance.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                                          u64p, u64p]
        L.oracle_ani.restype = ctypes.c_double
        L.oracle_ani.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int]
        L.oracle_pairs.restype = ctypes.c_uint64
        L.oracle_pairs.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                   ctypes.c_int, ctypes.c_float] + [ctypes.c_void_p] * 5 + [ctypes.c_uint64]
        L.oracle_pairs_parallel.restype = ctypes.c_uint64
        L.oracle_pairs_parallel.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                            ctypes.c_int, ctypes.c_float, ctypes.c_int, u64p]
        L.oracle_pair_list.restype = None
        L.oracle_pair_list.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_int]
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def murmur3_h1(data: bytes, seed: int = 0) -> int:
    return lib().oracle_murmur3_h1(data, len(data), seed)


def murmur3_x64_128(data: bytes, seed: int = 0):
    out = (ctypes.c_uint64 * 2)()
    lib().oracle_murmur3_x64_128(data, len(data), seed, out)
    return out[0], out[1]


def sketch_file(path: str, k: int = 21, s: int = 1000, seed: int = 0) -> np.ndarray:
    out = np.empty(max(s, 1), dtype=np.uint64)
    n = lib().oracle_sketch_file(path.encode(), k, s, seed, _ptr(out))
    if n < 0:
        raise IOError("oracle failed to sketch %s" % path)
    return out[:n].copy()


def sketch_sequence(seq: bytes, k: int = 21, s: int = 1000, seed: int = 0) -> np.ndarray:
    buf = np.frombuffer(seq, dtype=np.uint8)
    out = np.empty(max(s, 1), dtype=np.uint64)
    n = lib().oracle_sketch_sequence(_ptr(buf), len(seq), k, s, seed, _ptr(out))
    if n < 0:
        raise RuntimeError("oracle sketch failed")
    return out[:n].copy()


def sketch_records(records, k: int = 21, s: int = 1000, seed: int = 0) -> np.ndarray:
    """records: list of bytes objects (one FASTA record each, no header)."""
    offs = np.zeros(len(records) + 1, dtype=np.uint64)
    for i, r in enumerate(records):
        offs[i + 1] = offs[i] + len(r)
    buf = np.frombuffer(b"".join(records) or b"\0", dtype=np.uint8)
    out = np.empty(max(s, 1), dtype=np.uint64)
    n = lib().oracle_sketch_records(_ptr(buf), _ptr(offs), len(records), k, s, seed, _ptr(out))
    if n < 0:
        raise RuntimeError("oracle sketch failed")
    return out[:n].copy()


def sketch_files(paths, k: int = 21, s: int = 1000, seed: int = 0, threads: int = 1):
    """finch::sketch_files restated: returns (padded [n, s] u64, lens int32)."""
    n = len(paths)
    arr = (ctypes.c_char_p * n)(*[p.encode() for p in paths])
    out = np.zeros((n, max(s, 1)), dtype=np.uint64)
    lens = np.zeros(n, dtype=np.int32)
    bad = lib().oracle_sketch_files(arr, n, k, s, seed, threads, _ptr(out), _ptr(lens))
    if bad:
        raise IOError("oracle failed to sketch %s" % paths[bad - 1])
    return out, lens


def raw_distance(a: np.ndarray, b: np.ndarray):
    a = np.ascontiguousarray(a, dtype=np.uint64)
    b = np.ascontiguousarray(b, dtype=np.uint64)
    c = ctypes.c_uint64()
    t = ctypes.c_uint64()
    lib().oracle_raw_distance(_ptr(a), len(a), _ptr(b), len(b), ctypes.byref(c), ctypes.byref(t))
    return c.value, t.value


def ani(common: int, total: int, k: int = 21) -> float:
    return lib().oracle_ani(common, total, k)


def pairs(sketches: np.ndarray, lens: np.ndarray, min_ani: float, k: int = 21, cap: int = None):
    """src/finch.rs:53-73 restated.  Returns a structured array of passing
    pairs (i, j, common, total, ani) in the reference's loop order."""
    sketches = np.ascontiguousarray(sketches, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.int32)
    n, stride = sketches.shape
    if cap is None:
        cap = n * (n - 1) // 2
    cap = max(cap, 1)
    oi = np.empty(cap, np.uint32)
    oj = np.empty(cap, np.uint32)
    oc = np.empty(cap, np.uint32)
    ot = np.empty(cap, np.uint32)
    oa = np.empty(cap, np.float32)
    cnt = lib().oracle_pairs(_ptr(sketches), _ptr(lens), n, stride, k, ctypes.c_float(min_ani),
                             _ptr(oi), _ptr(oj), _ptr(oc), _ptr(ot), _ptr(oa), cap)
    m = min(cnt, cap)
    out = np.empty(m, dtype=[("i", np.uint32), ("j", np.uint32), ("common", np.uint32),
                             ("total", np.uint32), ("ani", np.float32)])
    out["i"], out["j"], out["common"], out["total"], out["ani"] = oi[:m], oj[:m], oc[:m], ot[:m], oa[:m]
    return out


def pair_list(sketches, lens, pi, pj, threads=8):
    """finch raw_distance (common, total) of the pairs (pi[x], pj[x])."""
    sketches = np.ascontiguousarray(sketches, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.int32)
    pi = np.ascontiguousarray(pi, dtype=np.uint32)
    pj = np.ascontiguousarray(pj, dtype=np.uint32)
    oc = np.zeros(max(len(pi), 1), np.uint32)
    ot = np.zeros(max(len(pi), 1), np.uint32)
    lib().oracle_pair_list(_ptr(sketches), _ptr(lens), sketches.shape[1], _ptr(pi), _ptr(pj), len(pi),
                           _ptr(oc), _ptr(ot), threads)
    return oc[:len(pi)], ot[:len(pi)]


def ani_array(common, total, k=21):
    """oracle_ani over arrays (same f64 expression, element by element)."""
    L = lib()
    return np.array([L.oracle_ani(int(c), int(t), k) for c, t in zip(common, total)], dtype=np.float64)


def pairs_parallel(sketches, lens, min_ani, k=21, threads=1):
    sketches = np.ascontiguousarray(sketches, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.int32)
    n, stride = sketches.shape
    cs = ctypes.c_uint64()
    cnt = lib().oracle_pairs_parallel(_ptr(sketches), _ptr(lens), n, stride, k, ctypes.c_float(min_ani),
                                      threads, ctypes.byref(cs))
    return cnt, cs.value


# --------------------------------------------------------------------------
# After distances(): galah's own loops, restated in plain Python (small N).
# --------------------------------------------------------------------------
def partition_sketches(n_genomes, pair_keys):
    """src/clusterer.rs:409-431 restated: for i, for j < i, join(i, j) iff
    the cache contains (i, j) (key normalised to (min, max)), then
    src/clusterer.rs:45-57: each set sorted ascending, sets ordered by size
    descending.  Ties among equal sizes are left to the reference's
    DisjointSetVec::sets() + sort_unstable; here they are ordered by
    smallest member (Python's sort is stable over first-member order)."""
    keys = {(min(a, b), max(a, b)) for a, b in pair_keys}
    parent = list(range(n_genomes))

    def find(x):
        while parent[x] != x:
            x = parent[x]
        return x

    for i in range(n_genomes):
        for j in range(i):
            if (j, i) in keys:
                ri, rj = find(i), find(j)
                if ri != rj:
                    parent[max(ri, rj)] = min(ri, rj)
    sets = {}
    for g in range(n_genomes):
        sets.setdefault(find(g), []).append(g)
    out = sorted(sets.values(), key=lambda s: s[0])
    out.sort(key=lambda s: -len(s))
    return out


def transform_ids(cache, input_ids):
    """src/sorted_pair_genome_distance_cache.rs:47-58 restated over a dict
    {(i, j): value} with i < j."""
    out = {}
    for i, g1 in enumerate(input_ids):
        for j in range(i + 1, len(input_ids)):
            g2 = input_ids[j]
            k = (min(g1, g2), max(g1, g2))
            if k in cache:
                out[(i, j)] = cache[k]
    return out
