"""galah_amd -- MI355X-native finch MinHash precluster path for galah.

Python host mirror of the reference interface for this path, over the C ABI
of libgalahgpu.so (include/galahgpu.h):

  reference (AroneyS/galah @ 2024-12-18)              here
  src/lib.rs:23-27     trait PreclusterDistanceFinder  PreclusterDistanceFinder
  src/finch.rs:4-24    struct FinchPreclusterer        FinchPreclusterer
  src/finch.rs:26-75   finch::distances                distances()
  src/sorted_pair_genome_distance_cache.rs:4-59        SortedPairGenomeDistanceCache
  src/cluster_argument_parsing.rs:1160-1182            parse_percentage()

There is no CPU fallback: importing works without a GPU (so the ABI can be
inspected), but every compute call needs a gfx950 device and raises
GalahGpuError otherwise.  The library must have been built in-tree
(`make -C galah_amd/csrc` or __graft_entry__.build()); a missing library is
an ImportError, never a silent substitute.
"""
import ctypes
import logging
import os

import numpy as np

__all__ = [
    "GalahGpuError", "Context", "Packed", "pack_files", "pack_records",
    "ani_f32", "ani_f64", "parse_percentage", "pair_tiles", "pair_partition",
    "SortedPairGenomeDistanceCache", "PreclusterDistanceFinder",
    "FinchPreclusterer", "distances", "PAIR_DTYPE", "LIB_PATH", "EXPORTED_SYMBOLS", "device_runs",
    "partition_preclusters", "precluster_pairs", "preclusters", "LOCAL_PAIR_DTYPE",
    "sketch_cache_load", "sketch_cache_store",
]

HERE = os.path.dirname(os.path.abspath(__file__))
# GALAHGPU_LIB points at an alternate build (A/B kernel experiments)
LIB_PATH = os.environ.get("GALAHGPU_LIB") or os.path.join(HERE, "lib", "libgalahgpu.so")

GG_PAIR_TILE = 64  # include/galahgpu.h: pair tiles are 64 x 64
PAIR_DTYPE = np.dtype([("i", np.uint32), ("j", np.uint32), ("common", np.uint32), ("total", np.uint32)])

# every function include/galahgpu.h declares
EXPORTED_SYMBOLS = (
    "gg_abi_version", "gg_status_string", "gg_last_error", "gg_thread_last_error",
    "gg_create", "gg_destroy", "gg_device",
    "gg_pack_files", "gg_pack_records", "gg_packed_free",
    "gg_sketch", "gg_sketch_device",
    "gg_pair_tiles", "gg_pair_partition", "gg_pairs", "gg_pairs_device",
    "gg_precluster_files", "gg_ani_f64", "gg_ani_f32", "gg_parse_percentage",
    "gg_free", "gg_synth_clustered_device", "gg_timing_enable", "gg_timing_read", "gg_pair_paths",
    "gg_partition_preclusters", "gg_precluster_pairs", "gg_synth_mixed_lengths", "gg_synth_mixed_device",
    "gg_sketch_cache_load", "gg_sketch_cache_store", "gg_sketch_files", "gg_precluster_files_cached",
    "gg_create_multi", "gg_device_count", "gg_device_ctx", "gg_set_host_threads", "gg_phase_times",
    "gg_precluster_shards", "gg_fallbacks", "gg_peer_links", "gg_info_line", "gg_precluster_files_each",
)

GG_OK = 0
GG_ERR_NO_DEVICE = 4


class GalahGpuError(RuntimeError):
    def __init__(self, status, message):
        super().__init__("%s (status %d)" % (message, status))
        self.status = status


class _Run(ctypes.Structure):
    _fields_ = [("genome", ctypes.c_uint32), ("len", ctypes.c_uint32), ("base", ctypes.c_uint64)]


class _Shard(ctypes.Structure):
    _fields_ = [("d_words", ctypes.c_void_p), ("n_words", ctypes.c_uint64), ("runs", ctypes.c_void_p),
                ("n_runs", ctypes.c_uint64), ("n_genomes", ctypes.c_uint32)]


class _Packed(ctypes.Structure):
    _fields_ = [("words", ctypes.POINTER(ctypes.c_uint32)), ("n_words", ctypes.c_uint64),
                ("n_bases", ctypes.c_uint64), ("runs", ctypes.POINTER(_Run)), ("n_runs", ctypes.c_uint64),
                ("n_genomes", ctypes.c_uint32), ("genome_kmers", ctypes.POINTER(ctypes.c_uint64))]


RUN_DTYPE = np.dtype([("genome", np.uint32), ("len", np.uint32), ("base", np.uint64)])

# torch ships its own libamdhip64 (same SONAME as /opt/rocm's).  Load it
# first when it is installed so the process has ONE HIP runtime, shared by
# torch tensors/streams and libgalahgpu; loading ours first would make
# torch load a second runtime beside it.
try:
    import torch  # noqa: F401
except ImportError:  # pragma: no cover - torch is optional for the ABI
    torch = None

if not os.path.exists(LIB_PATH):
    raise ImportError("libgalahgpu.so is not built (%s); run `make -C galah_amd/csrc` "
                      "or __graft_entry__.build()" % LIB_PATH)

_L = ctypes.CDLL(LIB_PATH)
_vp = ctypes.c_void_p
_u32, _u64, _i32 = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int


def _sig(name, res, args):
    try:
        f = getattr(_L, name)
    except AttributeError:
        if "GALAHGPU_LIB" in os.environ:  # (an older build under A/B: its missing entry points stay unbound)
            return
        raise
    f.restype = res
    f.argtypes = args


_sig("gg_abi_version", _u32, [])
_sig("gg_status_string", ctypes.c_char_p, [_i32])
_sig("gg_last_error", ctypes.c_char_p, [_vp])
_sig("gg_thread_last_error", ctypes.c_char_p, [])
_sig("gg_create", _vp, [_i32, _u32, _u64, _i32, ctypes.POINTER(_i32)])
_sig("gg_destroy", None, [_vp])
_sig("gg_device", _i32, [_vp])
_sig("gg_create_multi", _vp, [_i32, _u32, _u64, _vp, _u32, ctypes.POINTER(_i32)])
_sig("gg_device_count", _u32, [_vp])
_sig("gg_device_ctx", _vp, [_vp, _u32])
_sig("gg_set_host_threads", _i32, [_vp, _i32])
_sig("gg_phase_times", _i32, [_vp, _vp])
_sig("gg_precluster_shards", _i32, [_vp, _vp, ctypes.c_float, ctypes.POINTER(_vp), ctypes.POINTER(_vp),
                                    ctypes.POINTER(_u64)])
_sig("gg_pack_files", _i32, [ctypes.POINTER(ctypes.c_char_p), _u32, _i32, _i32, ctypes.POINTER(ctypes.POINTER(_Packed))])
_sig("gg_pack_records", _i32, [ctypes.POINTER(_vp), _vp, _vp, _u64, _u32, _i32, ctypes.POINTER(ctypes.POINTER(_Packed))])
_sig("gg_packed_free", None, [ctypes.POINTER(_Packed)])
_sig("gg_sketch", _i32, [_vp, ctypes.POINTER(_Packed), _vp, _vp])
_sig("gg_sketch_device", _i32, [_vp, _vp, _u64, _vp, _u64, _u32, _vp, _vp, _vp])
_sig("gg_pair_tiles", _u64, [_u32])
_sig("gg_pair_partition", None, [_u32, _u32, _u32, ctypes.POINTER(_u64), ctypes.POINTER(_u64)])
_sig("gg_pairs", _i32, [_vp, _vp, _vp, _u32, ctypes.c_float, ctypes.POINTER(_vp), ctypes.POINTER(_u64)])
_sig("gg_pairs_device", _i32, [_vp, _vp, _vp, _u32, _u64, _u64, ctypes.c_float, _vp, _u64, _vp, _vp])
_sig("gg_precluster_files", _i32, [_vp, ctypes.POINTER(ctypes.c_char_p), _u32, ctypes.c_float,
                                   ctypes.POINTER(_vp), ctypes.POINTER(_vp), ctypes.POINTER(_u64)])
_sig("gg_precluster_files_cached", _i32, [_vp, ctypes.POINTER(ctypes.c_char_p), _u32, ctypes.c_float,
                                          ctypes.c_char_p, ctypes.POINTER(_vp), ctypes.POINTER(_vp),
                                          ctypes.POINTER(_u64), ctypes.POINTER(_u32)])
# gg_pair_sink: int (*)(void* user, const gg_pair* pairs, uint64_t n)
PAIR_SINK = ctypes.CFUNCTYPE(_i32, _vp, _vp, _u64)
_sig("gg_precluster_files_each", _i32, [_vp, ctypes.POINTER(ctypes.c_char_p), _u32, ctypes.c_float, ctypes.c_char_p,
                                        PAIR_SINK, _vp, ctypes.POINTER(_vp), ctypes.POINTER(_vp),
                                        ctypes.POINTER(_u64), ctypes.POINTER(_u32)])
_sig("gg_sketch_files", _i32, [_vp, ctypes.POINTER(ctypes.c_char_p), _u32, ctypes.c_char_p, _vp, _vp,
                               ctypes.POINTER(_u32)])
_sig("gg_sketch_cache_load", _i32, [ctypes.c_char_p, ctypes.c_char_p, _i32, _u32, _u64, _vp,
                                    ctypes.POINTER(_u32), ctypes.POINTER(_i32)])
_sig("gg_sketch_cache_store", _i32, [ctypes.c_char_p, ctypes.c_char_p, _i32, _u32, _u64, _vp, _u32])
_sig("gg_ani_f64", ctypes.c_double, [_u32, _u32, _i32])
_sig("gg_ani_f32", ctypes.c_float, [_u32, _u32, _i32])
_sig("gg_parse_percentage", _i32, [ctypes.c_float, ctypes.POINTER(ctypes.c_float)])
_sig("gg_free", None, [_vp])
_sig("gg_synth_clustered_device", _i32, [_vp, _u32, _u32, _u32, _u32, ctypes.c_float, _u64, _vp, _vp, _vp])
_sig("gg_synth_mixed_lengths", _i32, [_u32, _u32, _u32, _u32, _u32, _u64, _vp])
_sig("gg_synth_mixed_device", _i32, [_vp, _u32, _u32, _vp, _u32, ctypes.c_float, ctypes.c_double, _u64, _vp, _vp,
                                     _u64, ctypes.POINTER(_u64), _vp])
_sig("gg_partition_preclusters", _i32, [_u32, _vp, _u64, _vp, _vp, ctypes.POINTER(_u32)])
_sig("gg_precluster_pairs", _i32, [_u32, _vp, _u64, _vp, _vp, _u32, _vp, _vp])


class _KStats(ctypes.Structure):
    _fields_ = [("ms", ctypes.c_double), ("launches", ctypes.c_uint64), ("work", ctypes.c_uint64)]


_sig("gg_timing_enable", _i32, [_vp, _i32])
_sig("gg_pair_paths", _i32, [_vp, _vp])
_sig("gg_fallbacks", _i32, [_vp, _vp])
_sig("gg_peer_links", _i32, [_vp, _vp])
_sig("gg_info_line", _i32, [_vp, ctypes.c_char_p, ctypes.c_size_t])
FALLBACKS = ("index_to_gate", "index_full_sort", "peer_staged", "sketch_retry", "inflate_host", "sketch_set")  # gg_fallbacks order
_sig("gg_timing_read", _i32, [_vp, _i32, ctypes.POINTER(_KStats)])
KERNEL_SKETCH, KERNEL_FINALIZE, KERNEL_PAIRS, KERNEL_PAIRS_INDEX = 0, 1, 2, 3
# the device-inflate ingest's kernels (gzip lists through precluster_files / sketch_files)
(KERNEL_INFLATE_SEARCH, KERNEL_INFLATE_DECODE, KERNEL_INFLATE_EXPAND, KERNEL_INFLATE_RESOLVE, KERNEL_INFLATE_CRC,
 KERNEL_PARSE, KERNEL_UPLOAD) = range(4, 11)
INGEST_KERNELS = {"search": KERNEL_INFLATE_SEARCH, "decode": KERNEL_INFLATE_DECODE, "expand": KERNEL_INFLATE_EXPAND,
                  "resolve": KERNEL_INFLATE_RESOLVE, "crc": KERNEL_INFLATE_CRC, "parse": KERNEL_PARSE,
                  "upload": KERNEL_UPLOAD}


def lib():
    """The loaded ctypes handle of libgalahgpu.so."""
    return _L


def _ptr(a):
    return a.ctypes.data_as(_vp)


def _thread_err(st):
    return GalahGpuError(st, _L.gg_thread_last_error().decode(errors="replace"))


def abi_version():
    return _L.gg_abi_version()


def ani_f64(common, total, k=21):
    """src/finch.rs:56-64: 1 - finch mash_distance (f64)."""
    return _L.gg_ani_f64(common, total, k)


def ani_f32(common, total, k=21):
    """The stored value, Some(ani as f32) (src/finch.rs:70)."""
    return np.float32(_L.gg_ani_f32(common, total, k))


def parse_percentage(value):
    """CAP:1160-1182 for --precluster-ani: [1,100] -> /100 in f32,
    [0,1) kept, anything else is an error."""
    out = ctypes.c_float()
    st = _L.gg_parse_percentage(ctypes.c_float(value), ctypes.byref(out))
    if st != GG_OK:
        raise ValueError(_L.gg_thread_last_error().decode())
    return np.float32(out.value)


def pair_tiles(n):
    return _L.gg_pair_tiles(n)


def pair_partition(n, parts, part):
    b, e = _u64(), _u64()
    _L.gg_pair_partition(n, parts, part, ctypes.byref(b), ctypes.byref(e))
    return b.value, e.value


LOCAL_PAIR_DTYPE = np.dtype([("precluster", np.uint32), ("i", np.uint32), ("j", np.uint32), ("src", np.uint32)])


def _as_pairs(pairs):
    p = np.zeros(len(pairs), dtype=PAIR_DTYPE)
    for f in ("i", "j"):
        p[f] = pairs[f]
    for f in ("common", "total"):
        if pairs.dtype.names and f in pairs.dtype.names:
            p[f] = pairs[f]
    return p


def synth_mixed_lengths(n_genomes, min_len, max_len, cluster_size, seed, first_genome=0):
    """Config C5 genome lengths: log-uniform in [min_len, max_len] per cluster."""
    lens = np.zeros(max(n_genomes, 1), np.uint32)
    st = _L.gg_synth_mixed_lengths(first_genome, n_genomes, min_len, max_len, cluster_size, seed, _ptr(lens))
    if st != GG_OK:
        raise _thread_err(st)
    return lens[:n_genomes]


def partition_preclusters(n_genomes, pairs):
    """src/clusterer.rs:409-431 partition_sketches + :45-57: single linkage
    over the passing pairs -> (members, offsets): precluster s is
    members[offsets[s]:offsets[s+1]], ascending; largest precluster first,
    ties by smallest member.  Host C++ (union-find), linear in the pairs."""
    p = _as_pairs(pairs)
    members = np.zeros(max(n_genomes, 1), np.uint32)
    offsets = np.zeros(n_genomes + 1, np.uint32)
    ns = _u32()
    st = _L.gg_partition_preclusters(n_genomes, _ptr(p), len(p), _ptr(members), _ptr(offsets), ctypes.byref(ns))
    if st != GG_OK:
        raise _thread_err(st)
    return members[:n_genomes], offsets[:ns.value + 1].copy()


def precluster_pairs(n_genomes, pairs, members, offsets):
    """transform_ids (src/sorted_pair_genome_distance_cache.rs:47-58) for
    every precluster at once -> (local pairs [LOCAL_PAIR_DTYPE] grouped by
    precluster and sorted by (i, j), pair_offsets)."""
    p = _as_pairs(pairs)
    members = np.ascontiguousarray(members, dtype=np.uint32)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint32)
    ns = len(offsets) - 1
    out = np.zeros(max(len(p), 1), LOCAL_PAIR_DTYPE)
    poff = np.zeros(ns + 1, np.uint64)
    st = _L.gg_precluster_pairs(n_genomes, _ptr(p), len(p), _ptr(members), _ptr(offsets), ns, _ptr(out),
                                _ptr(poff))
    if st != GG_OK:
        raise _thread_err(st)
    return out[:len(p)], poff


def preclusters(n_genomes, pairs):
    """The preclusters as galah's cluster() holds them (src/clusterer.rs:45-57):
    a list of ascending index lists, largest first."""
    members, offsets = partition_preclusters(n_genomes, pairs)
    return [members[offsets[s]:offsets[s + 1]].tolist() for s in range(len(offsets) - 1)]


def sketch_cache_load(cache_dir, path, k=21, s=1000, seed=0):
    """the cached bottom-s sketch of a genome file
    (ascending u64 array), or None when there is no valid entry.  Host only."""
    out = np.zeros(max(int(s), 1), dtype=np.uint64)
    n, hit = _u32(), _i32()
    st = _L.gg_sketch_cache_load(os.fsencode(cache_dir), os.fsencode(path), int(k), int(s), int(seed),
                                 _ptr(out), ctypes.byref(n), ctypes.byref(hit))
    if st != GG_OK:
        raise _thread_err(st)
    return out[:n.value].copy() if hit.value else None


def sketch_cache_store(cache_dir, path, hashes, k=21, s=1000, seed=0):
    """Store the sketch of a genome file (strictly ascending, len <= s).  Host only."""
    h = np.ascontiguousarray(hashes, dtype=np.uint64)
    st = _L.gg_sketch_cache_store(os.fsencode(cache_dir), os.fsencode(path), int(k), int(s), int(seed),
                                  _ptr(h), len(h))
    if st != GG_OK:
        raise _thread_err(st)


class Packed:
    """2-bit packed genomes (gg_packed), owned by the library."""

    def __init__(self, ptr):
        self._p = ptr
        self._free = _L.gg_packed_free  # kept: module globals may be gone at interpreter shutdown
        p = ptr.contents
        self.n_words = p.n_words
        self.n_bases = p.n_bases
        self.n_runs = p.n_runs
        self.n_genomes = p.n_genomes
        self.words = np.ctypeslib.as_array(p.words, shape=(max(p.n_words, 1),))[:p.n_words]
        runs_buf = (ctypes.c_char * (max(p.n_runs, 1) * RUN_DTYPE.itemsize)).from_address(
            ctypes.addressof(p.runs.contents))
        self.runs = np.frombuffer(runs_buf, dtype=RUN_DTYPE)[:p.n_runs]
        self.genome_kmers = np.ctypeslib.as_array(p.genome_kmers, shape=(max(p.n_genomes, 1),))[:p.n_genomes]

    def free(self):
        if self._p:
            self._free(self._p)
            self._p = None

    def __del__(self):
        self.free()


def pack_files(paths, k=21, threads=0):
    arr = (ctypes.c_char_p * len(paths))(*[os.fsencode(p) for p in paths])
    out = ctypes.POINTER(_Packed)()
    st = _L.gg_pack_files(arr, len(paths), k, threads, ctypes.byref(out))
    if st != GG_OK:
        raise _thread_err(st)
    return Packed(out)


def pack_records(genomes, k=21):
    """genomes: list (per genome) of lists of record byte strings."""
    recs, gid = [], []
    for g, rs in enumerate(genomes):
        for r in rs:
            recs.append(bytes(r))
            gid.append(g)
    bufs = [ctypes.create_string_buffer(r, len(r) + 1) for r in recs]
    seqs = (_vp * max(len(recs), 1))(*[ctypes.cast(b, _vp) for b in bufs])
    lens = np.array([len(r) for r in recs] or [0], dtype=np.uint64)
    gids = np.array(gid or [0], dtype=np.uint32)
    out = ctypes.POINTER(_Packed)()
    st = _L.gg_pack_records(seqs, _ptr(lens), _ptr(gids), len(recs), len(genomes), k, ctypes.byref(out))
    if st != GG_OK:
        raise _thread_err(st)
    return Packed(out)


def _take_pairs(ptr, n):
    if n == 0:
        _L.gg_free(ptr)
        return np.zeros(0, dtype=PAIR_DTYPE)
    # one memmove into a fresh array (a ctypes array type per call, or
    # np.ctypeslib.as_array, cost ~0.1-0.25 ms at C3's 15k pairs)
    out = np.empty(n, dtype=PAIR_DTYPE)
    ctypes.memmove(out.ctypes.data, ptr.value, n * PAIR_DTYPE.itemsize)
    _L.gg_free(ptr)
    return out


def _dev_ptr(t):
    """Device pointer of a torch tensor or an int."""
    return t if isinstance(t, int) else t.data_ptr()


def device_runs(runs, device):
    """A run table (RUN_DTYPE records) copied to a device tensor of 16-byte
    records, for sketch_device / precluster_shards to read in place."""
    runs = np.ascontiguousarray(runs, dtype=RUN_DTYPE)
    return torch.from_numpy(runs.view(np.uint8).copy()).to(device)


def _runs_arg(runs):
    """(pointer, count, object to keep alive) of a run table: a RUN_DTYPE
    array (host memory) or a device tensor of 16-byte records."""
    if hasattr(runs, "data_ptr") and getattr(runs, "is_cuda", False):
        nbytes = runs.numel() * runs.element_size()
        if nbytes % RUN_DTYPE.itemsize or not runs.is_contiguous():
            raise ValueError("device run table: contiguous 16-byte records")
        return (runs.data_ptr() if nbytes else None), nbytes // RUN_DTYPE.itemsize, runs
    if hasattr(runs, "data_ptr"):  # a host torch tensor of 16-byte records (device_runs(..., "cpu"))
        nbytes = runs.numel() * runs.element_size()
        if nbytes % RUN_DTYPE.itemsize:
            raise ValueError("host run table tensor: 16-byte records")
        runs = runs.contiguous().numpy().view(np.uint8).reshape(-1).view(RUN_DTYPE)
        return runs.ctypes.data, len(runs), runs
    if not (isinstance(runs, np.ndarray) and runs.dtype == RUN_DTYPE):
        raise TypeError("run table: a RUN_DTYPE array or a device tensor of 16-byte records")
    runs = np.ascontiguousarray(runs)
    return runs.ctypes.data, len(runs), runs


PHASES = ("sketch", "replicate", "pairs", "merge")  # gg_phase_times order


class Context:
    """A gg_ctx: fixed k / sketch size / seed on one HIP device (device=...),
    or on several (devices=[...] ordinals, repeats allowed; devices="all":
    every visible device, or GALAHGPU_DEVICES when set)."""

    def __init__(self, k=21, sketch_size=1000, seed=0, device=-1, devices=None, host_threads=0):
        st = _i32()
        if devices is None:
            self._c = _L.gg_create(k, sketch_size, seed, device, ctypes.byref(st))
        elif devices == "all":
            self._c = _L.gg_create_multi(k, sketch_size, seed, None, 0, ctypes.byref(st))
        else:
            arr = (ctypes.c_int * max(len(devices), 1))(*devices)
            self._c = _L.gg_create_multi(k, sketch_size, seed, arr, len(devices), ctypes.byref(st))
        if not self._c:
            raise _thread_err(st.value)
        self.k, self.s, self.seed = k, sketch_size, seed
        # held by the instance: module globals may already be None when a
        # Context is collected at interpreter shutdown
        self._destroy = _L.gg_destroy
        if host_threads:
            self.set_host_threads(host_threads)

    def close(self):
        if getattr(self, "_c", None):
            self._destroy(self._c)
            self._c = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _err(self, st):
        return GalahGpuError(st, _L.gg_last_error(self._c).decode(errors="replace"))

    @property
    def device(self):
        return _L.gg_device(self._c)

    @property
    def device_count(self):
        return _L.gg_device_count(self._c)

    def member(self, i):
        """Member i as a borrowed single-device handle (device-resident calls
        on that member's device); valid while this Context lives."""
        p = _L.gg_device_ctx(self._c, i)
        if not p:
            raise IndexError(i)
        m = Context.__new__(Context)
        m._c, m.k, m.s, m.seed = p, self.k, self.s, self.seed
        m._destroy = lambda _p: None  # owned by self
        m._owner = self
        return m

    def set_host_threads(self, n):
        """galah --threads (CAP:1327-1332): host threads for file ingest (<= 0: default)."""
        st = _L.gg_set_host_threads(self._c, int(n))
        if st != GG_OK:
            raise self._err(st)

    def phase_times(self):
        """Wall-clock ms of the last fused call's phases (PHASES)."""
        out = np.zeros(len(PHASES), np.float64)
        st = _L.gg_phase_times(self._c, _ptr(out))
        if st != GG_OK:
            raise self._err(st)
        return dict(zip(PHASES, out.tolist()))

    def precluster_shards(self, shards, min_ani):
        """shards: one (d_words tensor, runs, n_genomes) per member,
        device-resident on that member's device (runs: a RUN_DTYPE array, or
        a device tensor holding the same 16-byte records, see device_runs)
        -> (pairs sorted by (i, j), ani f32), genomes numbered shard after
        shard."""
        if len(shards) != self.device_count:
            raise ValueError("one shard per device")
        keep = []
        arr = (_Shard * len(shards))()
        for x, (d_words, runs, ng) in enumerate(shards):
            rp, nr, runs = _runs_arg(runs)
            keep.append(runs)
            arr[x].d_words = _dev_ptr(d_words)
            arr[x].n_words = d_words.numel()
            arr[x].runs = rp
            arr[x].n_runs = nr
            arr[x].n_genomes = int(ng)
        pp, ap, cnt = _vp(), _vp(), _u64()
        st = _L.gg_precluster_shards(self._c, arr, ctypes.c_float(min_ani), ctypes.byref(pp), ctypes.byref(ap),
                                     ctypes.byref(cnt))
        if st != GG_OK:
            raise self._err(st)
        return self._pairs_ani(pp, ap, cnt.value)

    @staticmethod
    def _pairs_ani(pp, ap, n):
        if n:
            ani = np.empty(n, np.float32)
            ctypes.memmove(ani.ctypes.data, ap.value, n * 4)
        else:
            ani = np.zeros(0, np.float32)
        _L.gg_free(ap)
        return _take_pairs(pp, n), ani

    def timing_enable(self, on=True):
        st = _L.gg_timing_enable(self._c, 1 if on else 0)
        if st != GG_OK:
            raise self._err(st)

    def pair_paths(self):
        """Which pair kernel ran, counted since the context was created
        (gg_pair_paths): {"index", "index_abandoned", "gate", "other",
        "index_full_sort"} ("index_full_sort" counts the index calls that
        used the full sort instead of the bucketed build)."""
        out = np.zeros(5, np.uint64)
        st = _L.gg_pair_paths(self._c, _ptr(out))
        if st != GG_OK:
            raise self._err(st)
        return dict(zip(("index", "index_abandoned", "gate", "other", "index_full_sort"), (int(x) for x in out)))

    def fallbacks(self):
        """Slow paths taken since the context was created (gg_fallbacks):
        {"index_to_gate", "index_full_sort", "peer_staged", "sketch_retry", "inflate_host", "sketch_set"}."""
        out = np.zeros(len(FALLBACKS), np.uint64)
        st = _L.gg_fallbacks(self._c, _ptr(out))
        if st != GG_OK:
            raise self._err(st)
        return dict(zip(FALLBACKS, (int(x) for x in out)))

    def peer_links(self):
        """[M, M] int array (gg_peer_links): 1 = member a copies from member b
        device to device, 0 = staged through host memory."""
        M = self.device_count
        out = np.zeros(M * M, np.int32)
        st = _L.gg_peer_links(self._c, _ptr(out))
        if st != GG_OK:
            raise self._err(st)
        return out.reshape(M, M)

    def info_line(self):
        """The one-line summary galah would log at info! after distances()."""
        buf = ctypes.create_string_buffer(1024)
        st = _L.gg_info_line(self._c, buf, len(buf))
        if st != GG_OK:
            raise self._err(st)
        return buf.value.decode()

    def timing_read(self, kernel):
        """-> dict(ms, launches, work) summed since timing_enable."""
        k = _KStats()
        st = _L.gg_timing_read(self._c, kernel, ctypes.byref(k))
        if st != GG_OK:
            raise self._err(st)
        return {"ms": k.ms, "launches": k.launches, "work": k.work}

    # -- host-buffer API -------------------------------------------------
    def sketch(self, packed):
        """-> (sketches [n_genomes, s] u64 padded with 0, lens [n] u32)."""
        ng = packed.n_genomes
        out = np.zeros((max(ng, 1), self.s), dtype=np.uint64)
        lens = np.zeros(max(ng, 1), dtype=np.uint32)
        st = _L.gg_sketch(self._c, packed._p, _ptr(out), _ptr(lens))
        if st != GG_OK:
            raise self._err(st)
        return out[:ng], lens[:ng]

    def pairs(self, sketches, lens, min_ani):
        sk = np.ascontiguousarray(sketches, dtype=np.uint64)
        ln = np.ascontiguousarray(lens, dtype=np.uint32)
        n = ln.shape[0]
        if n and sk.shape != (n, self.s):
            raise ValueError("sketches must be [n, sketch_size]")
        outp, cnt = _vp(), _u64()
        st = _L.gg_pairs(self._c, _ptr(sk), _ptr(ln), n, ctypes.c_float(min_ani), ctypes.byref(outp),
                         ctypes.byref(cnt))
        if st != GG_OK:
            raise self._err(st)
        return _take_pairs(outp, cnt.value)

    def sketch_files(self, paths, cache_dir=None):
        """finch sketch_files (src/finch.rs:47) for files -> (sketches [n, s] u64
        padded with 0, lens [n] u32, number of genomes served by cache_dir)."""
        n = len(paths)
        arr = (ctypes.c_char_p * max(n, 1))(*[os.fsencode(p) for p in paths])
        out = np.zeros((max(n, 1), self.s), dtype=np.uint64)
        lens = np.zeros(max(n, 1), dtype=np.uint32)
        hits = _u32()
        st = _L.gg_sketch_files(self._c, arr, n, None if cache_dir is None else os.fsencode(cache_dir),
                                _ptr(out), _ptr(lens), ctypes.byref(hits))
        if st != GG_OK:
            raise self._err(st)
        return out[:n], lens[:n], hits.value

    def precluster_files(self, paths, min_ani, cache_dir=None):
        """-> (pairs structured array sorted by (i, j), ani f32 array).  With
        cache_dir, genomes sketched by an earlier call are read from the
        sketch cache (self.last_cached counts them)."""
        arr = (ctypes.c_char_p * max(len(paths), 1))(*[os.fsencode(p) for p in paths])
        pp, ap, cnt, hits = _vp(), _vp(), _u64(), _u32()
        st = _L.gg_precluster_files_cached(self._c, arr, len(paths), ctypes.c_float(min_ani),
                                           None if cache_dir is None else os.fsencode(cache_dir),
                                           ctypes.byref(pp), ctypes.byref(ap), ctypes.byref(cnt),
                                           ctypes.byref(hits))
        self.last_cached = hits.value
        if st != GG_OK:
            raise self._err(st)
        return self._pairs_ani(pp, ap, cnt.value)

    def precluster_files_each(self, paths, min_ani, each, cache_dir=None):
        """precluster_files, and every compared pair (i < j, all N (N - 1) / 2,
        whatever the ANI) handed to each(block) in (i, j) order as PAIR_DTYPE
        arrays of at most ~4M pairs (gg_precluster_files_each: galah's debug
        level, src/finch.rs:65-68, without holding every pair).  each returning
        True stops the call (GalahGpuError, status 9)."""
        arr = (ctypes.c_char_p * max(len(paths), 1))(*[os.fsencode(p) for p in paths])
        pp, ap, cnt, hits = _vp(), _vp(), _u64(), _u32()
        raised = []

        def sink(_user, ptr, n):
            try:
                blk = np.empty(n, dtype=PAIR_DTYPE)
                if n:
                    ctypes.memmove(blk.ctypes.data, ptr, n * PAIR_DTYPE.itemsize)
                return 1 if each(blk) else 0
            except BaseException as e:  # (an exception may not cross the C frame)
                raised.append(e)
                return 1

        cb = PAIR_SINK(sink)
        st = _L.gg_precluster_files_each(self._c, arr, len(paths), ctypes.c_float(min_ani),
                                         None if cache_dir is None else os.fsencode(cache_dir), cb, None,
                                         ctypes.byref(pp), ctypes.byref(ap), ctypes.byref(cnt), ctypes.byref(hits))
        self.last_cached = hits.value
        if raised:
            raise raised[0]
        if st != GG_OK:
            raise self._err(st)
        return self._pairs_ani(pp, ap, cnt.value)

    # -- device-resident API (torch tensors on this context's device) ---------
    def sketch_device(self, d_words, runs, n_genomes, d_out, d_lens, stream=None):
        rp, nr, runs = _runs_arg(runs)
        st = _L.gg_sketch_device(self._c, _dev_ptr(d_words), d_words.numel(), rp, nr,
                                 n_genomes, _dev_ptr(d_out), _dev_ptr(d_lens),
                                 None if stream is None else stream)
        if st != GG_OK:
            raise self._err(st)

    def pairs_device(self, d_sketches, d_lens, n, tile_begin, tile_end, min_ani, d_out, out_cap, d_count,
                     stream=None):
        st = _L.gg_pairs_device(self._c, _dev_ptr(d_sketches), _dev_ptr(d_lens), n, tile_begin, tile_end,
                                ctypes.c_float(min_ani), _dev_ptr(d_out), out_cap, _dev_ptr(d_count),
                                None if stream is None else stream)
        if st != GG_OK:
            raise self._err(st)

    def synth_mixed_device(self, lens, cluster_size, max_sub_rate, n_run_rate, seed, d_words, stream=None,
                           first_genome=0):
        """Config C5: genomes of lengths `lens` (see synth_mixed_lengths) with
        N runs; -> the host run table (RUN_DTYPE)."""
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        cap = max(1024, int(lens.sum() * max(n_run_rate, 1e-6) * 2) + 4 * len(lens))
        for _ in range(2):
            runs = np.zeros(cap, dtype=RUN_DTYPE)
            nr = _u64()
            st = _L.gg_synth_mixed_device(self._c, first_genome, len(lens), _ptr(lens), cluster_size,
                                          ctypes.c_float(max_sub_rate), ctypes.c_double(n_run_rate), seed,
                                          _dev_ptr(d_words), _ptr(runs), cap, ctypes.byref(nr),
                                          None if stream is None else stream)
            if st == GG_OK:
                return runs[:nr.value]
            if st != 8:
                raise self._err(st)
            cap = nr.value
        raise self._err(st)

    def synth_device(self, n_genomes, genome_len, cluster_size, max_sub_rate, seed, d_words, stream=None,
                     first_genome=0):
        runs = np.zeros(n_genomes, dtype=RUN_DTYPE)
        st = _L.gg_synth_clustered_device(self._c, first_genome, n_genomes, genome_len, cluster_size,
                                          ctypes.c_float(max_sub_rate), seed, _dev_ptr(d_words), _ptr(runs),
                                          None if stream is None else stream)
        if st != GG_OK:
            raise self._err(st)
        return runs


# ---------------------------------------------------------------------------
# Reference-interface mirror
# ---------------------------------------------------------------------------
def _rust_f32_debug(x):
    """Rust `{:?}` of an f32: shortest round-trip decimal, always with a '.'."""
    s = np.format_float_positional(np.float32(x), unique=True, trim="-")
    if "." not in s and "inf" not in s and "nan" not in s:
        s += ".0"
    return s


class SortedPairGenomeDistanceCache:
    """src/sorted_pair_genome_distance_cache.rs:4-59: a map keyed by (min, max)."""

    def __init__(self):
        self.internal = {}

    @staticmethod
    def _key(ids):
        a, b = ids
        return (a, b) if a < b else (b, a)

    def insert(self, genome_ids, distance):
        self.internal[self._key(genome_ids)] = distance

    def get(self, genome_ids):
        """Option<&Option<f32>>: KeyError-free; returns the stored value or the
        sentinel `MISSING` when absent."""
        return self.internal.get(self._key(genome_ids), MISSING)

    def contains_key(self, genome_ids):
        return self._key(genome_ids) in self.internal

    def transform_ids(self, input_ids):
        """:47-58 -- subset with ids re-numbered by position in input_ids."""
        out = SortedPairGenomeDistanceCache()
        for i, g1 in enumerate(input_ids):
            for j in range(i + 1, len(input_ids)):
                v = self.get((g1, input_ids[j]))
                if v is not MISSING:
                    out.insert((i, j), v)
        return out

    def __len__(self):
        return len(self.internal)

    def __eq__(self, other):
        if not isinstance(other, SortedPairGenomeDistanceCache):
            return NotImplemented
        if self.internal.keys() != other.internal.keys():
            return False
        for k, v in self.internal.items():
            w = other.internal[k]
            if (v is None) != (w is None):
                return False
            if v is not None and np.float32(v) != np.float32(w):
                return False
        return True

    def __repr__(self):
        items = ", ".join(
            "(%d, %d): %s" % (k[0], k[1], "None" if v is None else "Some(%s)" % _rust_f32_debug(v))
            for k, v in sorted(self.internal.items()))
        return "SortedPairGenomeDistanceCache { internal: {%s} }" % items


MISSING = object()


class PreclusterDistanceFinder:
    """src/lib.rs:23-27."""

    def distances(self, genome_fasta_paths):
        raise NotImplementedError

    def method_name(self):
        raise NotImplementedError


_CTX_CACHE = {}


def _context(k, s, seed=0):
    """Every visible GPU (or GALAHGPU_DEVICES), as FinchPreclusterer::distances
    uses them; host ingest threads from GALAHGPU_THREADS / the affinity mask."""
    key = (k, s, seed)
    c = _CTX_CACHE.get(key)
    if c is None:
        c = Context(k, s, seed, devices="all")
        _CTX_CACHE[key] = c
    return c


def distances(genome_fasta_paths, min_ani, num_kmers, kmer_length, sketch_cache_dir=None):
    """src/finch.rs:26-75 -> SortedPairGenomeDistanceCache, computed on the GPU.
    sketch_cache_dir (not in galah) reuses sketches of
    unchanged genome files from earlier runs; the result is the same."""
    log = logging.getLogger("galah")
    # At debug level the reference logs every compared pair
    # (src/finch.rs:65-68): the library then streams all N (N - 1) / 2 pairs
    # in row blocks (gg_precluster_files_each), each logged with its f64
    # distance in the reference's loop order; the cache is filled from the
    # passing pairs as at any other level, so no block outlives its lines.
    every = log.isEnabledFor(logging.DEBUG)
    paths = list(genome_fasta_paths)
    k = int(kmer_length)

    def each(block):
        for p in block:
            d = ani_f64(int(p["common"]), int(p["total"]), k)
            log.debug("Comparing %s and %s, distance %s", paths[int(p["i"])], paths[int(p["j"])], rust_f64(d))
        return False

    try:
        ctx = _context(k, int(num_kmers))
        log.info("Sketching MinHash representations of each genome with finch ..")  # src/finch.rs:46
        thr = float(np.float32(min_ani))
        if every:
            pairs, ani = ctx.precluster_files_each(paths, thr, each, cache_dir=sketch_cache_dir)
        else:
            pairs, ani = ctx.precluster_files(paths, thr, cache_dir=sketch_cache_dir)
    except GalahGpuError as e:
        # src/finch.rs:50
        raise RuntimeError("Failed to sketch genomes with finch: %s" % e) from e
    log.info("Finished sketching genomes")  # src/finch.rs:48
    log.info(ctx.info_line())  # device count, phase times, fallbacks (gg_info_line)
    cache = SortedPairGenomeDistanceCache()
    for p, a in zip(pairs, ani):
        cache.insert((int(p["i"]), int(p["j"])), np.float32(a))
    return cache


def rust_f64(x):
    """Rust's `{}` of an f64: the shortest round-trip digits, no exponent, no
    trailing ".0" (1.0 -> "1", 0.0 -> "0")."""
    x = float(x)
    if x != x:
        return "NaN"
    if x in (float("inf"), float("-inf")):
        return "inf" if x > 0 else "-inf"
    r = repr(x)
    if "e" in r or "E" in r:
        m, e = r.lower().split("e")
        neg = m.startswith("-")
        m = m.lstrip("-")
        digits = m.replace(".", "")
        point = (m.index(".") if "." in m else len(m)) + int(e)
        if point <= 0:
            r = "0." + "0" * (-point) + digits
        elif point >= len(digits):
            r = digits + "0" * (point - len(digits))
        else:
            r = digits[:point] + "." + digits[point:]
        r = ("-" if neg else "") + r
    if r.endswith(".0"):
        r = r[:-2]
    return r


class FinchPreclusterer(PreclusterDistanceFinder):
    """src/finch.rs:4-24: min_ani is a fraction (f32), num_kmers = s, kmer_length = k."""

    def __init__(self, min_ani, num_kmers=1000, kmer_length=21, sketch_cache_dir=None):
        self.min_ani = np.float32(min_ani)
        self.num_kmers = int(num_kmers)
        self.kmer_length = int(kmer_length)
        self.sketch_cache_dir = sketch_cache_dir

    def distances(self, genome_fasta_paths):
        return distances(genome_fasta_paths, self.min_ani, self.num_kmers, self.kmer_length,
                         sketch_cache_dir=self.sketch_cache_dir)

    def method_name(self):
        return "finch"
