"""Compressed FASTA inputs: gzip, bzip2 and xz, as finch's parser reads them.

galah sketches its genome paths through finch -> needletail 0.5
(src/finch.rs:47; Cargo.toml:30,32), whose reader picks gzip, bzip2 or xz by
the file's magic bytes.  needletail's source is not in the container, so this
behaviour is restated (parity unpinned): the same FASTA as plain text, gzip,
bzip2 and xz -- single streams and concatenated ones -- must give the same
genome everywhere.

CPU: gg_pack_files packs all four identically, and a corrupt bzip2 / xz file
fails with a decode error naming it.  GPU: sketches through
gg_precluster_files / gg_sketch_files are identical whatever the compression,
on the device-inflate path (the list starts with gzip files: bzip2 and xz
files are decoded on the host as they are staged) and on the host path."""
import bz2
import gzip
import lzma
import os

import numpy as np
import pytest

import galah_amd as ga
import oracle
from conftest import golden_path
from test_host import packed_records

ACGT = np.frombuffer(b"ACGT", np.uint8)


def fasta(seed, n_rec=3, rec_len=40000):
    rng = np.random.default_rng(seed)
    out = b""
    for r in range(n_rec):
        seq = ACGT[rng.integers(0, 4, rec_len)].tobytes().lower() if r == 1 else ACGT[rng.integers(0, 4, rec_len)].tobytes()
        out += b">rec%d some header\n" % r + b"\n".join(seq[i:i + 70] for i in range(0, len(seq), 70)) + b"\n"
    return out


def half(data):
    return data[:len(data) // 2], data[len(data) // 2:]


def variants(tmp, name, text):
    """The same FASTA text as plain, gzip, bzip2, xz, and as concatenated
    streams of each compression (two halves of the text)."""
    a, b = half(text)
    out = {
        "plain": text,
        "gz": gzip.compress(text),
        "bz2": bz2.compress(text),
        "xz": lzma.compress(text),
        "gz2": gzip.compress(a) + gzip.compress(b),
        "bz22": bz2.compress(a) + bz2.compress(b),
        "xz2": lzma.compress(a) + lzma.compress(b),
    }
    paths = {}
    for k, data in out.items():
        p = os.path.join(tmp, "%s.%s" % (name, k))
        with open(p, "wb") as f:
            f.write(data)
        paths[k] = p
    return paths


def same_packing(pk, g0, g1):
    return packed_records(pk)[g0] == packed_records(pk)[g1]


def test_pack_files_same_for_every_compression(tmp_path):
    texts = [fasta(1), open_golden_text()]
    for t, text in enumerate(texts):
        paths = variants(str(tmp_path), "g%d" % t, text)
        keys = list(paths)
        pk = ga.pack_files([paths[k] for k in keys], threads=3)
        recs = packed_records(pk)
        for g, k in enumerate(keys):
            assert recs[g] == recs[0], k
        assert sum(len(r) for r in recs[0]) > 0


def open_golden_text():
    with gzip.open(golden_path("set1/500kb.fna"), "rb") as f:
        return f.read()


def test_corrupt_bzip2_and_xz_fail_naming_the_file(tmp_path):
    text = fasta(2)
    for ext, data in (("bz2", bz2.compress(text)), ("xz", lzma.compress(text))):
        bad = bytearray(data)
        bad[len(bad) // 2] ^= 0x5A
        p = tmp_path / ("bad.fa." + ext)
        p.write_bytes(bytes(bad))
        with pytest.raises(ga.GalahGpuError) as e:
            ga.pack_files([str(p)])
        assert "decode error in" in str(e.value) and "bad.fa." + ext in str(e.value)
        trunc = tmp_path / ("trunc.fa." + ext)
        trunc.write_bytes(data[:len(data) // 2])
        with pytest.raises(ga.GalahGpuError):
            ga.pack_files([str(trunc)])


def test_fastq_in_bzip2_and_xz(tmp_path):
    rng = np.random.default_rng(3)
    seq = ACGT[rng.integers(0, 4, 3000)].tobytes()
    fq = b"@r1\n" + seq + b"\n+\n" + b"I" * len(seq) + b"\n"
    paths = []
    for ext, data in (("fq", fq), ("fq.bz2", bz2.compress(fq)), ("fq.xz", lzma.compress(fq))):
        p = tmp_path / ("reads." + ext)
        p.write_bytes(data)
        paths.append(str(p))
    recs = packed_records(ga.pack_files(paths))
    assert recs[0] == recs[1] == recs[2] and recs[0] == [seq]


# ---------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("inflate", ["device", "host", "auto"])
def test_sketches_same_for_every_compression(tmp_path, monkeypatch, inflate):
    """A list led by gzip files (the device-inflate default) with the same
    genomes in every compression further on: identical sketches, equal to
    the oracle's; no batch goes back to the host."""
    if inflate == "auto":
        monkeypatch.delenv("GALAHGPU_INFLATE", raising=False)
    else:
        monkeypatch.setenv("GALAHGPU_INFLATE", inflate)
    texts = [fasta(10 + t, rec_len=60000) for t in range(3)]
    keys = None
    paths = []
    for t, text in enumerate(texts):
        v = variants(str(tmp_path), "g%d" % t, text)
        # (two gzip members hand their batch to the host: test_inflate.py)
        keys = ["gz"] + [k for k in v if k not in ("gz", "gz2")]
        paths += [v[k] for k in keys]
    exp_sk, exp_len = oracle.sketch_files([p for p in paths if p.endswith(".gz")], threads=4)
    with ga.Context(k=21, sketch_size=1000) as ctx:
        sk, lens, _ = ctx.sketch_files(paths)
        fb = ctx.fallbacks()
        line = ctx.info_line()
    assert fb["inflate_host"] == 0
    if inflate != "host":
        assert "(device-inflated 0)" not in line, line
    per = len(keys)
    for t in range(len(texts)):
        for q in range(per):
            g = t * per + q
            assert lens[g] == exp_len[t], (t, keys[q])
            assert (sk[g][:lens[g]] == exp_sk[t][:exp_len[t]]).all(), (t, keys[q])
    # pairs through gg_precluster_files: every variant of a genome is an identical copy
    with ga.Context(k=21, sketch_size=1000) as ctx:
        pairs, ani = ctx.precluster_files(paths, ga.parse_percentage(99))
    assert len(pairs) == len(texts) * per * (per - 1) // 2
    assert (ani == np.float32(1.0)).all()


@pytest.mark.gpu
def test_device_inflate_chosen_by_magic_not_name(tmp_path, monkeypatch):
    """gzip files whose names do not end in .gz, and a list whose first file
    is plain FASTA: the device inflate is chosen by the bytes (the info line
    counts device-inflated batches) and the sketches equal the oracle's."""
    monkeypatch.delenv("GALAHGPU_INFLATE", raising=False)
    texts = [fasta(20 + t) for t in range(4)]
    paths = []
    p = tmp_path / "first_plain.fna"
    p.write_bytes(texts[0])
    paths.append(str(p))
    for t in range(1, 4):
        p = tmp_path / ("g%d.fasta" % t)
        p.write_bytes(gzip.compress(texts[t]))
        paths.append(str(p))
    exp_sk, exp_len = oracle.sketch_files(paths, threads=4)
    with ga.Context(k=21, sketch_size=1000) as ctx:
        sk, lens, _ = ctx.sketch_files(paths)
        line = ctx.info_line()
    assert "(device-inflated 0)" not in line and "host-inflated batches 0" in line, line
    assert (lens == exp_len).all()
    for g in range(len(paths)):
        assert (sk[g][:lens[g]] == exp_sk[g][:lens[g]]).all()
