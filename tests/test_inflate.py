"""The device gzip inflate (galah_amd/csrc/inflate.hip, inflate_core.hpp;
GALAHGPU_INFLATE=device): gzip FASTA goes to the GPU compressed and is
inflated there.

CPU: the DEFLATE core (the bit-level decoding the kernels run) decodes every
stream both serially and as the device does -- block starts searched every
`chunk` bytes, one independent decode per start, back-references placed as
pointers and followed -- and both equal zlib, for the reference's test
genomes and for streams of every block type and zlib strategy.

GPU: sketches and pairs with the device inflate equal the host path and the
committed golden table; the cases it hands back to the host (several gzip
members, FASTQ, a corrupt stream) give the host path's result or error and
are counted."""
import gzip
import json
import os
import subprocess
import zlib

import numpy as np
import pytest

import galah_amd as ga
import oracle
from conftest import GOLD_DATA, ROOT

BIN = os.path.join(ROOT, "tests", "cpp", "build", "test_inflate_core")


def golden_gz():
    out = []
    for d, _, fs in os.walk(GOLD_DATA):
        out += [os.path.join(d, f) for f in sorted(fs) if f.endswith(".gz")]
    return sorted(out)


def synthetic_streams(tmp):
    rng = np.random.default_rng(8)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    seq = acgt[rng.integers(0, 4, 400000)].tobytes()
    fa = b"".join(b">rec%d header text\n" % i + b"\n".join(seq[j:j + 60] for j in range(i * 20000, (i + 1) * 20000, 60))
                  + b"\n" for i in range(20))
    paths = []

    def put(name, data, level=6, strategy=zlib.Z_DEFAULT_STRATEGY):
        c = zlib.compressobj(level, zlib.DEFLATED, 31, 8, strategy)
        p = os.path.join(tmp, name)
        with open(p, "wb") as f:
            f.write(c.compress(data) + c.flush())
        paths.append(p)

    for lvl in (0, 1, 6, 9):
        put("l%d.fa.gz" % lvl, fa, lvl)
    for name, strat in (("huff", zlib.Z_HUFFMAN_ONLY), ("rle", zlib.Z_RLE), ("fixed", zlib.Z_FIXED)):
        put(name + ".fa.gz", fa, 6, strat)
    put("nrun.fa.gz", fa.replace(b"ACGTA", b"NNNNNNNNNNNNNN"))
    put("tiny.fa.gz", b">x\nACGT\n")
    put("empty.gz", b"")
    put("binary.gz", rng.integers(0, 256, 200000, dtype=np.uint8).tobytes())
    return paths


@pytest.fixture(scope="module")
def core_binary():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")])
    return BIN


@pytest.mark.parametrize("chunk,window", [(4096, 0), (300, 0), (4096, 20000), (65536, 100000)])
def test_core_chunked_decode_equals_zlib(core_binary, tmp_path, chunk, window):
    """window > 0: the staged device decode's windows (a block body longer
    than the LDS stage continues from the last sub-span's end); with 64 KB
    chunks most segments hold several blocks."""
    paths = golden_gz() + synthetic_streams(str(tmp_path))
    r = subprocess.run([core_binary, "--chunk", str(chunk), "--window", str(window)] + paths, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    rows = [json.loads(x) for x in r.stdout.splitlines()]
    assert len(rows) == len(paths)
    # the search finds block starts in the multi-block streams
    big = [x for x in rows if x["file"].endswith("l6.fa.gz") or "abisko4" in x["file"]]
    assert big and all(x["starts_found"] > 1 for x in big)
    if window:  # (bodies longer than a window were decoded in several)
        assert sum(x["windows"] for x in rows) > sum(x["lanes"] for x in rows)


# ---------------------------------------------------------------------------
def sketch_files(paths, monkeypatch, inflate, k=21, s=1000):
    monkeypatch.setenv("GALAHGPU_INFLATE", inflate)
    with ga.Context(k=k, sketch_size=s) as ctx:
        sk, lens, _ = ctx.sketch_files([str(p) for p in paths])
        fb = ctx.fallbacks()
    return sk, lens, fb


@pytest.mark.gpu
def test_device_inflate_golden(golden, monkeypatch):
    sk, lens, fb = sketch_files(golden["paths"], monkeypatch, "device")
    assert fb["inflate_host"] == 0
    assert (lens == golden["lens"]).all()
    for g in range(len(lens)):
        assert (sk[g][:lens[g]] == golden["sketches"][g][:lens[g]]).all(), golden["names"][g]
    monkeypatch.setenv("GALAHGPU_INFLATE", "device")
    thr = ga.parse_percentage(90)
    with ga.Context(k=21, sketch_size=1000) as ctx:
        pairs, ani = ctx.precluster_files(golden["paths"], thr)
        assert ctx.fallbacks()["inflate_host"] == 0
    exp = [(i, j, c, t) for (i, j, c, t, a) in golden["pairs"] if oracle.ani(c, t) >= np.float64(np.float32(thr))]
    assert [(int(r["i"]), int(r["j"]), int(r["common"]), int(r["total"])) for r in pairs] == exp


@pytest.mark.gpu
def test_device_inflate_streams_and_handbacks(tmp_path, monkeypatch):
    """Every block type and zlib strategy, several gzip members, FASTQ, plain
    FASTA beside gzip files, many files in one batch: the host path's
    sketches; the members / FASTQ batches are handed back and counted."""
    rng = np.random.default_rng(3)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    paths = [p for p in synthetic_streams(str(tmp_path)) if not p.endswith(("empty.gz", "binary.gz"))]
    for i in range(60):  # many small genomes in one batch
        seq = acgt[rng.integers(0, 4, int(rng.integers(20000, 300000)))].tobytes()
        p = tmp_path / ("g%02d.fna.gz" % i)
        p.write_bytes(gzip.compress(b">g%d\n" % i + b"\n".join(seq[j:j + 80] for j in range(0, len(seq), 80)) + b"\n"))
        paths.append(str(p))
    plain = tmp_path / "plain.fa"
    plain.write_bytes(b">p\n" + acgt[rng.integers(0, 4, 50000)].tobytes() + b"\n")
    paths.append(str(plain))
    hsk, hl, _ = sketch_files(paths, monkeypatch, "host")
    dsk, dl, fb = sketch_files(paths, monkeypatch, "device")
    assert fb["inflate_host"] == 0
    assert (dl == hl).all() and all((dsk[g][:dl[g]] == hsk[g][:hl[g]]).all() for g in range(len(paths)))
    # two concatenated members: inflated on the device (its boundary found
    # by the decode); FASTQ: the batch goes back to the host
    seq = acgt[rng.integers(0, 4, 100000)].tobytes()
    multi = tmp_path / "multi.fa.gz"
    multi.write_bytes(gzip.compress(b">m\n" + seq[:50000]) + gzip.compress(seq[50000:] + b"\n"))
    fq = tmp_path / "reads.fq.gz"
    fq.write_bytes(gzip.compress(b"@r1\n" + seq[:5000] + b"\n+\n" + b"I" * 5000 + b"\n"))
    for extra, host_batches in ((multi, 0), (fq, 1)):
        ps = paths[:3] + [str(extra)]
        hsk, hl, _ = sketch_files(ps, monkeypatch, "host")
        dsk, dl, fb = sketch_files(ps, monkeypatch, "device")
        assert fb["inflate_host"] == host_batches, extra
        assert (dl == hl).all() and all((dsk[g][:dl[g]] == hsk[g][:hl[g]]).all() for g in range(len(ps)))


def bgzip(data, level=6, block=65280, eof=True):
    """BGZF (bgzip; SAM/BAM specification 4.1): members of <= 64 KB of
    input, each header with the 'BC' extra subfield holding the member's
    size - 1, then the 28-byte empty end-of-file member."""
    out = []
    for i in range(0, max(len(data), 1), block):
        chunk = data[i:i + block]
        c = zlib.compressobj(level, zlib.DEFLATED, -15)
        body = c.compress(chunk) + c.flush()
        bsize = 18 + len(body) + 8 - 1
        hdr = bytes([0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 66, 67, 2, 0]) + bsize.to_bytes(2, "little")
        out.append(hdr + body + zlib.crc32(chunk).to_bytes(4, "little") + (len(chunk) & 0xffffffff).to_bytes(4, "little"))
    if eof:
        out.append(bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000"))
    return b"".join(out)


def fasta_text(rng, n, name, width=80):
    seq = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, n)].tobytes()
    return b">%s\n" % name + b"\n".join(seq[j:j + width] for j in range(0, len(seq), width)) + b"\n"


@pytest.mark.gpu
def test_device_inflate_gzip_members(tmp_path, monkeypatch):
    """needletail 0.5 (Cargo.toml:32, behind src/finch.rs:47) reads a file of
    several gzip members as one stream.  bgzip (BGZF) files -- their members
    known from the headers' size field -- and concatenated members of plain
    gzip (`cat a.gz b.gz`, boundaries found by the decode) in a list with
    single-member files: every batch inflated on the device (inflate_host 0),
    sketches equal to the oracle's (zlib's gzread reads every member)."""
    rng = np.random.default_rng(31)
    paths = []
    for i in range(6):  # bgzip: 1.2 Mbp, ~19 members of 64 KB each + the EOF member
        p = tmp_path / ("bgz%d.fna.gz" % i)
        p.write_bytes(bgzip(fasta_text(rng, 1200000, b"bgz%d" % i), level=1 + i % 9))
        paths.append(str(p))
    for i in range(4):  # concatenated: 2-5 members of random sizes, some beyond a search chunk
        parts, text = [], fasta_text(rng, int(rng.integers(300000, 900000)), b"cat%d" % i)
        cuts = sorted(rng.choice(np.arange(1, len(text)), size=1 + i, replace=False).tolist())
        for a, b in zip([0] + cuts, cuts + [len(text)]):
            parts.append(gzip.compress(text[a:b], 6))
        p = tmp_path / ("cat%d.fna.gz" % i)
        p.write_bytes(b"".join(parts))
        paths.append(str(p))
    for i in range(3):  # single members between them
        p = tmp_path / ("one%d.fna.gz" % i)
        p.write_bytes(gzip.compress(fasta_text(rng, 700000, b"one%d" % i), 6))
        paths.insert(3 * i + 1, str(p))
    small = tmp_path / "bgz_small.fna.gz"  # one data member + the EOF member
    small.write_bytes(bgzip(fasta_text(rng, 20000, b"small")))
    paths.append(str(small))
    exp_sk, exp_len = oracle.sketch_files(paths, threads=8)
    for batch_files in ("4096", "3"):
        monkeypatch.setenv("GALAHGPU_GZ_BATCH_FILES", batch_files)
        monkeypatch.setenv("GALAHGPU_INFLATE", "device")
        with ga.Context(k=21, sketch_size=1000) as ctx:
            sk, lens, _ = ctx.sketch_files(paths)
            fb = ctx.fallbacks()
            line = ctx.info_line()
        assert fb["inflate_host"] == 0, line
        assert "inflate replans: members " in line and "members 0," not in line, line
        assert (lens == exp_len).all()
        for g in range(len(paths)):
            assert (sk[g][:lens[g]] == exp_sk[g][:lens[g]]).all(), paths[g]
    # a member header after the last member's end that is cut short: the host path's result
    bad = tmp_path / "cat_trailing.fna.gz"
    bad.write_bytes(gzip.compress(fasta_text(rng, 100000, b"t"), 6) + b"\x1f\x8b\x08\x00")
    errs = {}
    for mode in ("host", "device"):
        monkeypatch.setenv("GALAHGPU_INFLATE", mode)
        with ga.Context(k=21, sketch_size=1000) as ctx:
            try:
                sk, lens, _ = ctx.sketch_files([str(bad)])
                errs[mode] = ("ok", sk[0][:lens[0]].tolist())
            except ga.GalahGpuError as e:
                errs[mode] = (e.status, str(e))
    assert errs["device"] == errs["host"]


@pytest.mark.gpu
def test_device_inflate_full_areas_after_a_tight_plan(tmp_path, monkeypatch):
    """Token areas are first sized at 1/4 token per compressed bit; a stream
    denser than that (Huffman-only over a 2-letter alphabet: ~1 token per
    1.x bits) fills them, and the batch is planned again with full areas --
    same sketches as the host path, no batch handed back, the replan counted
    in the info line.  GALAHGPU_GZ_TIGHT=0 starts with full areas."""
    rng = np.random.default_rng(41)
    paths = []
    for i in range(3):
        seq = np.frombuffer(b"AC", np.uint8)[rng.integers(0, 2, 600000)].tobytes()
        text = b">dense%d\n" % i + b"\n".join(seq[j:j + 70] for j in range(0, len(seq), 70)) + b"\n"
        c = zlib.compressobj(6, zlib.DEFLATED, 31, 8, zlib.Z_HUFFMAN_ONLY)
        p = tmp_path / ("dense%d.fna.gz" % i)
        p.write_bytes(c.compress(text) + c.flush())
        paths.append(str(p))
    hsk, hl, _ = sketch_files(paths, monkeypatch, "host")
    for tight in ("1", "0"):
        monkeypatch.setenv("GALAHGPU_GZ_TIGHT", tight)
        monkeypatch.setenv("GALAHGPU_INFLATE", "device")
        with ga.Context(k=21, sketch_size=1000) as ctx:
            dsk, dl, _ = ctx.sketch_files(paths)
            fb = ctx.fallbacks()
            line = ctx.info_line()
        assert fb["inflate_host"] == 0, line
        assert ("full areas 0;" in line) == (tight == "0"), line
        assert (dl == hl).all() and all((dsk[g][:dl[g]] == hsk[g][:hl[g]]).all() for g in range(len(paths)))


@pytest.mark.gpu
def test_device_inflate_blocks_longer_than_the_stage(tmp_path, monkeypatch):
    """zlib memLevel 9 (as GNU gzip: 32k symbols per block, ~53 KB of
    FASTA) makes block bodies longer than the staged decode's 30 KB LDS
    window: they are decoded in windows.  Sketches equal the oracle's and
    the host path's, no batch handed back."""
    rng = np.random.default_rng(9)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    paths = []
    for i in range(12):
        seq = acgt[rng.integers(0, 4, 1500000)].tobytes()
        text = b">big%d\n" % i + b"\n".join(seq[j:j + 60] for j in range(0, len(seq), 60)) + b"\n"
        c = zlib.compressobj(9 if i % 2 else 6, zlib.DEFLATED, 31, 9)
        p = tmp_path / ("big%02d.fna.gz" % i)
        p.write_bytes(c.compress(text) + c.flush())
        paths.append(str(p))
    exp_sk, exp_len = oracle.sketch_files(paths, threads=8)
    dsk, dl, fb = sketch_files(paths, monkeypatch, "device")
    assert fb["inflate_host"] == 0
    assert (dl == exp_len).all()
    for g in range(len(paths)):
        assert (dsk[g][:dl[g]] == exp_sk[g][:dl[g]]).all(), paths[g]
    # the global-memory decode (A/B knob) agrees
    monkeypatch.setenv("GALAHGPU_DECODE_GLOBAL", "1")
    gsk, gl, fb = sketch_files(paths, monkeypatch, "device")
    assert fb["inflate_host"] == 0 and (gl == dl).all() and (gsk == dsk).all()


@pytest.mark.gpu
@pytest.mark.parametrize("stage_kb", ["0", "2"])
def test_device_inflate_false_starts_absorbed(tmp_path, monkeypatch, stage_kb):
    """A false block start (GALAHGPU_TEST_FAKE_STARTS: one midway between
    every two starts the search found) is passed by the lane before, which
    decodes again from the start of the block that ran past it and absorbs
    the false lane; with a 2 KB LDS stage (GALAHGPU_TEST_STAGE_KB) every block
    takes many windows, and the block that overran must not count its earlier
    windows' tokens twice (that sent C2 batches back to the host on ISIZE).
    No batch handed back, sketches equal the host path's."""
    rng = np.random.default_rng(21)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    paths = []
    for i in range(8):
        seq = acgt[rng.integers(0, 4, 700000)].tobytes()
        text = b">f%d\n" % i + b"\n".join(seq[j:j + 80] for j in range(0, len(seq), 80)) + b"\n"
        p = tmp_path / ("f%02d.fna.gz" % i)
        p.write_bytes(gzip.compress(text, 6))
        paths.append(str(p))
    hsk, hl, _ = sketch_files(paths, monkeypatch, "host")
    monkeypatch.setenv("GALAHGPU_TEST_FAKE_STARTS", "1")
    monkeypatch.setenv("GALAHGPU_TEST_STAGE_KB", stage_kb)
    monkeypatch.setenv("GALAHGPU_GZ_CHUNK_KB", "16")  # (more chunks: more starts, more false ones)
    dsk, dl, fb = sketch_files(paths, monkeypatch, "device")
    assert fb["inflate_host"] == 0
    assert (dl == hl).all() and all((dsk[g][:dl[g]] == hsk[g][:hl[g]]).all() for g in range(len(paths)))


@pytest.mark.gpu
def test_device_inflate_corrupt_and_empty_fail_as_host(tmp_path, monkeypatch):
    rng = np.random.default_rng(4)
    seq = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, 200000)].tobytes()
    good = gzip.compress(b">c\n" + seq + b"\n")
    bad = bytearray(good)
    bad[len(bad) // 2] ^= 0x55  # inside the deflate data: a CRC or stream error
    cases = {"corrupt.fa.gz": bytes(bad), "empty.fa.gz": gzip.compress(b""), "truncated.fa.gz": good[:len(good) // 2]}
    for name, data in cases.items():
        p = tmp_path / name
        p.write_bytes(data)
        errs = {}
        for mode in ("host", "device"):
            monkeypatch.setenv("GALAHGPU_INFLATE", mode)
            with ga.Context(k=21, sketch_size=1000) as ctx:
                with pytest.raises(ga.GalahGpuError) as e:
                    ctx.sketch_files([str(p)])
                errs[mode] = (e.value.status, str(e.value))
        assert errs["device"] == errs["host"], name


@pytest.mark.gpu
def test_device_inflate_corrupt_streams_fail_as_host(tmp_path, monkeypatch):
    """Bytes flipped at several places of a multi-block stream: whatever the
    lanes decode (garbage that may still add up to ISIZE), the device path
    hands the batch to the host and reports the host's error -- no device
    fault, no other error."""
    rng = np.random.default_rng(5)
    seq = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, 600000)].tobytes()
    good = gzip.compress(b">c\n" + b"\n".join(seq[i:i + 80] for i in range(0, len(seq), 80)) + b"\n", 6)
    for frac in (0.2, 0.35, 0.5, 0.65, 0.8):
        for pat in (0x55, 0x01, 0xFF):
            bad = bytearray(good)
            bad[int(len(bad) * frac)] ^= pat
            p = tmp_path / ("c%d_%d.fa.gz" % (int(frac * 100), pat))
            p.write_bytes(bytes(bad))
            errs = {}
            for mode in ("host", "device"):
                monkeypatch.setenv("GALAHGPU_INFLATE", mode)
                with ga.Context(k=21, sketch_size=1000) as ctx:
                    try:
                        ctx.sketch_files([str(p)])
                        errs[mode] = None
                    except ga.GalahGpuError as e:
                        errs[mode] = (e.status, str(e))
            assert errs["device"] == errs["host"], p.name


@pytest.mark.gpu
@pytest.mark.parametrize("poison", ["0", "0x8101", "0xffff"])
def test_device_inflate_does_not_read_stale_val(golden, monkeypatch, tmp_path, poison):
    """The resolve pass reads the expand's sym array (u16 per text byte) only
    in the gzip members' ranges, where the expand wrote every byte.  Before
    round 5 the resolve read val (u32) entries in the '\n' padding between
    files, which no kernel writes, and stale words there appended bases to a
    genome's last record.  sym filled with zeros, with a pointer into the
    ring (0x8101) and with an invalid value: the same sketches, no batch
    handed back; a plain FASTA file first in the batch (its text is never in
    sym) included."""
    monkeypatch.setenv("GALAHGPU_TEST_POISON_VAL", poison)
    plain = tmp_path / "plain_first.fna"
    with gzip.open(golden["paths"][0], "rb") as f:
        plain.write_bytes(f.read())
    paths = [str(plain)] + list(golden["paths"])
    sk, lens, fb = sketch_files(paths, monkeypatch, "device")
    assert fb["inflate_host"] == 0
    exp_sk = [golden["sketches"][0]] + list(golden["sketches"])
    exp_len = [golden["lens"][0]] + list(golden["lens"])
    assert list(lens) == exp_len
    for g in range(len(lens)):
        assert (sk[g][:lens[g]] == exp_sk[g][:lens[g]]).all(), paths[g]


@pytest.mark.gpu
def test_device_inflate_is_the_default_and_knobs_change_nothing(golden, monkeypatch):
    """A .gz list takes the device path with no knob set (the info line
    counts no host-inflated batch); mapped vs read files, small batches and
    one staging thread (tuning knobs) give the same sketches."""
    monkeypatch.delenv("GALAHGPU_INFLATE", raising=False)
    with ga.Context(k=21, sketch_size=1000) as ctx:
        sk0, l0, _ = ctx.sketch_files([str(p) for p in golden["paths"]])
        assert ctx.fallbacks()["inflate_host"] == 0
        assert "host-inflated batches 0" in ctx.info_line()
    assert (l0 == golden["lens"]).all()
    for knobs in ({"GALAHGPU_GZ_MMAP": "0"}, {"GALAHGPU_GZ_COPY_THREADS": "1"}):
        for k, v in knobs.items():
            monkeypatch.setenv(k, v)
        sk, lens, fb = sketch_files(golden["paths"], monkeypatch, "device")
        for k in knobs:
            monkeypatch.delenv(k)
        assert fb["inflate_host"] == 0
        assert (lens == l0).all() and all((sk[g][:lens[g]] == sk0[g][:l0[g]]).all() for g in range(len(lens)))


@pytest.mark.gpu
def test_lowest_failing_file_reported_when_its_batch_is_dropped(tmp_path, monkeypatch):
    """a corrupt .gz (index 2) and an unreadable path (index 4)
    claimed into one batch: the unreadable file stops the batch before any
    decode, so the corrupt one was never decoded there.  The call must still
    report the corrupt file -- the lowest failing index, as a serial reader
    (and the host path) meets it -- not the unreadable one."""
    rng = np.random.default_rng(51)
    paths = []
    for i in range(6):
        p = tmp_path / ("f%d.fna.gz" % i)
        data = gzip.compress(fasta_text(rng, 200000, b"f%d" % i), 6)
        if i == 2:
            bad = bytearray(data)
            bad[len(bad) // 2] ^= 0x55
            data = bytes(bad)
        if i != 4:
            p.write_bytes(data)
        paths.append(str(p))
    monkeypatch.setenv("GALAHGPU_GZ_COPY_THREADS", "1")
    monkeypatch.setenv("GALAHGPU_GZ_LANES", "1")
    errs = {}
    for mode in ("host", "device"):
        monkeypatch.setenv("GALAHGPU_INFLATE", mode)
        with ga.Context(k=21, sketch_size=1000) as ctx:
            with pytest.raises(ga.GalahGpuError) as e:
                ctx.sketch_files(paths)
            errs[mode] = (e.value.status, str(e.value))
    assert errs["device"] == errs["host"]
    assert "f2.fna.gz" in errs["device"][1] and "f4.fna.gz" not in errs["device"][1], errs
