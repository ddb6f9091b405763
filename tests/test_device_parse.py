"""Device-side FASTA parsing (galah_amd/csrc/parse.hip):
gg_sketch_files with GALAHGPU_PARSE=device gives the same
sketches as the host packer (GALAHGPU_PARSE=host) and as the oracle on the
same files, across line layouts, record boundaries, byte classes, FASTQ,
gzip, many files per batch, and the file errors.  Needs an MI355X."""
import gzip

import numpy as np
import pytest

import galah_amd as ga
import oracle
from test_host import EDGE_RECORDS

pytestmark = pytest.mark.gpu


def sketches(paths, mode, monkeypatch, k=21, s=1000):
    monkeypatch.setenv("GALAHGPU_PARSE", mode)
    with ga.Context(k=k, sketch_size=s) as ctx:
        sk, lens, _ = ctx.sketch_files([str(p) for p in paths])
    return sk, lens


def assert_same(paths, monkeypatch, k=21, s=1000, expect=None):
    dsk, dl = sketches(paths, "device", monkeypatch, k, s)
    hsk, hl = sketches(paths, "host", monkeypatch, k, s)
    assert (dl == hl).all()
    for g in range(len(paths)):
        assert (dsk[g][:dl[g]] == hsk[g][:hl[g]]).all(), paths[g]
        if expect is not None:
            e = expect[g]
            assert dl[g] == len(e) and (dsk[g][:dl[g]] == e).all(), paths[g]


def wrap(seq, width):
    if width <= 0:
        return seq + b"\n"
    return b"".join(seq[i:i + width] + b"\n" for i in range(0, len(seq), width))


def test_golden_files_device_equals_host(golden, monkeypatch):
    assert_same(golden["paths"], monkeypatch,
                expect=[golden["sketches"][g][:golden["lens"][g]] for g in range(len(golden["paths"]))])


def test_layouts_and_byte_classes(tmp_path, monkeypatch):
    rng = np.random.default_rng(41)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    rnd = lambda n: acgt[rng.integers(0, 4, n)].tobytes()
    files, expect = [], []

    def add(name, data, records):
        p = tmp_path / name
        p.write_bytes(data)
        files.append(p)
        expect.append(oracle.sketch_records(records) if records else np.zeros(0, np.uint64))

    seq = rnd(50000)
    for width in (0, 60, 61, 80, 8191, 8192, 8193):  # line lengths around the 8 KiB parse block
        add("w%d.fa" % width, b">g desc\n" + wrap(seq, width), [seq])
    recs = [rnd(int(n)) for n in rng.integers(0, 3000, 9)]
    add("multi.fa", b"".join(b">r%d\n%s" % (i, wrap(r, 70)) for i, r in enumerate(recs)), recs)
    add("crlf.fa", b">x\r\n" + wrap(seq[:3000], 60).replace(b"\n", b"\r\n"), [seq[:3000]])
    add("blank.fa", b">x\n\n\n" + seq[:500] + b"\n\n   \n" + seq[500:2000] + b"\n>y\n\n", [seq[:2000]])
    add("edge.fa", b"".join(b">e%d\n%s\n" % (i, r) for i, r in enumerate(EDGE_RECORDS)), EDGE_RECORDS)
    add("lower.fa", b">x\n" + seq[:4000].lower() + b"\n", [seq[:4000]])
    # '>' not at a line start is a sequence byte that breaks k-mers; ' >' too
    add("gt.fa", b">x\n" + seq[:300] + b">" + seq[300:900] + b"\n >" + seq[900:1500] + b"\n",
        [seq[:300] + b"N" + seq[300:900] + b"N" + seq[900:1500]])
    add("hdr_only.fa", b">only a header", [])
    add("hdr_then_empty.fa", b">a\n>b\n" + seq[:100] + b"\n>c", [seq[:100]])
    add("no_newline.fa", b">x\n" + seq[:5000], [seq[:5000]])
    add("iupac.fa", b">x\n" + b"".join(seq[i:i + 37] + b"RYKMSWN"[i % 7:i % 7 + 1] for i in range(0, 8000, 37)) + b"\n",
        None)
    expect[-1] = None
    fq = b"".join(b"@q%d\n%s\n+\n%s\n" % (i, r, b"I" * len(r)) for i, r in enumerate(recs[:4]))
    add("reads.fq", fq, recs[:4])
    gz = tmp_path / "gz.fa.gz"
    gz.write_bytes(gzip.compress(b">z\n" + wrap(seq[:20000], 80)))
    files.append(gz)
    expect.append(oracle.sketch_records([seq[:20000]]))
    exp = [e for e in expect]
    dsk, dl = sketches(files, "device", monkeypatch)
    hsk, hl = sketches(files, "host", monkeypatch)
    for g, p in enumerate(files):
        assert dl[g] == hl[g] and (dsk[g][:dl[g]] == hsk[g][:hl[g]]).all(), p.name
        if exp[g] is not None:
            assert dl[g] == len(exp[g]) and (dsk[g][:dl[g]] == exp[g]).all(), p.name
    # the IUPAC file against the oracle on the bytes as they are
    g = [p.name for p in files].index("iupac.fa")
    assert (dsk[g][:dl[g]] == oracle.sketch_file(str(files[g]))).all()


def test_many_files_other_k_and_s(tmp_path, monkeypatch):
    """70 files (3 batches of 32) of ragged sizes, k = 16 and 31, s = 10000."""
    rng = np.random.default_rng(43)
    acgt = np.frombuffer(b"ACGTN", np.uint8)
    files = []
    for i in range(70):
        n = int(rng.integers(0, 40000))
        seq = acgt[rng.integers(0, 4010, n) // 1000].tobytes()  # an N in ~400 bases
        p = tmp_path / ("f%02d.fa" % i)
        p.write_bytes(b">f\n" + wrap(seq, int(rng.integers(50, 200))))
        files.append(p)
    for k, s in ((21, 1000), (16, 200), (31, 10000)):
        assert_same(files, monkeypatch, k=k, s=s)


def test_device_parse_errors(tmp_path, monkeypatch):
    monkeypatch.setenv("GALAHGPU_PARSE", "device")
    bad = tmp_path / "bad.fa"
    bad.write_bytes(b"ACGT\n")
    empty = tmp_path / "empty.fa"
    empty.write_bytes(b"")
    good = tmp_path / "good.fa"
    good.write_bytes(b">g\nACGTACGTACGTACGTACGTACGTACGT\n")
    with ga.Context(k=21, sketch_size=100) as ctx:
        for p, status in ((bad, 3), (empty, 3), (tmp_path / "missing.fa", 2)):
            with pytest.raises(ga.GalahGpuError) as e:
                ctx.sketch_files([str(good), str(p)])
            assert e.value.status == status


def test_precluster_files_device_parse(golden, monkeypatch):
    monkeypatch.setenv("GALAHGPU_PARSE", "device")
    with ga.Context(k=21, sketch_size=1000) as ctx:
        pairs, ani = ctx.precluster_files(golden["paths"], ga.parse_percentage(90))
    assert len(pairs) == 161


def test_device_parse_three_members(tmp_path, monkeypatch):
    """The device parser inside a 3-member context (batches dealt to the
    members, each parsing on its own stream): same sketches as one member."""
    rng = np.random.default_rng(47)
    acgt = np.frombuffer(b"ACGTN", np.uint8)
    files = []
    for i in range(40):
        seq = acgt[rng.integers(0, 4010, int(rng.integers(1000, 60000))) // 1000].tobytes()
        p = tmp_path / ("m%02d.fa" % i)
        p.write_bytes(b">m\n" + wrap(seq, 80))
        files.append(str(p))
    monkeypatch.setenv("GALAHGPU_PARSE", "device")
    with ga.Context(k=21, sketch_size=500) as ctx:
        sk1, l1, _ = ctx.sketch_files(files)
    with ga.Context(k=21, sketch_size=500, devices=[0, 0, 0]) as ctx:
        sk3, l3, _ = ctx.sketch_files(files)
    assert (l1 == l3).all() and (sk1 == sk3).all()
    monkeypatch.setenv("GALAHGPU_PARSE", "host")
    with ga.Context(k=21, sketch_size=500) as ctx:
        skh, lh, _ = ctx.sketch_files(files)
    assert (lh == l1).all() and (skh == sk1).all()
