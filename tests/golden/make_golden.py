"""Generate the committed golden fixtures for the finch precluster path.

Run from the repo root in the build container (it reads /root/reference,
which does not exist on the GPU box):

    python tests/golden/make_golden.py

Outputs (all data, no reference source):
  tests/golden/data/<set>/<genome>.fna.gz   the 27 FASTA genomes of the
        reference's tests/data (inputs of src/finch.rs:85-107,
        src/clusterer.rs:482-612, tests/test_cmdline.rs), gzip-compressed
        (finch/needletail read gzip transparently; so does gg_pack_files)
  tests/golden/sketches_k21_s1000.npz       oracle sketches (names, hashes, lens)
  tests/golden/pairs_k21_s1000.tsv          all 351 pairs: i j common total ani_f32
  tests/golden/murmur3_kat.json             murmur3 x64_128 vectors

The oracle is pinned before use by the reference's own known answers (see
tests/test_oracle_golden.py): set1/1mbp vs set1/500kb -> 0.9808188
(src/finch.rs:96), and the threshold facts of SURVEY.md section 4.
"""
import glob
import gzip
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402

REF_DATA = "/root/reference/tests/data"
GOLD = os.path.join(ROOT, "tests", "golden")


def main():
    paths = sorted(glob.glob(os.path.join(REF_DATA, "*", "*.fna")))
    assert len(paths) == 27, paths
    names = [os.path.relpath(p, REF_DATA) for p in paths]
    for p, n in zip(paths, names):
        dst = os.path.join(GOLD, "data", n + ".gz")
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        with open(p, "rb") as f:
            raw = f.read()
        with gzip.GzipFile(dst, "wb", compresslevel=9, mtime=0) as g:
            g.write(raw)
    sk, lens = oracle.sketch_files(paths, k=21, s=1000, seed=0, threads=8)
    # the gz copies must sketch identically
    gz = [os.path.join(GOLD, "data", n + ".gz") for n in names]
    sk2, lens2 = oracle.sketch_files(gz, k=21, s=1000, seed=0, threads=8)
    assert (sk == sk2).all() and (lens == lens2).all()
    np.savez_compressed(os.path.join(GOLD, "sketches_k21_s1000.npz"), names=np.array(names),
                        sketches=sk, lens=lens)
    allp = oracle.pairs(sk, lens, 0.0)
    assert len(allp) == 27 * 26 // 2
    with open(os.path.join(GOLD, "pairs_k21_s1000.tsv"), "w") as f:
        f.write("i\tj\tcommon\ttotal\tani_f32\n")
        for r in allp:
            f.write("%d\t%d\t%d\t%d\t%s\n" % (r["i"], r["j"], r["common"], r["total"],
                                               np.format_float_positional(np.float32(r["ani"]), unique=True)))
    kat = {
        "published": [  # MurmurHash3_x64_128 reference outputs, seed 0
            {"input": "", "h1": 0, "h2": 0},
            {"input": "hello", "h1": 0xcbd8a7b341bd9b02, "h2": 0x5b1e906a48ae1d19},
            {"input": "The quick brown fox jumps over the lazy dog",
             "h1": 0xe34bbc7bbc071b6c, "h2": 0x7a433ca9c49a9347},
        ],
        "kmers21": [],
    }
    for s in ["ACGTACGTACGTACGTACGTA", "AAAAAAAAAAAAAAAAAAAAA", "GTCACCGTGAACTTAGACGGG",
              "TTTTTTTTTTTTTTTTTTTTT", "CGCGCGCGCGCGCGCGCGCGC"]:
        kat["kmers21"].append({"kmer": s, "h1": oracle.murmur3_h1(s.encode())})
    for e in kat["published"]:
        h1, h2 = oracle.murmur3_x64_128(e["input"].encode())
        assert (h1, h2) == (e["h1"], e["h2"]), e
    with open(os.path.join(GOLD, "murmur3_kat.json"), "w") as f:
        json.dump(kat, f, indent=1)
    print("wrote fixtures for %d genomes" % len(names))


if __name__ == "__main__":
    main()
