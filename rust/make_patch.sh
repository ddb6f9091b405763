#!/bin/bash
# Writes rust/galah_gpu.patch: the change a galah maintainer applies to the
# reference tree (git apply / patch -p1 at galah's root) to build galah's
# finch precluster path on MI355X GPUs with `cargo build --features gpu`:
#   Cargo.toml     galah-gpu-sys as an optional dependency, feature "gpu"
#   src/lib.rs     the finch_gpu module (feature "gpu" only)
#   src/finch.rs   distances() (src/finch.rs:26-31) returns finch_gpu::distances
#                  when the feature is on; its CPU body is untouched
#   src/finch_gpu.rs  rust/galah/src/finch_gpu.rs (new file)
# Without the feature galah builds and behaves exactly as before.
# usage: rust/make_patch.sh [reference root, default /root/reference]
set -euo pipefail
here=$(cd "$(dirname "$0")" && pwd)
ref=${1:-/root/reference}
t=$(mktemp -d)
trap 'rm -rf "$t"' EXIT
mkdir -p "$t/a/src" "$t/b/src"
for f in Cargo.toml src/lib.rs src/finch.rs; do cp "$ref/$f" "$t/a/$f"; cp "$ref/$f" "$t/b/$f"; done
cp "$here/galah/src/finch_gpu.rs" "$t/b/src/finch_gpu.rs"
python3 - "$t/b" <<'PY'
import sys
b = sys.argv[1]
def edit(path, old, new):
    s = open(path).read()
    assert s.count(old) == 1, (path, old)
    open(path, "w").write(s.replace(old, new))
edit(b + "/Cargo.toml", 'concurrent-queue = "2"\n',
     'concurrent-queue = "2"\n'
     '# MI355X finch precluster path (libgalahgpu.so); path to a checkout of galah_amd\n'
     'galah-gpu-sys = { path = "../galah_amd/rust/galah-gpu-sys", optional = true }\n')
s = open(b + "/Cargo.toml").read()
open(b + "/Cargo.toml", "w").write(s + '\n[features]\n# `cargo build --features gpu`: finch::distances on the GPUs\ngpu = ["galah-gpu-sys"]\n')
edit(b + "/src/lib.rs", "pub mod finch;\n", 'pub mod finch;\n#[cfg(feature = "gpu")]\npub mod finch_gpu;\n')
edit(b + "/src/finch.rs", "pub fn distances(\n", '#[cfg_attr(feature = "gpu", allow(unreachable_code, unused_variables))]\npub fn distances(\n')
edit(b + "/src/finch.rs", ") -> SortedPairGenomeDistanceCache {\n    // Hash all the files\n",
     ") -> SortedPairGenomeDistanceCache {\n"
     "    #[cfg(feature = \"gpu\")]\n"
     "    return crate::finch_gpu::distances(genome_fasta_paths, min_ani, num_kmers, kmer_length);\n"
     "    // Hash all the files\n")
PY
(cd "$t" && diff -ruN a b || true) | sed -E "s/^((---|\+\+\+) [^\t]*)\t.*/\1/" > "$here/galah_gpu.patch"
echo "wrote $here/galah_gpu.patch"
