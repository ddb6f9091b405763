"""K1's machine code, classified by VALU issue cost (round-2 roofline).

The per-opcode issue costs come from scripts/ubench_valu2.hip and
scripts/ubench_dual.hip (profiles/r02_ubench_*.txt, cycles per wave64
instruction at the effective clock, 8 waves per SIMD, independent chains):

  dual   ~2.3  co-issued in pairs (SQ_ACTIVE_INST_VALU2 counts them): 32-bit
               add/sub/xor/and/or/lshrrev/mov/add_f32 whose sources are
               VGPRs or inline constants
  full   ~4.2  everything else 32-bit: multiplies, alignbit, add3, bfe, sdwa,
               lshlrev_b32, cndmask, compares, any SGPR source
  wide   ~5.0  64-bit results: v_mad_u64_u32, v_lshl_add_u64, 64-bit shifts

Usage: python scripts/k1_isa.py [lib.so]   (prints the class histogram)
"""
import hashlib
import os
import re
import shutil
import subprocess
import sys
import tempfile

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
K1_SYMBOL = "sketch_candidates_kernelILi21ELb1E"


def kernel_listing(lib_path, symbol=K1_SYMBOL, with_addr=False):
    """[(mnemonic, operands)] of the kernel whose mangled name contains symbol
    ([(address, mnemonic, operands, branch target or None)] with with_addr)."""
    tmp = tempfile.mkdtemp(prefix="k1isa")
    try:
        lib = os.path.join(tmp, "lib.so")
        shutil.copy(lib_path, lib)
        subprocess.run([OBJDUMP, "--offloading", lib], cwd=tmp, capture_output=True, timeout=120)
        out = []
        for f in sorted(os.listdir(tmp)):
            if "gfx950" not in f:
                continue
            txt = subprocess.run([OBJDUMP, "-d", os.path.join(tmp, f)], capture_output=True, text=True,
                                 timeout=120).stdout
            on = False
            for line in txt.splitlines():
                if re.match(r"^[0-9a-f]+ <.*>:$", line):
                    on = symbol in line
                    continue
                if on and line.startswith("\t"):
                    code, _, comment = line.partition("//")
                    ins = code.strip()
                    if not ins:
                        continue
                    parts = ins.split(None, 1)
                    if with_addr:
                        m = re.match(r"\s*([0-9A-Fa-f]+):", comment)
                        t = re.search(r"<[^>]*\+0x([0-9a-f]+)>", comment)
                        out.append((int(m.group(1), 16) if m else None, parts[0], parts[1] if len(parts) > 1 else "",
                                    int(t.group(1), 16) if t else None))
                    else:
                        out.append((parts[0], parts[1] if len(parts) > 1 else ""))
            if out:
                break
        return out
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def hot_path(listing_addr):
    """The instructions one segment of the hashing loop executes when no
    candidate branch is taken: from the first k-mer's table read to the last
    k-mer's, skipping every forward s_cbranch_execz body inside that span (the
    candidate test and queue push run for ~12% of 4-k-mer groups at C3, so
    the static listing over-weights them).  [(mnemonic, operands)]"""
    if not listing_addr:
        return []
    base = listing_addr[0][0]
    reads = [i for i, x in enumerate(listing_addr) if x[1] == "ds_read_b128"]
    if len(reads) < 2:
        return [(x[1], x[2]) for x in listing_addr]
    lo, hi = reads[0], reads[-1]
    # the last k-mer's body: up to the next guarded branch after the last read
    end = hi
    while end < len(listing_addr) and listing_addr[end][1] != "s_cbranch_execz":
        end += 1
    out, i = [], lo
    while i < end:
        addr, mn, ops, tgt = listing_addr[i]
        if mn == "s_cbranch_execz" and tgt is not None and tgt + base > addr:
            j = i + 1
            while j < len(listing_addr) and listing_addr[j][0] < tgt + base:
                j += 1
            i = j
            continue
        out.append((mn, ops))
        i += 1
    return out


def fingerprint(listing):
    return hashlib.sha1("\n".join("%s %s" % x for x in listing).encode()).hexdigest()


DUAL_OPS = re.compile(r"^v_(add_u32|sub_u32|subrev_u32|xor_b32|and_b32|or_b32|lshrrev_b32|mov_b32|add_f32|"
                      r"sub_f32|mul_f32|max_f32|min_f32)(_e32)?$")
WIDE_OPS = re.compile(r"^v_(mad_u64_u32|mad_i64_i32|lshl_add_u64|lshlrev_b64|lshrrev_b64|ashrrev_i64|"
                      r"pk_\w+|cmp\w*_u64|cmp\w*_i64|cmpx\w*_u64)(_e32|_e64)?$")


def classify(mn, ops):
    """'dual' | 'full' | 'wide' for a VALU instruction, None otherwise."""
    if not mn.startswith("v_"):
        return None
    if WIDE_OPS.match(mn):
        return "wide"
    m = DUAL_OPS.match(mn)
    if m and "sdwa" not in mn and "_e64" not in mn:
        srcs = [x.strip() for x in ops.split(",")[1:]]
        if not any(re.match(r"^(s\d|s\[|vcc|exec|m0)", x) for x in srcs):
            return "dual"
    return "full"


def histogram(listing):
    h = {"dual": 0, "full": 0, "wide": 0, "other": 0}
    for mn, ops in listing:
        c = classify(mn, ops)
        h[c or "other"] += 1
    return h


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "galah_amd", "lib",
                                                             "libgalahgpu.so")
    L = kernel_listing(lib)
    print(len(L), "instructions; fingerprint", fingerprint(L))
    print("static", histogram(L))
    H = hot_path(kernel_listing(lib, with_addr=True))
    print("hot path (%d instructions)" % len(H), histogram(H))
    from collections import Counter
    c = Counter((mn, classify(mn, ops)) for mn, ops in L if mn.startswith("v_"))
    for (mn, cl), k in c.most_common(40):
        print("%6d  %-28s %s" % (k, mn, cl))
