"""The reference-side binding (rust/) against the C ABI it declares (CPU only).

rust/galah-gpu-sys/src/lib.rs is the `extern "C"` crate galah links
(INTEGRATION.md), and rust/galah_gpu.patch the change to galah's
src/finch.rs:26-31, src/lib.rs and Cargo.toml that makes finch::distances
call rust/galah/src/finch_gpu.rs.  Rust is not installed here, so nothing
compiles the crate; instead this test parses both sides and checks what the
compiler's linker and ABI would rely on:

  - the same set of functions, each with the same argument count and the
    same C type at every position (const-ness of pointees included) and the
    same return type;
  - every #[repr(C)] struct with the header's fields in the header's order,
    and the same size and field offsets as the compiled header (gcc);
  - every enum constant and #define the header has, with equal values;
  - the callback typedef gg_pair_sink;
  - the galah-side body calls only declared functions, with their arity;
  - the patch is what rust/make_patch.sh writes and applies to the
    reference tree (when /root/reference is present).
"""
import ctypes
import os
import re
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "galahgpu.h")
RS = os.path.join(ROOT, "rust", "galah-gpu-sys", "src", "lib.rs")
BODY = os.path.join(ROOT, "rust", "galah", "src", "finch_gpu.rs")
PATCH = os.path.join(ROOT, "rust", "galah_gpu.patch")
REFERENCE = "/root/reference"

C_BASE = {"int": "c_int", "uint32_t": "u32", "uint64_t": "u64", "uint8_t": "u8", "float": "f32", "double": "f64",
          "size_t": "usize", "char": "c_char", "void": "c_void", "gg_status": "GgStatus"}


def _strip_c_comments(s):
    s = re.sub(r"/\*.*?\*/", " ", s, flags=re.S)
    return re.sub(r"//[^\n]*", " ", s)


def _c_type(decl, named=True):
    """A C declaration ('const uint8_t* const* seqs') -> its Rust spelling."""
    toks = re.findall(r"[A-Za-z_]\w*|\*", decl)
    if named:
        toks = toks[:-1]  # the parameter / field name
    base_const, base, levels = False, None, []
    for t in toks:
        if t == "const":
            if base is None:
                base_const = True
            elif levels:
                levels[-1] = True  # the pointer itself is const: irrelevant to the ABI, kept for the pointee below
            else:
                base_const = True
        elif t == "*":
            levels.append(False)
        else:
            assert base is None, decl
            base = t
    rust = C_BASE.get(base, base)
    pointee_const = base_const
    for self_const in levels:
        rust = ("*const " if pointee_const else "*mut ") + rust
        pointee_const = self_const
    return rust


def _split_args(s):
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "(<":
            depth += 1
        elif ch in ")>":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return [a.strip() for a in out]


def parse_header():
    src = _strip_c_comments(open(HEADER).read())
    funcs = {}
    src_nopp = re.sub(r"^\s*#[^\n]*", " ", src, flags=re.M).replace('extern "C" {', " ")
    body = re.sub(r"typedef[^;]*;", " ", re.sub(r"typedef\s+(struct|enum)\s+\w*\s*\{.*?\}\s*\w+\s*;", " ", src_nopp,
                                                flags=re.S))
    for m in re.finditer(r"([A-Za-z_][\w\s\*]*?)\b(gg_\w+)\s*\(([^()]*)\)\s*;", body, flags=re.S):
        ret, name, args = m.group(1).strip(), m.group(2), m.group(3).strip()
        ret_rs = None if ret == "void" else _c_type(ret, named=False)
        arg_rs = [] if args in ("", "void") else [_c_type(a) for a in _split_args(args)]
        funcs[name] = (arg_rs, ret_rs)
    structs = {}
    for m in re.finditer(r"typedef\s+struct\s+(\w+)\s*\{(.*?)\}\s*(\w+)\s*;", src, flags=re.S):
        fields = []
        for f in m.group(2).split(";"):
            f = " ".join(f.split())
            if f:
                fields.append((re.findall(r"\w+", f)[-1], _c_type(f)))
        structs[m.group(3)] = fields
    consts = {}
    for m in re.finditer(r"enum\s*\w*\s*\{(.*?)\}", src, flags=re.S):
        for name, val in re.findall(r"(GG_\w+)\s*=\s*(\d+)", m.group(1)):
            consts[name] = int(val)
    for name, val in re.findall(r"#define\s+(GG_\w+)\s+(\d+)u?\b", src):
        consts[name] = int(val)
    sink = re.search(r"typedef\s+int\s*\(\s*\*\s*gg_pair_sink\s*\)\s*\(([^)]*)\)\s*;", src)
    return funcs, structs, consts, [_c_type(a) for a in _split_args(sink.group(1))]


def parse_rust():
    src = re.sub(r"//[^\n]*", " ", open(RS).read())
    ext = re.search(r'extern "C" \{(.*)\n\}', src, flags=re.S).group(1)
    funcs = {}
    for m in re.finditer(r"pub fn (\w+)\((.*?)\)\s*(?:->\s*([^;]+?))?\s*;", ext, flags=re.S):
        args = [" ".join(a.split(":", 1)[1].split()) for a in _split_args(m.group(2))]
        funcs[m.group(1)] = (args, " ".join(m.group(3).split()) if m.group(3) else None)
    structs = {}
    for m in re.finditer(r"#\[repr\(C\)\]\s*(?:#\[derive\([^)]*\)\]\s*)?pub struct (\w+)\s*\{(.*?)\}", src, flags=re.S):
        fields = [(n, " ".join(t.split())) for n, t in re.findall(r"pub (\w+):\s*([^,]+),", m.group(2))]
        if fields:  # (no public field: an opaque handle, checked separately)
            structs[m.group(1)] = fields
    consts = {n: int(v) for n, v in re.findall(r"pub const (GG_\w+):\s*\w+\s*=\s*(\d+);", src)}
    sink = re.search(r"pub type gg_pair_sink = Option<unsafe extern \"C\" fn\((.*?)\)\s*->\s*(\w+)>;", src, flags=re.S)
    sink_args = [" ".join(a.split(":", 1)[1].split()) for a in _split_args(sink.group(1))]
    return funcs, structs, consts, (sink_args, sink.group(2))


@pytest.fixture(scope="module")
def sides():
    return parse_header(), parse_rust()


def test_same_functions_and_signatures(sides):
    (hf, _, _, _), (rf, _, _, _) = sides
    assert len(hf) >= 40
    assert sorted(hf) == sorted(rf), (set(hf) ^ set(rf))
    for name, (args, ret) in hf.items():
        rargs, rret = rf[name]
        assert len(rargs) == len(args), name
        for k, (a, b) in enumerate(zip(args, rargs)):
            assert a == b, "%s argument %d: header %s, rust %s" % (name, k, a, b)
        assert ret == rret, "%s returns %s in the header, %s in rust" % (name, ret, rret)


def test_python_mirror_declares_the_same_functions(sides):
    (hf, _, _, _), _ = sides
    import galah_amd as ga
    assert sorted(ga.EXPORTED_SYMBOLS) == sorted(hf)


def test_struct_fields_in_order(sides):
    (_, hs, _, _), (_, rs, _, _) = sides
    assert sorted(hs) == sorted(rs)
    for name, fields in hs.items():
        assert rs[name] == fields, name


def test_opaque_context():
    assert re.search(r"typedef struct gg_ctx gg_ctx;", open(HEADER).read())
    assert re.search(r"#\[repr\(C\)\]\s*pub struct gg_ctx \{\s*_private: \[u8; 0\],\s*\}", open(RS).read())


def test_constants_equal(sides):
    (_, _, hc, _), (_, _, rc, _) = sides
    for name, v in hc.items():
        assert rc.get(name) == v, name
    for name in rc:
        assert name in hc, name
    assert hc["GG_FALLBACK_COUNT"] == 6 and hc["GG_OK"] == 0


def test_pair_sink_typedef(sides):
    (_, _, _, hsink), (_, _, _, (rargs, rret)) = sides
    assert hsink == rargs and rret == "c_int"


_CT = {"u32": ctypes.c_uint32, "u64": ctypes.c_uint64, "f64": ctypes.c_double, "c_int": ctypes.c_int}


def _ctype(t):
    return ctypes.c_void_p if t.startswith("*") else _CT[t]


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc")
def test_struct_layout_matches_compiled_header(sides):
    """sizeof / offsetof of every struct as gcc lays the header out, against
    the #[repr(C)] layout of the Rust field types (C rules, via ctypes)."""
    (_, hs, _, _), (_, rs, _, _) = sides
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "galahgpu.h"', "int main(void) {"]
    for name, fields in hs.items():
        lines.append('printf("%s %%zu\\n", sizeof(%s));' % (name, name))
        for f, _ in fields:
            lines.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (name, f, name, f))
    lines.append("return 0; }")
    d = tempfile.mkdtemp()
    try:
        c = os.path.join(d, "layout.c")
        open(c, "w").write("\n".join(lines))
        exe = os.path.join(d, "layout")
        subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe])
        got = dict(l.split() for l in subprocess.check_output([exe]).decode().splitlines())
    finally:
        shutil.rmtree(d)
    for name, fields in rs.items():
        S = type(name, (ctypes.Structure,), {"_fields_": [(f, _ctype(t)) for f, t in fields]})
        assert ctypes.sizeof(S) == int(got[name]), name
        for f, _ in fields:
            assert getattr(S, f).offset == int(got["%s.%s" % (name, f)]), (name, f)


def test_galah_body_calls_declared_functions(sides):
    _, (rf, _, _, _) = sides
    body = re.sub(r"//[^\n]*", " ", open(BODY).read())
    calls = 0
    for m in re.finditer(r"\b(gg_\w+)\(", body):
        name = m.group(1)
        assert name in rf, name
        depth, i = 1, m.end()
        while depth:
            depth += {"(": 1, ")": -1}.get(body[i], 0)
            i += 1
        inner = body[m.end():i - 1].strip()
        n = len(_split_args(inner)) if inner else 0
        assert n == len(rf[name][0]), "%s called with %d arguments" % (name, n)
        calls += 1
    assert calls >= 10


def _patch_new_file(patch, path):
    """The content a unified diff gives a new file."""
    out, on = [], False
    for line in patch.splitlines():
        if line.startswith("+++ "):
            on = line[4:].strip() == "b/" + path
            continue
        if on and line.startswith("diff "):
            break
        if on and line.startswith("+"):
            out.append(line[1:])
    return "\n".join(out) + "\n"


def test_patch_carries_the_body():
    patch = open(PATCH).read()
    assert _patch_new_file(patch, "src/finch_gpu.rs") == open(BODY).read()
    assert 'gpu = ["galah-gpu-sys"]' in patch and "pub mod finch_gpu;" in patch
    assert "return crate::finch_gpu::distances(genome_fasta_paths, min_ani, num_kmers, kmer_length);" in patch


@pytest.mark.skipif(not os.path.isdir(os.path.join(REFERENCE, "src")), reason="reference tree not present")
def test_patch_is_current_and_applies_to_the_reference():
    d = tempfile.mkdtemp()
    try:
        tree = os.path.join(d, "galah")
        os.makedirs(os.path.join(tree, "src"))
        for f in ("Cargo.toml", "src/lib.rs", "src/finch.rs"):
            shutil.copy(os.path.join(REFERENCE, f), os.path.join(tree, f))
        subprocess.check_call(["patch", "-p1", "-s", "-i", PATCH], cwd=tree)
        assert open(os.path.join(tree, "src", "finch_gpu.rs")).read() == open(BODY).read()
        # regenerating it gives the committed file
        saved = open(PATCH).read()
        try:
            subprocess.check_call(["bash", os.path.join(ROOT, "rust", "make_patch.sh"), REFERENCE],
                                  stdout=subprocess.DEVNULL)
            assert open(PATCH).read() == saved
        finally:
            open(PATCH, "w").write(saved)
    finally:
        shutil.rmtree(d)
