"""The Rust side of the boundary (rust/aggregator/src/gpu/ffi.rs, the `extern "C"` block a Janus
build links) checked mechanically against include/prio3gpu.h, the way tests/test_abi.py checks the
ctypes declarations: every header function is declared once, with the same argument count and the
same pointer depth / constness / integer width per argument and for the result, and every
#[repr(C)] struct has the header's fields in the header's order with the same types.  (No cargo in
this image: this is what keeps the uncompiled binding honest.)"""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "prio3gpu.h")
FFI = os.path.join(ROOT, "rust", "aggregator", "src", "gpu", "ffi.rs")

C_BASE = {"uint8_t": "u8", "uint16_t": "u16", "uint32_t": "u32", "uint64_t": "u64", "int64_t": "i64",
          "size_t": "usize", "int": "c_int", "double": "f64", "void": "c_void", "char": "c_char"}


def _strip_c_comments(s):
    s = re.sub(r"/\*.*?\*/", " ", s, flags=re.S)
    return re.sub(r"//[^\n]*", " ", s)


def c_type(decl, is_param=True):
    """'const uint8_t* nonces' -> ('ptr_const', 'u8'); arrays are pointers (parameters)."""
    decl = " ".join(decl.replace("*", " * ").split())
    arr = re.search(r"\[(\d*)\]\s*$", decl)
    if arr:
        decl = decl[:arr.start()].strip()
    toks = decl.split()
    if is_param:  # every header parameter is named: drop the name
        assert re.match(r"^[A-Za-z_]\w*$", toks[-1]) and len(toks) > 1, decl
        toks = toks[:-1]
    const_base = toks[0] == "const"
    if const_base:
        toks = toks[1:]
    base = C_BASE.get(toks[0], toks[0])
    depth = toks.count("*") + (1 if arr else 0)
    t = base
    for d in range(depth):
        inner_const = const_base and d == 0
        t = ("ptr_const" if inner_const else "ptr_mut", t)
    return t


def rust_type(t):
    t = t.strip()
    m = re.match(r"^\*(const|mut)\s+(.*)$", t)
    if m:
        return ("ptr_const" if m.group(1) == "const" else "ptr_mut", rust_type(m.group(2)))
    m = re.match(r"^\[\s*(\w+)\s*;\s*(\d+)\s*\]$", t)
    if m:
        return ("array", rust_type(m.group(1)), int(m.group(2)))
    return t


def header_functions():
    src = _strip_c_comments(open(HEADER).read())
    out = {}
    for m in re.finditer(r"(?m)^\s*((?:const\s+)?[\w]+\s*\**)\s*(prio3gpu_\w+)\s*\(([^;{]*?)\)\s*;",
                         src):
        ret, name, args = m.group(1), m.group(2), " ".join(m.group(3).split())
        params = [] if args in ("", "void") else [a.strip() for a in args.split(",")]
        out[name] = (c_type(ret, is_param=False), [c_type(p) for p in params])
    return out


def rust_functions():
    src = open(FFI).read()
    block = src[src.index('extern "C" {'):]
    block = re.sub(r"//[^\n]*", " ", block)
    out = {}
    for m in re.finditer(r"pub fn (prio3gpu_\w+)\s*\((.*?)\)\s*(?:->\s*([^;]+))?;", block, re.S):
        name, args, ret = m.group(1), " ".join(m.group(2).split()), m.group(3)
        params = [a for a in (x.strip() for x in args.split(",")) if a]
        assert name not in out, f"{name} declared twice in ffi.rs"
        out[name] = (rust_type(ret) if ret else "()", [rust_type(p.split(":", 1)[1]) for p in params])
    return out


def test_every_header_function_is_bound_with_matching_signature():
    h, r = header_functions(), rust_functions()
    assert len(h) >= 55, sorted(h)
    missing = sorted(set(h) - set(r))
    extra = sorted(set(r) - set(h))
    assert not missing, f"ffi.rs lacks {missing}"
    assert not extra, f"ffi.rs declares functions the header does not: {extra}"
    for name, (ret, params) in h.items():
        rret, rparams = r[name]
        assert rret == ret, f"{name}: result {rret} != header {ret}"
        assert len(rparams) == len(params), f"{name}: {len(rparams)} args != header {len(params)}"
        for i, (a, b) in enumerate(zip(rparams, params)):
            assert a == b, f"{name} arg {i}: ffi.rs {a} != header {b}"


def test_ctypes_exports_are_all_bound():
    from janus_amd._lib import EXPORTED
    r = rust_functions()
    assert sorted(set(EXPORTED) - set(r)) == []


def _c_structs():
    src = _strip_c_comments(open(HEADER).read())
    out = {}
    for m in re.finditer(r"typedef struct (prio3gpu_\w+)\s*\{(.*?)\}\s*\1\s*;", src, re.S):
        fields = []
        for decl in m.group(2).split(";"):
            decl = " ".join(decl.split())
            if not decl:
                continue
            first, *rest = [x.strip() for x in decl.split(",")]
            toks = first.replace("*", " * ").split()
            const = toks[0] == "const"
            if const:
                toks = toks[1:]
            base = C_BASE.get(toks[0], toks[0])
            stars = toks.count("*")
            names = [toks[-1]] + rest
            for nm in names:
                arr = re.match(r"^(\w+)\[(\d+)\]$", nm)
                t = base
                for d in range(stars):
                    t = ("ptr_const" if const and d == 0 else "ptr_mut", t)
                if arr:
                    fields.append((arr.group(1), ("array", t, int(arr.group(2)))))
                else:
                    fields.append((nm, t))
        out[m.group(1)] = fields
    return out


def _rust_structs():
    src = open(FFI).read()
    out = {}
    for m in re.finditer(r"#\[repr\(C\)\][^\n]*\n(?:#\[[^\n]*\]\n)*pub struct (prio3gpu_\w+)\s*\{(.*?)\n\}",
                         src, re.S):
        body = re.sub(r"//[^\n]*", " ", m.group(2))
        fields = []
        for f in body.split(",\n"):
            f = " ".join(f.split()).rstrip(",")
            if not f or f.startswith("_p:"):
                continue
            nm, t = f.replace("pub ", "", 1).split(":", 1)
            fields.append((nm.strip(), rust_type(t)))
        out[m.group(1)] = fields
    return out


@pytest.mark.parametrize("name", ["prio3gpu_sizes", "prio3gpu_batch_aggregation",
                                  "prio3gpu_prepare_init_view", "prio3gpu_prepare_resp_view",
                                  "prio3gpu_hpke_keypair"])
def test_repr_c_structs_match_header(name):
    c, r = _c_structs(), _rust_structs()
    assert name in c and name in r
    assert r[name] == c[name]


def test_parser_sees_what_it_should():
    h = header_functions()
    assert h["prio3gpu_ctx_create"][1][4] == ("ptr_const", "u8")          # verify_key[16]
    assert h["prio3gpu_ctx_create"][1][6] == ("ptr_mut", ("ptr_mut", "prio3gpu_ctx"))
    assert h["prio3gpu_ctx_stream"][0] == ("ptr_mut", "c_void")
    assert h["prio3gpu_last_error"] == (("ptr_const", "c_char"), [])
    assert h["prio3gpu_comm_unique_id"][1] == [("ptr_mut", "u8")]          # out_id[128]
    assert h["prio3gpu_unshard"][1][5] == ("ptr_mut", "f64")


MOD = os.path.join(ROOT, "rust", "aggregator", "src", "gpu", "mod.rs")
BUILD_RS = os.path.join(ROOT, "rust", "aggregator", "build.rs")


def _ffi_calls(src):
    """(name, argument count) of every `ffi::prio3gpu_*(...)` call, arguments split at the
    call's top-level commas."""
    src = re.sub(r"//[^\n]*", " ", src)
    out = []
    for m in re.finditer(r"ffi::(prio3gpu_\w+)\s*\(", src):
        i, depth, args, cur = m.end(), 1, [], ""
        while depth:
            ch = src[i]
            if ch in "([{":
                depth += 1
            elif ch in ")]}":
                depth -= 1
            if depth == 1 and ch == ",":
                args.append(cur)
                cur = ""
            elif depth:
                cur += ch
            i += 1
        if cur.strip():
            args.append(cur)
        out.append((m.group(1), len([a for a in args if a.strip()])))
    return out


def test_mod_rs_calls_header_functions_with_their_arity():
    h = header_functions()
    calls = _ffi_calls(open(MOD).read())
    assert len(calls) >= 15
    for name, n in calls:
        assert name in h, f"mod.rs calls {name}, which the header does not declare"
        assert n == len(h[name][1]), f"mod.rs calls {name} with {n} args, header has {len(h[name][1])}"


def test_build_rs_keeps_rustc_semver_and_checks_the_hash():
    """The reference's aggregator/build.rs:3-6 (used by env!("RUSTC_SEMVER"),
    aggregator/src/metrics.rs:227) stays; the engine build refuses an empty/failed hash."""
    src = open(BUILD_RS).read()
    assert "cargo:rustc-env=RUSTC_SEMVER=" in src and "rustc_version::version" in src
    assert "cargo:rerun-if-env-changed=RUSTC" in src
    assert "status.success()" in src.split("python3", 1)[1].split("hipcc", 1)[0]
    assert "len() == 64" in src and "is_ascii_hexdigit" in src


def test_every_prio3_vdaf_ops_variant_and_engine_kind_has_an_arm():
    """GpuVdafOps mirrors the reference's Prio3 VdafOps variants (aggregator.rs:1040-1058) and
    every `enum prio3gpu_kind` value is reached by some arm."""
    src = re.sub(r"//[^\n]*", " ", open(MOD).read())
    enum = re.search(r"pub enum GpuVdafOps \{(.*?)\n\}", src, re.S).group(1)
    variants = set(re.findall(r"(Prio3\w+)\(", enum))
    ref = {"Prio3Count", "Prio3CountVec", "Prio3Sum", "Prio3SumVec", "Prio3Histogram",
           "Prio3FixedPoint16BitBoundedL2VecSum", "Prio3FixedPoint32BitBoundedL2VecSum",
           "Prio3FixedPoint64BitBoundedL2VecSum"}
    assert variants == ref
    kind_fn = re.search(r"pub fn kind\(&self\).*?\n    \}", src, re.S).group(0)
    for v in ref:
        assert f"GpuVdafOps::{v}(" in kind_fn, f"kind() has no arm for {v}"
    hdr = _strip_c_comments(open(HEADER).read())
    kinds = re.findall(r"(PRIO3GPU_(?:COUNT|SUM|SUMVEC|HISTOGRAM|FPVEC))\s*=", hdr)
    assert len(kinds) == 5
    for k in kinds:
        assert f"ffi::{k}" in kind_fn, f"no GpuVdafOps arm maps to {k}"
        assert f"ffi::{k}" in re.search(r"pub fn engine_params.*?\n\}", src, re.S).group(0)
    # leader and helper entry points on every arm (through task())
    for f in ("helper_aggregate_init", "leader_aggregate_init", "leader_process_response"):
        assert re.search(rf"impl GpuVdafOps \{{.*pub fn {f}\(", src, re.S), f
