"""INTEGRATION.md's Rust FFI block (section 2) against include/sdl_batcher.h:
every `#[repr(C)]` struct has the header struct's fields in order with the
corresponding Rust types, every header function is declared in the
`extern "C"` block with the same parameter and return types, and nothing is
declared there that the header does not have.  (The ctypes mirror is checked
the same way in test_abi.py; this is the binding a Rust maintainer would copy.)
"""
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "sdl_batcher.h")
DOC = os.path.join(REPO, "INTEGRATION.md")

SCALAR = {"int32_t": "i32", "uint32_t": "u32", "int64_t": "i64", "uint64_t": "u64", "double": "f64",
          "float": "f32", "int": "c_int", "size_t": "usize", "uint8_t": "u8", "char": "c_char", "void": "c_void"}


def camel(c_name):
    return "".join(w.capitalize() for w in c_name.split("_"))


def c_to_rust(ctype):
    """'const int32_t *' -> '*const i32'; 'sdl_batcher **' -> '*mut *mut SdlBatcher'."""
    t = ctype.replace("*", " * ").split()
    const = "const" in t
    t = [w for w in t if w not in ("const", "struct")]
    base, stars = t[0], t.count("*")
    r = SCALAR.get(base) or camel(base)
    if stars == 0:
        return r
    # the innermost pointer carries the const; outer pointers are mutable
    r = ("*const " if const else "*mut ") + r
    for _ in range(stars - 1):
        r = "*mut " + r
    return r


def strip_comments(s):
    s = re.sub(r"/\*.*?\*/", " ", s, flags=re.S)
    return re.sub(r"//[^\n]*", " ", s)


def header_api():
    h = strip_comments(open(HEADER).read())
    structs = {}
    for m in re.finditer(r"typedef struct (\w+) \{(.*?)\}\s*(\w+);", h, re.S):
        fields = []
        for decl in m.group(2).split(";"):
            decl = " ".join(decl.split())
            if not decl:
                continue
            mt = re.match(r"((?:const )?\w+(?: \*+)?\s*\**)\s*(.*)", decl)
            ctype, names = mt.group(1).strip(), mt.group(2)
            for name in [n.strip() for n in names.split(",")]:
                stars = len(name) - len(name.lstrip("*"))
                name = name.lstrip("*")
                arr = re.match(r"(\w+)\[(\d+)\]", name)
                t = c_to_rust(ctype + " *" * stars)
                if arr:
                    fields.append((arr.group(1), f"[{t}; {arr.group(2)}]"))
                else:
                    fields.append((name, t))
        structs[camel(m.group(3))] = fields
    sink = re.search(r"typedef int \(\*(\w+)\)\((.*?)\);", h)
    funcs = {}
    body = re.sub(r"typedef[^;]*;", " ", h)
    for m in re.finditer(r"([\w ]+?\**)\s*\b(sdl_\w+)\(([^)]*)\);", body):
        ret = " ".join(m.group(1).split())
        params = []
        for p in [p.strip() for p in m.group(3).split(",") if p.strip() and p.strip() != "void"]:
            mp = re.match(r"(.*?)(\w+)$", p)
            params.append((mp.group(2), c_to_rust(mp.group(1)) if mp.group(1).strip() != "sdl_frame_sink"
                           else camel("sdl_frame_sink")))
        funcs[m.group(2)] = (params, None if ret == "void" else c_to_rust(ret))
    return structs, funcs, sink


def rust_block():
    doc = open(DOC).read()
    sec = doc[doc.index("## 2. FFI declarations"):doc.index("## 3.")]
    return sec[sec.index("```rust") + 7:sec.rindex("```")]


def rust_api():
    r = rust_block()
    structs = {}
    for m in re.finditer(r"#\[repr\(C\)\] pub struct (\w+) \{(.*?)\}", r, re.S):
        fields = []
        for f in re.finditer(r"pub (\w+): (\[[^\]]+\]|[^,]+?)\s*(?:,|$)", m.group(2).strip()):
            fields.append((f.group(1), " ".join(f.group(2).split())))
        structs[m.group(1)] = fields
    ext = r[r.index('extern "C" {'):]
    funcs = {}
    for m in re.finditer(r"pub fn (\w+)\((.*?)\)(?:\s*->\s*([^;]+))?;", ext, re.S):
        params = []
        for p in [p.strip() for p in " ".join(m.group(2).split()).split(",") if p.strip()]:
            name, t = p.split(":", 1)
            params.append((name.strip(), t.strip()))
        funcs[m.group(1)] = (params, m.group(3).strip() if m.group(3) else None)
    return structs, funcs, r


def test_rust_structs_match_header():
    hs, _, _ = header_api()
    rs, _, _ = rust_api()
    assert set(hs) - {"SdlBatcher"} <= set(rs), f"missing #[repr(C)] structs: {set(hs) - set(rs)}"
    for name, fields in hs.items():
        assert rs[name] == fields, (name, rs[name], fields)


def test_rust_extern_block_matches_header():
    _, hf, sink = header_api()
    _, rf, block = rust_api()
    assert set(hf) == set(rf), f"header only: {set(hf) - set(rf)}; Rust only: {set(rf) - set(hf)}"
    for name, (params, ret) in hf.items():
        rparams, rret = rf[name]
        assert [t for _, t in rparams] == [t for _, t in params], (name, rparams, params)
        assert [n for n, _ in rparams] == [n for n, _ in params], (name, rparams, params)
        assert rret == ret, (name, rret, ret)
    # the frame sink callback: int (*)(void *user, const uint8_t *frame, uint64_t bytes)
    assert sink is not None
    assert "pub type SdlFrameSink = Option<unsafe extern \"C\" fn(user: *mut c_void, frame: *const u8, " \
           "bytes: u64) -> c_int>;" in block
    assert "pub enum SdlBatcher {}" in block


def test_every_exported_symbol_is_in_both():
    from streaming_data_loader_amd import native
    _, hf, _ = header_api()
    assert set(native.EXPORTS) == set(hf)
