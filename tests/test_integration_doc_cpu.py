"""INTEGRATION.md is the Rust side of the drop-in boundary: the extern "C"
blocks a fuse-query maintainer adds.  This pins it to the headers so an ABI
change cannot land without the document changing too:

* every ```rust extern "C" block is parsed; each declaration must match the
  header's by name, arity and Rust parameter types (tools/gen_rust_ffi.py maps
  the C declarations), and every function include/*.h declares is bound once;
* every #[repr(C)] struct in the document has the C struct's fields in order,
  and every struct the headers define is there;
* the SURVEY 8b trait surface (function.rs:28-131) and the engine lifecycle
  are bound by name;
* section headings are unique (round 5 had two "2b")."""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_rust_ffi as G  # noqa: E402

DOC = open(os.path.join(ROOT, "INTEGRATION.md")).read()
RUST_BLOCKS = re.findall(r"```rust\n(.*?)```", DOC, flags=re.S)


def norm(s):
    return " ".join(s.replace("(", " ( ").replace(")", " ) ").replace(",", " , ").replace(";", " ; ").split())


def doc_decls():
    out = []
    for blk in RUST_BLOCKS:
        for body in re.findall(r'extern "C" \{(.*?)\n\}', blk, flags=re.S):
            body = re.sub(r"//[^\n]*", "", body)
            out += [norm(d) for d in re.findall(r"pub fn [^;]*;", body, flags=re.S)]
    return out


def header_decls():
    return {name: norm(G.rust_decl(name, ret, params))
            for h in G.HEADERS for name, ret, params in G.c_declarations(h)}


def decl_name(d):
    return re.match(r"pub fn (\w+)", d).group(1)


def arity(d):
    inner = d[d.index("(") + 1:d.rindex(")")].strip()
    return 0 if not inner else inner.count(",") + 1


def test_every_header_function_is_bound_once_with_its_signature():
    docs = doc_decls()
    hdr = header_decls()
    names = [decl_name(d) for d in docs]
    assert len(names) == len(set(names)), sorted(n for n in names if names.count(n) > 1)
    assert sorted(names) == sorted(hdr), (sorted(set(hdr) - set(names)), sorted(set(names) - set(hdr)))
    for d in docs:
        n = decl_name(d)
        assert arity(d) == arity(hdr[n]), (n, arity(d), arity(hdr[n]))
        assert d == hdr[n], (d, hdr[n])


def c_structs():
    out = {}
    for h in G.HEADERS:
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for body, name in re.findall(r"typedef struct \w+ \{(.*?)\} (\w+);", src, flags=re.S):
            fields = []
            for line in body.split(";"):
                line = line.strip()
                if not line:
                    continue
                decl = re.sub(r"\[[^\]]*\]", "", line)  # arrays: the name before [N]
                fields += [re.findall(r"(\w+)\s*$", part.strip())[0] for part in decl.split(",")]
            out[name] = fields
    return out


def doc_structs():
    out = {}
    for blk in RUST_BLOCKS:
        for name, body in re.findall(r"pub struct (\w+)\s*\{(.*?)\}", blk, flags=re.S):
            body = re.sub(r"//[^\n]*", "", body)
            out[name] = re.findall(r"pub (\w+):", body)
    return out


def test_structs_mirror_the_headers():
    c, d = c_structs(), doc_structs()
    missing = sorted(set(c) - set(d))
    assert not missing, missing
    for name, fields in c.items():
        assert d[name] == fields, (name, d[name], fields)


def test_trait_surface_and_lifecycle_are_bound():
    names = {decl_name(x) for x in doc_decls()}
    # Function trait methods (function.rs:28-131) and constructors
    trait = {"fq_function_field", "fq_function_constant", "fq_function_create", "fq_function_clone",
             "fq_function_display", "fq_function_return_type", "fq_function_nullable", "fq_function_set_depth",
             "fq_function_eval", "fq_function_accumulate", "fq_functions_accumulate",
             "fq_function_accumulate_result", "fq_function_merge_state", "fq_function_merge_result",
             "fq_function_free"}
    lifecycle = {"fq_engine_create", "fq_engine_destroy", "fq_engine_set_option", "fq_engine_execute",
                 "fq_engine_execute_row", "fq_engine_explain", "fq_engine_execute_partial",
                 "fq_engine_execute_final", "fq_engine_execute_blocks", "fq_block_stream_next",
                 "fq_block_stream_free", "fq_result_free"}
    split = {"fq_engine_execute_partial", "fq_engine_partial_state_bytes", "fq_engine_execute_final",
             "fq_engine_execute_rccl", "fq_engine_execute_rccl_row", "fq_comm_init", "fq_comm_destroy",
             "fq_comm_set_timeout"}
    assert trait <= names and lifecycle <= names and split <= names, sorted((trait | lifecycle | split) - names)


def test_headings_are_unique():
    heads = re.findall(r"^#+ (.*)$", DOC, flags=re.M)
    numbered = [h.split()[0] for h in heads if re.match(r"\d+[a-z]?\.", h)]
    assert len(numbered) == len(set(numbered)), numbered
