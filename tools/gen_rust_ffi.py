"""The Rust `extern "C"` blocks of INTEGRATION.md, generated from include/*.h.

Every function the three C-ABI headers declare, in header order, with its
parameters mapped to Rust FFI types (opaque handles as `*mut` zero-sized
structs, `fq_allreduce_fn` as an `Option<extern fn>`).  INTEGRATION.md carries
the output verbatim; tests/test_integration_doc_cpu.py parses the document and
checks every declaration against this mapping of the headers, so the document
cannot drift from the ABI.

python tools/gen_rust_ffi.py [fq_gpu.h|fq_engine.h|fq_comm.h]   (default: all three)
"""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = ("fq_gpu.h", "fq_engine.h", "fq_comm.h")
SCALARS = {"int32_t": "i32", "int64_t": "i64", "uint32_t": "u32", "uint64_t": "u64", "size_t": "usize",
           "fq_status": "fq_status", "char": "c_char", "void": "c_void", "double": "f64",
           "fq_allreduce_fn": "fq_allreduce_fn"}
RUST_KEYWORDS = {"in": "input", "type": "ty", "ref": "r#ref", "fn": "f", "mod": "m"}


def c_declarations(header):
    """[(name, return type, [(param type, param name)])] in header order."""
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"^\s*#.*$", "", src, flags=re.M)
    src = re.sub(r"typedef[^;]*;", "", src)
    out = []
    for ret, name, args in re.findall(r"([A-Za-z_][\w\s\*]*?)\b(fq_\w+)\s*\(([^;{]*?)\)\s*;", src, flags=re.S):
        a = " ".join(args.split())
        params = []
        if a not in ("", "void"):
            for p in a.split(","):
                m = re.match(r"(.*?)(\w+)$", p.strip())
                params.append((m.group(1).strip(), m.group(2)))
        out.append((name, " ".join(ret.split()), params))
    return out


def rust_type(c):
    """C parameter / return type -> Rust FFI type."""
    c = c.replace("*", " * ").split()
    # parse right to left: pointer levels, each with its own const
    levels = []
    while c and c[-1] in ("*", "const"):
        if c[-1] == "*":
            levels.append("mut")
            c.pop()
        else:  # `T *const *p`: the pointer to the right of const is const
            c.pop()
            if levels:
                levels[-1] = "const"
    base_const = "const" in c
    base = [w for w in c if w != "const"][-1]
    t = SCALARS.get(base, base)
    for i, lv in enumerate(reversed(levels)):
        # the innermost pointer's constness comes from the base's const
        kind = ("const" if base_const else "mut") if i == 0 else lv
        t = "*%s %s" % (kind, t)
    return t


def rust_decl(name, ret, params):
    ps = ", ".join("%s: %s" % (RUST_KEYWORDS.get(n, n), rust_type(t)) for t, n in params)
    r = "" if ret == "void" else " -> " + rust_type(ret)
    return "pub fn %s(%s)%s;" % (name, ps, r)


def wrap(decl, width=116, indent="    "):
    if len(indent + decl) <= width:
        return indent + decl
    head, rest = decl.split("(", 1)
    lines, cur = [], indent + head + "("
    cont = " " * len(cur)
    for i, piece in enumerate(rest.split(", ")):
        piece = piece if i == len(rest.split(", ")) - 1 else piece + ","
        if len(cur) + len(piece) + 1 > width and cur.strip() and not cur.endswith("("):
            lines.append(cur.rstrip())
            cur = cont + piece
        else:
            cur = cur + ("" if cur.endswith("(") else " ") + piece
    lines.append(cur)
    return "\n".join(lines)


def extern_block(header):
    body = "\n".join(wrap(rust_decl(*d)) for d in c_declarations(header))
    return 'extern "C" {\n' + body + "\n}"


if __name__ == "__main__":
    for h in (sys.argv[1:] or HEADERS):
        print("// %s\n%s\n" % (h, extern_block(h)))
