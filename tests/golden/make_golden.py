#!/usr/bin/env python3
"""Regenerates tests/golden/reference_vectors.json: the reference's own
table-driven test vectors for the hot path, extracted as DATA (inputs,
operator, expected outputs / error texts) from its Rust test sources:

  src/datavalues/data_array_arithmetic_test.rs   array op array, array op scalar, scalar op array
  src/datavalues/data_array_comparison_test.rs   idem for = < <= > >=
  src/datavalues/data_array_aggregate_test.rs    min/max/sum over one array
  src/datavalues/data_value_aggregate_test.rs    scalar state merges
  src/datavalues/data_value_arithmetic_test.rs   scalar add
  src/datavalues/data_array_logic_test.rs        and / or over Boolean arrays
  src/functions/function_arithmetic_test.rs      ArithmeticFunction over a block's fields
  src/functions/function_comparison_test.rs      ComparisonFunction over a block's fields

Only literal values are read (the XArray::from(vec![...]) and
DataValue::X(Some(..)) literals of each table row); nothing is executed.
Usage: python tests/golden/make_golden.py [/root/reference]
"""
import json
import os
import re
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_vectors.json")


def block(src, start):
    """Text between the bracket at src[start] and its match (exclusive)."""
    pairs = {"[": "]", "(": ")", "{": "}"}
    open_c = src[start]
    close_c = pairs[open_c]
    depth = 0
    i = start
    in_str = False
    while i < len(src):
        c = src[i]
        if in_str:
            if c == "\\":
                i += 2
                continue
            if c == '"':
                in_str = False
        elif c == '"':
            in_str = True
        elif c == open_c:
            depth += 1
        elif c == close_c:
            depth -= 1
            if depth == 0:
                return src[start + 1:i], i + 1
        i += 1
    raise ValueError("unbalanced")


def split_top(s):
    """Split a comma-separated list at depth 0."""
    out, depth, cur, in_str = [], 0, "", False
    i = 0
    while i < len(s):
        c = s[i]
        if in_str:
            cur += c
            if c == "\\":
                cur += s[i + 1]
                i += 2
                continue
            if c == '"':
                in_str = False
        elif c == '"':
            in_str = True
            cur += c
        elif c in "([{":
            depth += 1
            cur += c
        elif c in ")]}":
            depth -= 1
            cur += c
        elif c == "," and depth == 0:
            if cur.strip():
                out.append(cur.strip())
            cur = ""
        else:
            cur += c
        i += 1
    if cur.strip():
        out.append(cur.strip())
    return out


def num(tok, tname):
    tok = tok.strip()
    if tname in ("Float32", "Float64"):
        return float(tok)
    return int(tok)


ARR = re.compile(r"^Arc::new\((\w+)Array::from\(vec!\[(.*)\]\)\)$", re.S)
VAL = re.compile(r"^DataValue::(\w+)\((.*)\)$", re.S)


def literal(expr):
    expr = expr.strip()
    m = ARR.match(expr)
    if m:
        t, body = m.group(1), m.group(2)
        t = {"String": "Utf8"}.get(t, t)
        items = split_top(body)
        if t == "Utf8":
            vals = [json.loads(x) for x in items]
        elif t == "Boolean":
            vals = [x == "true" for x in items]
        else:
            vals = [num(x, t) for x in items]
        return {"array": True, "type": t, "values": vals}
    m = VAL.match(expr)
    if m:
        t, inner = m.group(1), m.group(2).strip()
        t = {"String": "Utf8"}.get(t, t)
        if inner == "None":
            return {"array": False, "type": t, "kind": "none"}
        mm = re.match(r"^Some\((.*)\)$", inner, re.S)
        v = mm.group(1).strip()
        if t == "Utf8":
            v = json.loads(v.replace(".to_string()", ""))
        elif t == "Boolean":
            v = v == "true"
        else:
            v = num(v, t)
        return {"array": False, "type": t, "kind": "some", "value": v}
    raise ValueError("unparsed literal: %r" % expr[:80])


def field(body, name):
    m = re.search(r"\b%s:\s*" % name, body)
    if not m:
        return None
    i = m.end()
    if body.startswith("vec!", i):
        inner, _ = block(body, body.index("[", i))
        return ("vec", inner)
    # single expression up to the next top-level comma
    rest = body[i:]
    return ("one", split_top(rest)[0])


OPS = {"Add": "+", "Sub": "-", "Mul": "*", "Div": "/", "Eq": "=", "Lt": "<", "LtEq": "<=", "Gt": ">",
       "GtEq": ">=", "Min": "min", "Max": "max", "Sum": "sum", "Count": "count", "And": "and", "Or": "or"}


def tests_in(path, struct):
    src = open(os.path.join(REF, path)).read()
    out = []
    for fm in re.finditer(r"fn (test_\w+)\(\)", src):
        fn_name = fm.group(1)
        fn_end = src.find("\nfn ", fm.end())
        body_fn = src[fm.end(): fn_end if fn_end > 0 else len(src)]
        for m in re.finditer(r"\b%s \{" % struct, body_fn):
            if body_fn[m.start() - 7:m.start()].strip().startswith("struct"):
                continue
            body, _ = block(body_fn, m.end() - 1)
            if "name:" not in body:
                continue
            line = src[:fm.end()].count("\n") + body_fn[:m.start()].count("\n") + 1
            t = {"fn": fn_name, "line": line, "name": json.loads(field(body, "name")[1])}
            op = field(body, "op")[1]
            t["op"] = OPS[op.split("::")[-1]]
            for key in ("args", "expect", "array", "scalar", "error"):
                f = field(body, key)
                if f is None:
                    continue
                kind, text = f
                if key == "error":
                    t["error"] = [json.loads(x) for x in split_top(text)] if kind == "vec" else json.loads(text)
                elif key == "args":
                    items = split_top(text)
                    if items and items[0].startswith("vec!"):
                        t["args"] = [[literal(x) for x in split_top(block(it, it.index("["))[0])] for it in items]
                    else:
                        t["args"] = [literal(x) for x in items]
                elif kind == "vec":
                    t[key] = [literal(x) for x in split_top(text)]
                else:
                    t[key] = literal(text)
            out.append(t)
    return out


def function_tests(path, fn):
    """Function-level tables (function_arithmetic_test.rs, function_comparison_test.rs):
    the block's columns (named by the schema order a, b, c), the display
    (which names the two argument fields), the expected array or error."""
    src = open(os.path.join(REF, path)).read()
    fm = re.search(r"fn %s\(\)" % fn, src)
    body_fn = src[fm.end():]
    out = []
    for m in re.finditer(r"\bTest \{", body_fn):
        if body_fn[m.start() - 7:m.start()].strip().startswith("struct"):
            continue
        body, _ = block(body_fn, m.end() - 1)
        if "name:" not in body:
            continue
        line = src[:fm.end()].count("\n") + body_fn[:m.start()].count("\n") + 1
        t = {"fn": fn, "line": line, "name": json.loads(field(body, "name")[1]),
             "op": OPS[field(body, "op")[1].split("::")[-1]],
             "display": json.loads(field(body, "display")[1]),
             "nullable": field(body, "nullable")[1] == "true",
             "error": json.loads(field(body, "error")[1])}
        bi = body.index("DataBlock::create(")
        inner, _ = block(body, bi + len("DataBlock::create"))
        cols = split_top(inner)[1]
        t["columns"] = [literal(x) for x in split_top(block(cols, cols.index("["))[0])]
        t["expect"] = literal(field(body, "expect")[1])
        out.append(t)
    return out


def main():
    data = {
        "generator": "tests/golden/make_golden.py (parses the literal tables of the reference's tests)",
        "reference": "dantengsky/fuse-query @ /root/reference",
        "array_arithmetic": tests_in("src/datavalues/data_array_arithmetic_test.rs", "ArrayTest"),
        "array_comparison": tests_in("src/datavalues/data_array_comparison_test.rs", "ArrayTest"),
        "array_aggregate": tests_in("src/datavalues/data_array_aggregate_test.rs", "ArrayTest"),
        "value_aggregate": tests_in("src/datavalues/data_value_aggregate_test.rs", "ScalarTest"),
        "value_arithmetic": tests_in("src/datavalues/data_value_arithmetic_test.rs", "ScalarTest"),
        "array_logic": tests_in("src/datavalues/data_array_logic_test.rs", "ArrayTest"),
        "function_arithmetic": function_tests("src/functions/function_arithmetic_test.rs",
                                              "test_arithmetic_function"),
        "function_comparison": function_tests("src/functions/function_comparison_test.rs",
                                              "test_comparison_function"),
    }
    for k, v in data.items():
        if isinstance(v, list):
            print(k, len(v), "tables")
    json.dump(data, open(OUT, "w"), indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
