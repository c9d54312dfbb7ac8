"""CPU: the library's host code (SQL planner / EXPLAIN, AggregateFinal merge of
exchanged states, the cross-rank exchange protocol, scalar state merge) built
with AddressSanitizer + UBSan and with ThreadSanitizer (`make asan tsan`,
tests/native/fq_host_check.cpp), run over the statements and states the other
CPU tests use plus a deterministic mutation fuzz of the planner.  Results must
equal the regular build's (loaded through ctypes) and the sanitizers must stay
silent.  SURVEY.md section 5: sanitizers on host code only -- no GPU here."""
import os
import subprocess

import pytest

import fq_ref as R
from fq_amd import FQError
from fq_amd.engine import Engine
from fq_amd.numbers import generate_parts, shard
from test_engine_cpu import README_SQL, encode_states

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "fuse-query_amd")

SQLS = [
    "SELECT sum(number)/count(number), max(number), min(number) FROM system.numbers_mt(10000000000)",
    "SELECT max(number+1) FROM system.numbers_mt(10000000000) WHERE (number%8)<3",
    README_SQL,
    "SELECT number%10, count(number), sum(number)/count(number), max(number+1) FROM system.numbers_mt(80000) "
    "WHERE (number%8)<3 GROUP BY number%10",
    "SELECT sum(number) FROM system.numbers_mt(80000) WHERE number > 1 AND number < 5 OR number = 7",
    "SELECT (number+1) as c1 FROM system.numbers_mt(7) LIMIT 2",
    "SELECT sum(number*1.5)/2, min(number-3) FROM system.numbers_mt(123457)",
    "SELECT avg(number) FROM system.numbers_mt(10)",
    "SELECT number FROM system.nope(10)",
    "SELECT sum(number), number FROM system.numbers_mt(10)",
    "SELECT number FROM system.numbers_mt(10) LIMIT 1.5",
    "SELECT sum(number) + 'a' FROM system.numbers_mt(10)",
    "SELECT nope FROM system.numbers_mt(10)",
    "SELECT sum(number) FROM system.numbers_mt(10) HAVING sum(number) > 1",
    "SELECT number, number+1, sum(number) FROM system.numbers_mt(10) GROUP BY number%3",
    "SELECT 1+2*3-4/5 FROM system.numbers_mt(18446744073709551615)",
    "EXPLAIN SELECT sum(number) FROM system.numbers_mt",
    "",
    "SELECT",
    "SELECT ((((number)))) FROM system.numbers_mt(((3)))",
]


def _esc(s):
    return s.replace("\\", "\\\\").replace("\n", "\\n")


def _explain_expected(eng, sql):
    try:
        return "OK " + _esc(eng.explain(sql))
    except FQError as e:
        return "ERR %d %s" % (e.status, _esc(str(e)))


def _final_cases():
    num = R.E_field("number")
    cases = []
    exprs = [R.E_bin("/", R.E_fn("sum", num), R.E_fn("count", num)), R.E_fn("max", num), R.E_fn("min", num)]
    for world, n in ((1, 80), (3, 123457), (8, 1000000)):
        parts = generate_parts(n)
        st = [encode_states(R.aggregate_partial_states(n, exprs, [(b, e) for _, b, e in shard(parts, r, world)]))
              for r in range(world)]
        cases.append(("SELECT sum(number)/count(number), max(number), min(number) FROM system.numbers_mt(%d)" % n,
                      st))
    where = R.E_bin("<", num, R.E_const(5))
    parts = generate_parts(80)
    st = [encode_states(R.aggregate_partial_states(80, [R.E_fn("sum", num)], [(b, e) for _, b, e in
                                                                              shard(parts, r, 8)], where))
          for r in range(8)]
    cases.append(("SELECT sum(number) FROM system.numbers_mt(80) WHERE number < 5", st))  # None error
    key = R.E_bin("%", num, R.E_const(10))
    gexprs = [R.E_fn("count", num), R.E_fn("max", R.E_bin("+", num, R.E_const(1)))]
    parts = [(b, e) for _, b, e in generate_parts(80000)]
    st = [encode_states(R.group_by_partial_states(80000, key, gexprs, parts[4 * r:4 * r + 4])) for r in range(2)]
    cases.append(("SELECT number%10, count(number), max(number+1) FROM system.numbers_mt(80000) GROUP BY number%10",
                  st))
    return cases


def _final_expected(eng, sql, states):
    try:
        r = eng.execute_final(sql, states)
    except FQError as e:
        return "ERR %d %s" % (e.status, _esc(str(e)))
    return "OK " + ";".join(",".join(t if t is not None else "NULL" for t in row) for row in r.text_rows)


@pytest.fixture(scope="module")
def built():
    subprocess.run(["make", "-s", "-j8", "-C", PKG, "asan", "tsan"], check=True, capture_output=True, timeout=600)
    return {k: os.path.join(PKG, "build", k, "fq_host_check") for k in ("asan", "tsan")}


def _run(binary, script, env_extra):
    env = dict(os.environ, **env_extra)
    p = subprocess.run([binary], input=script, capture_output=True, text=True, timeout=600, env=env)
    assert "Sanitizer" not in p.stderr and "runtime error" not in p.stderr, p.stderr[-4000:]
    assert p.returncode == 0, p.stderr[-4000:]
    return p.stdout.splitlines()


def test_asan_ubsan_planner_final_exchange_fuzz(built):
    cmds, expected = [], []
    with Engine(device=-1) as eng:
        for sql in SQLS:
            cmds.append("EXPLAIN " + sql)
            expected.append(_explain_expected(eng, sql))
        for sql, states in _final_cases():
            cmds.append("FINAL %d %s %s" % (len(states), " ".join(s.hex() for s in states), sql))
            expected.append(_final_expected(eng, sql, states))
    for lens in ((5000, 40), (0, 0, 7), (4096, 4097, 1), (10, 20, 30, 40, 50, 60, 70, 80)):
        cmds.append("EXCHANGE " + " ".join(map(str, lens)))
        expected.append("OK")
    for cap, lens in ((0, (10, 20)), (96, (96, 97, 96)), (5, (3, 0)), (104, (104,) * 8)):
        cmds.append("XSIZED %d %s" % (cap, " ".join(map(str, lens))))
        expected.append("OK")
    for sql in ("SELECT sum(number) FROM system.numbers_mt(1000)",
                "SELECT sum(number)/count(number), max(number), min(number) FROM system.numbers_mt(1000)"):
        cmds.append("XERRORS 3 " + sql)
        expected.append("OK")
    cmds.append("MERGE")
    expected.append("OK")
    cmds.append("FUZZ 12345 20000")
    out = _run(built["asan"], "\n".join(cmds) + "\n",
               {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0", "UBSAN_OPTIONS": "print_stacktrace=1"})
    assert len(out) == len(cmds)
    assert out[:-1] == expected
    ok, err = map(int, out[-1].split()[1:])
    assert ok + err == 20000


def test_tsan_exchange_threads(built):
    cmds = ["EXCHANGE 5000 40 3", "EXCHANGE 4096 4097 1 9000", "EXCHANGE " + " ".join(["100"] * 8), "MERGE",
            "XSIZED 96 96 97 96", "XERRORS 4 SELECT sum(number) FROM system.numbers_mt(1000)"]
    out = _run(built["tsan"], "\n".join(cmds) + "\n", {"TSAN_OPTIONS": "halt_on_error=1"})
    assert out == ["OK"] * len(cmds)
