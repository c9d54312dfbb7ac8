"""Randomised SQL parity: seeded random expression trees over `number`
(+ - * / % with UInt64 and Float64 literals, nested both sides), random WHERE
predicates (comparisons, and/or), random aggregates and projections, run
through the engine on the GPU (fused scans, hipRTC trees, fused projection,
node-by-node fallbacks) and through oracle/fq_ref.py (the numpy restatement
of the reference's Function machinery).  Results must be identical (f64
sums within a relative 1e-12: the reduction order differs); when the
reference raises, the engine must raise the same text."""
import math
import os
import random

import pytest

pytestmark = pytest.mark.gpu

E = None
R = None


def setup_module():
    global E, R
    from fq_amd import ops
    ops.require_gpu()
    from fq_amd.engine import Engine
    import fq_ref
    R = fq_ref
    E = Engine()


def teardown_module():
    if E is not None:
        E.close()


OPS = ["+", "-", "*", "/", "%"]


def gen_expr(rng, depth):
    """(sql, fq_ref expression) of an arithmetic tree that uses `number`."""
    if depth == 0 or rng.random() < 0.25:
        return "number", R.E_field("number")
    op = rng.choice(OPS)
    left = gen_expr(rng, depth - 1)
    if op in ("/", "%") and rng.random() < 0.9:
        # mostly divisors that cannot be zero (a few that can: the error path)
        u = rng.random()
        if u < 0.6:
            v = rng.choice([1, 2, 3, 7, 8, 1000, 2.5])
            right = (repr(v), R.E_const(v))
        else:
            k = rng.choice([1, 7])
            sub = gen_expr(rng, depth - 1) if u < 0.8 else ("number", R.E_field("number"))
            right = ("(%s %% 1000 + %d)" % (sub[0], k),
                     R.E_bin("+", R.E_bin("%", sub[1], R.E_const(1000)), R.E_const(k)))
    else:
        right = gen_expr(rng, depth - 1) if rng.random() < 0.5 else gen_leaf(rng)
        if rng.random() < 0.3:
            left, right = right, left
    return "(%s %s %s)" % (left[0], op, right[0]), R.E_bin(op, left[1], right[1])


def gen_leaf(rng):
    if rng.random() < 0.8:
        v = rng.choice([0, 1, 2, 3, 7, 8, 10, 100, 1000])
        return str(v), R.E_const(v)
    v = rng.choice([0.5, 2.5, 3.0])
    return repr(v), R.E_const(v)


def gen_pred(rng):
    cmp = rng.choice(["<", "<=", ">", ">=", "="])
    e = gen_expr(rng, 2)
    k = rng.choice([0, 3, 50, 1000, 40000])
    p = ("%s %s %d" % (e[0], cmp, k), R.E_bin(cmp, e[1], R.E_const(k)))
    if rng.random() < 0.3:
        q = gen_pred_leaf(rng)
        lo = rng.choice(["and", "or"])
        p = ("(%s) %s (%s)" % (p[0], lo.upper(), q[0]), R.E_bin(lo, p[1], q[1]))
    return p


def gen_pred_leaf(rng):
    e = gen_expr(rng, 1)
    k = rng.choice([5, 500, 60000])
    return "%s < %d" % (e[0], k), R.E_bin("<", e[1], R.E_const(k))


def same(a, b):
    if isinstance(a, float) or isinstance(b, float):
        if a is None or b is None:
            return a is b
        if math.isnan(a) or math.isnan(b):
            return math.isnan(a) and math.isnan(b)
        return a == b or abs(a - b) <= 1e-12 * max(abs(a), abs(b))
    return a == b


def run_ref(fn):
    try:
        return fn(), None
    except R.RefError as e:
        return None, str(e)


def run_engine(sql):
    from fq_amd import FQError
    try:
        return E.execute(sql).rows, None
    except FQError as e:
        return None, str(e)


N_CHOICES = [1000, 80000, 100001, 1_000_003]
# FQ_FUZZ_SCALE=k runs k times the seeds (a deeper one-off run; the suite runs 1)
SCALE = max(1, int(os.environ.get("FQ_FUZZ_SCALE", "1")))


@pytest.fixture(params=["auto", "always"])
def jit(request):
    """AUTO: chains on these small blocks run on the interpreting kernels and
    trees on hipRTC; ALWAYS: every fused shape is specialised."""
    from fq_amd import abi, ops
    ops.jit_config(abi.JIT_ALWAYS if request.param == "always" else abi.JIT_AUTO, 0 if request.param == "always" else 1 << 22)
    yield request.param
    ops.jit_config(abi.JIT_AUTO, 1 << 22)


@pytest.mark.parametrize("seed", range(64 * SCALE))
def test_random_aggregate_query(seed, jit):
    rng = random.Random(1000 + seed + (100000 if jit == "always" else 0))
    n = rng.choice(N_CHOICES)
    items = []
    for _ in range(rng.randint(1, 3)):
        agg = rng.choice(["sum", "min", "max", "count"])
        e = gen_expr(rng, rng.randint(1, 3))
        items.append(("%s(%s)" % (agg, e[0]), R.E_fn(agg, e[1])))
    where = gen_pred(rng) if rng.random() < 0.6 else None
    sql = "SELECT %s FROM system.numbers_mt(%d)%s" % (", ".join(s for s, _ in items), n,
                                                       " WHERE " + where[0] if where else "")
    exp, exp_err = run_ref(lambda: [v.value for v in R.aggregate_query(n, [x for _, x in items],
                                                                       where=where[1] if where else None)])
    got, got_err = run_engine(sql)
    if exp_err is not None:
        assert got_err == exp_err, (sql, got, got_err, exp_err)
        return
    assert got_err is None, (sql, got_err, exp)
    assert len(got) == 1 and all(same(g, x) for g, x in zip(got[0], exp)), (sql, got, exp)


@pytest.mark.parametrize("seed", range(48 * SCALE))
def test_random_projection_query(seed):
    rng = random.Random(5000 + seed)
    n = rng.choice([1000, 100001])
    items = [gen_expr(rng, rng.randint(0, 3)) for _ in range(rng.randint(1, 3))]
    where = gen_pred(rng)
    sql = "SELECT %s FROM system.numbers_mt(%d) WHERE %s" % (", ".join(s for s, _ in items), n, where[0])
    exp, exp_err = run_ref(lambda: R.projection_query(n, [x for _, x in items], where=where[1]))
    got, got_err = run_engine(sql)
    if exp_err is not None:
        assert got_err == exp_err, (sql, got_err, exp_err)
        return
    assert got_err is None, (sql, got_err)
    key = lambda r: tuple((0, v) if v is not None else (1, 0) for v in r)  # noqa: E731
    g, x = sorted(got, key=key), sorted(exp, key=key)
    assert len(g) == len(x), (sql, len(g), len(x))
    assert all(all(same(a, b) for a, b in zip(rg, rx)) for rg, rx in zip(g, x)), (sql, g[:5], x[:5])


def gen_int_expr(rng, depth):
    """An expression without Float64 literals (GROUP BY keys are integers)."""
    for _ in range(100):
        e = gen_expr(rng, depth)
        if "." not in e[0]:
            return e
    return "number", R.E_field("number")


@pytest.mark.parametrize("seed", range(20 * SCALE))
def test_random_group_by_query(seed):
    # GROUP BY has no reference transform: fq_ref.group_by_query states the
    # device path's semantics with the reference's Function machinery
    rng = random.Random(9000 + seed)
    n = rng.choice([1000, 80000])
    k = gen_int_expr(rng, rng.randint(0, 1))  # GROUP BY needs a fusable key (<= 8 steps)
    mod = rng.choice([3, 10, 97])
    key = ("(%s) %% %d" % (k[0], mod), R.E_bin("%", k[1], R.E_const(mod)))
    items = []
    for _ in range(rng.randint(1, 3)):
        agg = rng.choice(["sum", "min", "max", "count"])
        e = gen_int_expr(rng, rng.randint(0, 1))
        items.append(("%s(%s)" % (agg, e[0]), R.E_fn(agg, e[1])))
    where = gen_pred(rng) if rng.random() < 0.4 else None
    sql = "SELECT %s, %s FROM system.numbers_mt(%d)%s GROUP BY %s" % (
        key[0], ", ".join(s for s, _ in items), n, " WHERE " + where[0] if where else "", key[0])
    exp, exp_err = run_ref(lambda: R.group_by_query(n, key[1], [x for _, x in items], where=where[1] if where else None))
    got, got_err = run_engine(sql)
    if exp_err is not None:
        assert got_err == exp_err, (sql, got_err, exp_err)
        return
    assert got_err is None, (sql, got_err)
    assert len(got) == len(exp), (sql, got[:5], exp[:5])
    assert all(all(same(a, b) for a, b in zip(rg, rx)) for rg, rx in zip(got, exp)), (sql, got[:5], exp[:5])
