"""Randomised GROUP BY at scale: seeded key shapes over `number` -- scattered
(`% m`), clustered (`/ d`, runs of d rows) and both (`(number / d) % m`) --
with random predicates and integer aggregates, through the engine on the GPU
(sampled LDS-table launches, dense keys, the clustered row layout, radix-
partitioned launches by key range or hash) against the C GROUP BY
restatement (oracle/fq_oracle.c fqo_numbers_group) over the same numbers_mt
blocks.  GROUP BY has no reference transform (plan_parser.rs:284-308 plans it,
pipeline_builder.rs:50-66 ignores it): the semantics are the ungrouped path's
per group, pinned for small sizes against fq_ref in test_fuzz_gpu.py."""
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

E = None
U = None


def setup_module():
    global E, U
    from fq_amd import abi, ops
    ops.require_gpu()
    from fq_amd.engine import Engine
    U = abi.DT_UINT64
    E = Engine()


def teardown_module():
    if E is not None:
        E.close()


def chain_sql(steps):
    s = "number"
    for op, v in steps:
        s = "(%s %s %d)" % (s, op, v)
    return s


def gen_key(rng):
    d = rng.choice([3, 8, 64, 100, 1000, 4096, 70000])
    m = rng.choice([7, 1000, 5000, 65536, 100003, 200000])
    a = rng.choice([3, 7])
    c = rng.choice([1, 12345])
    shape = rng.choice(["mod", "div", "divmod", "muldivmod", "adddivmod", "modmul"])
    return {"mod": [("%", m)], "div": [("/", max(d, 64))], "divmod": [("/", d), ("%", m)],
            "muldivmod": [("*", a), ("/", d), ("%", m)], "adddivmod": [("+", c), ("/", d), ("%", m)],
            "modmul": [("%", min(m, 5000)), ("*", a)]}[shape]


@pytest.mark.parametrize("seed", range(16))
def test_random_group_by_at_scale_matches_c_oracle(seed):
    import oracle_c
    from fq_amd import abi
    from fq_amd.expr import chain, predicate
    rng = random.Random(0x6B00 + seed)
    n = rng.choice([4_000_000, 12_000_000, 40_000_000])
    key_steps = gen_key(rng)
    aggs_sql, aggs = [], []
    for _ in range(rng.randint(1, 4)):
        kind = rng.choice(["count", "sum", "max", "min"])
        vsteps = rng.choice([[], [("+", 1)], [("*", 3)], [("%", 1000)]])
        aggs_sql.append("%s(%s)" % (kind, chain_sql(vsteps)))
        op = {"count": abi.AGG_COUNT, "sum": abi.AGG_SUM, "max": abi.AGG_MAX, "min": abi.AGG_MIN}[kind]
        aggs.append((op, U, chain(U, vsteps)[0] if vsteps else None))
    pred, where = None, ""
    if rng.random() < 0.5:
        p, q = rng.choice([(5, 3), (8, 3), (97, 50)])
        pred = predicate(U, [("%", p)], "<", q)
        where = " WHERE number %% %d < %d" % (p, q)
    k = chain_sql(key_steps)
    sql = "SELECT %s, %s FROM system.numbers_mt(%d)%s GROUP BY %s" % (k, ", ".join(aggs_sql), n, where, k)
    got = [tuple(r) for r in E.execute(sql).rows]
    keys, st = oracle_c.numbers_group(n, chain(U, key_steps)[0], aggs, pred=pred, threads=8, cap_groups=1 << 21)
    o = np.argsort(keys)
    exp = [(int(kk),) + tuple(int(x) for x in s) for kk, s in zip(keys[o], st[o])]
    assert len(got) == len(exp), (sql, len(got), len(exp))
    assert got == exp, (sql, [g for g, e in zip(got, exp) if g != e][:3])
