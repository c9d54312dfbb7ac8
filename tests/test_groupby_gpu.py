"""GROUP BY hash aggregation kernels (include/fq_gpu.h fq_group_*) against a
numpy group-by on the same seeded columns.

The reference has no GROUP BY execution (plan_parser.rs:284-308 plans it,
pipeline_builder.rs:50-66 ignores group_expr), so there is nothing of the
reference to pin these results to: they are checked against numpy with the
ungrouped path's value semantics (wrapping u64/i64 sums, IEEE f64, f64 sums
within a written tolerance because atomics add in no fixed order)."""
import numpy as np
import pytest

from fq_amd import abi
from fq_amd.expr import COL, chain, predicate

pytestmark = pytest.mark.gpu

ops = None
U, I, F = abi.DT_UINT64, abi.DT_INT64, abi.DT_FLOAT64


def setup_module():
    global ops
    from fq_amd import ops as _ops
    _ops.require_gpu()
    ops = _ops


def np_groupby_arrays(keys, vals_list, kinds):
    """-> (sorted distinct keys, [state array per aggregate]) with the device's
    state semantics (wrapping integer sums, f64 sums in sorted-key order)."""
    order = np.argsort(keys, kind="stable")
    k = keys[order]
    uniq, start = np.unique(k, return_index=True)
    counts = np.diff(np.append(start, len(k)))
    out = []
    for kind, vals in zip(kinds, vals_list):
        if kind == abi.AGG_COUNT:
            out.append(counts.astype(np.uint64))
            continue
        v = vals[order]
        if kind == abi.AGG_SUM:
            out.append(np.add.reduceat(v, start) if v.dtype != np.float64 else np.add.reduceat(v, start))
        elif kind == abi.AGG_MAX:
            out.append(np.maximum.reduceat(v, start))
        else:
            out.append(np.minimum.reduceat(v, start))
    return uniq, out


def np_groupby(keys, vals_list, kinds):
    """-> {key: [state per aggregate]} with the device's state semantics."""
    uniq, st = np_groupby_arrays(keys, vals_list, kinds)
    cols = [a.tolist() for a in st]
    return {int(key): [c[i] for c in cols] for i, key in enumerate(uniq.tolist())}


def decode(states, dts):
    res = []
    for s, dt in zip(states, dts):
        if dt == F:
            res.append(s.view(np.float64))
        elif dt == I:
            res.append(s.view(np.int64))
        else:
            res.append(s)
    return res


def run(col, aggs, key=None, values=None, pred=None, key_dtype=U, capacity=1 << 12):
    t = ops.GroupTable(capacity, aggs, key_dtype)
    t.aggregate(col, pred, key, values)
    keys, states = t.extract()
    if key_dtype == I:
        keys = keys.view(np.int64)
    st = decode(states, [dt for _, dt in aggs])
    return {int(k): [st[a][i] for a in range(len(aggs))] for i, k in enumerate(keys)}


def compare(got, exp, kinds, dts, fsum_bound=None):
    assert set(got) == set(exp), (len(got), len(exp))
    for k, e in exp.items():
        g = got[k]
        for a, (kind, dt) in enumerate(zip(kinds, dts)):
            if dt == F and kind == abi.AGG_SUM:
                assert abs(g[a] - e[a]) <= fsum_bound[k], (k, a, g[a], e[a])
            elif dt == F:
                assert g[a] == e[a] or (np.isnan(g[a]) and np.isnan(e[a])), (k, a, g[a], e[a])
            else:
                assert int(g[a]) == int(e[a]), (k, a, g[a], e[a])


def test_low_cardinality_mod_key_all_aggregates():
    n = 3_000_017
    col = ops.splitmix_column(0x6B, 0, n)
    x = col.to_numpy()
    key, _ = chain(U, [("%", 1000)])
    vf, _ = chain(U, [("*", 1.5)])
    aggs = [(abi.AGG_COUNT, U), (abi.AGG_SUM, U), (abi.AGG_MAX, U), (abi.AGG_MIN, U), (abi.AGG_SUM, F),
            (abi.AGG_MAX, F)]
    got = run(col, aggs, key=key, values=[None, None, None, None, vf, vf])
    xf = x.astype(np.float64) * 1.5
    exp = np_groupby(x % np.uint64(1000), [None, x, x, x, xf, xf], [k for k, _ in aggs])
    # f64 sum tolerance: 1e-12 * sum(|v|) of the group (atomic add order is unspecified)
    k = x % np.uint64(1000)
    bound = {int(g): 1e-12 * float(np.abs(xf[k == g]).sum()) for g in np.unique(k)}
    compare(got, exp, [k for k, _ in aggs], [d for _, d in aggs], bound)


def test_filtered_group_by_c4_shape():
    # SELECT number%10, max(number+1), count(number) ... WHERE (number%8)<3 GROUP BY number%10
    n = 2_000_000
    col = ops.numbers_column(0, n)
    x = np.arange(n, dtype=np.uint64)
    key, _ = chain(U, [("%", 10)])
    v, _ = chain(U, [("+", 1)])
    pred = predicate(U, [("%", 8)], "<", 3)
    aggs = [(abi.AGG_MAX, U), (abi.AGG_COUNT, U)]
    got = run(col, aggs, key=key, values=[v, None], pred=pred)
    m = (x % np.uint64(8)) < 3
    exp = np_groupby((x % np.uint64(10))[m], [(x + np.uint64(1))[m], None], [abi.AGG_MAX, abi.AGG_COUNT])
    compare(got, exp, [abi.AGG_MAX, abi.AGG_COUNT], [U, U])


@pytest.mark.parametrize("length", [3, 4, 20, 100, 1000, 70000])
def test_clustered_key_runs_match_numpy(length):
    # keys constant over runs of `length` consecutive rows: a workgroup whose
    # first tile shows such runs switches to eight consecutive rows per lane
    # (LDS transpose, in-lane and wave-wide merging, fq_jit_groupby mode 1;
    # shapes whose kernel would spill registers keep mode 0 only, so the
    # aggregates here are the spill-free integer ones); start 123 puts the
    # runs off the tile grid, the odd length leaves a tail, the predicate
    # removes rows from inside runs
    n = 6_000_013
    col = ops.numbers_column(123, n)
    x = np.arange(123, 123 + n, dtype=np.uint64)
    key, _ = chain(U, [("/", length), ("%", 1000)])
    pred = predicate(U, [("%", 7)], "<", 5)
    aggs = [(abi.AGG_COUNT, U), (abi.AGG_SUM, U), (abi.AGG_MAX, U), (abi.AGG_MIN, U)]
    got = run(col, aggs, key=key, values=[None] * 4, pred=pred)
    m = (x % np.uint64(7)) < 5
    xm = x[m]
    exp = np_groupby((xm // np.uint64(length)) % np.uint64(1000), [None, xm, xm, xm], [a for a, _ in aggs])
    compare(got, exp, [a for a, _ in aggs], [U] * 4)


def test_clustered_f64_and_signed_states_match_numpy():
    # the same over f64 / Int64 values (whichever mode their kernel takes)
    n = 4_000_037
    col = ops.numbers_column(5, n)
    x = np.arange(5, 5 + n, dtype=np.uint64)
    key, _ = chain(U, [("/", 100), ("%", 1000)])
    vf, _ = chain(U, [("*", 1.5)])
    vi, _ = chain(U, [("-", (7, "Int64"))])
    aggs = [(abi.AGG_COUNT, U), (abi.AGG_SUM, F), (abi.AGG_MAX, F), (abi.AGG_MIN, I)]
    got = run(col, aggs, key=key, values=[None, vf, vf, vi])
    k = (x // np.uint64(100)) % np.uint64(1000)
    xf = x.astype(np.float64) * 1.5
    exp = np_groupby(k, [None, xf, xf, x.astype(np.int64) - 7], [a for a, _ in aggs])
    bound = {int(g): 1e-12 * float(np.abs(xf[k == g]).sum()) for g in np.unique(k)}
    compare(got, exp, [a for a, _ in aggs], [d for _, d in aggs], bound)


def test_clustered_sorted_random_column_matches_numpy():
    # a sorted column of random values with random run lengths (1..300),
    # grouped by the value itself: clustered keys that are not a function of
    # the row index
    rng = np.random.default_rng(0xC1)
    vals = np.sort(rng.integers(0, 1 << 40, 40_000, dtype=np.uint64))
    x = np.repeat(vals, rng.integers(1, 300, len(vals)))[:5_000_011]
    col = ops.from_numpy(x)
    aggs = [(abi.AGG_COUNT, U), (abi.AGG_SUM, U), (abi.AGG_MAX, U)]
    got = run(col, aggs, values=[None] * 3, capacity=1 << 17)
    exp = np_groupby(x, [None, x, x], [a for a, _ in aggs])
    compare(got, exp, [a for a, _ in aggs], [U] * 3)


def test_high_cardinality_bypasses_lds():
    n = 1_000_003
    col = ops.splitmix_column(0x77, 5, n)
    x = col.to_numpy()
    aggs = [(abi.AGG_COUNT, U), (abi.AGG_SUM, U)]
    got = run(col, aggs, capacity=1 << 21)
    uniq, cnt = np.unique(x, return_counts=True)
    assert len(got) == len(uniq)
    for kk, c in zip(uniq[:1000], cnt[:1000]):
        assert got[int(kk)] == [c, kk * np.uint64(c)]


def test_signed_keys_and_states():
    n = 500_000
    col = ops.numbers_column(0, n)
    x = np.arange(n, dtype=np.int64)
    key, kdt = chain(U, [("-", (250_000, "Int64")), ("/", (1000, "Int64"))])  # Int64, negative keys
    assert kdt == I
    v, _ = chain(U, [("-", (300_000, "Int64"))])
    aggs = [(abi.AGG_MIN, I), (abi.AGG_MAX, I), (abi.AGG_SUM, I)]
    got = run(col, aggs, key=key, values=[v, v, v], key_dtype=I)
    kk = np.trunc((x - 250_000) / 1000).astype(np.int64)  # truncating division
    vv = x - 300_000
    exp = np_groupby(kk, [vv, vv, vv], [abi.AGG_MIN, abi.AGG_MAX, abi.AGG_SUM])
    compare(got, exp, [abi.AGG_MIN, abi.AGG_MAX, abi.AGG_SUM], [I, I, I])


def test_empty_marker_key_gets_its_own_slot():
    col = ops.numbers_column(0, 10_000)
    key, _ = chain(U, [("*", 0), ("-", 1)])  # every key = 2^64-1 (the table's empty marker)
    got = run(col, [(abi.AGG_COUNT, U), (abi.AGG_MAX, U)], key=key)
    assert got == {2**64 - 1: [10_000, 9_999]}
    key2, _ = chain(U, [("%", 2), ("-", 1)])  # keys 2^64-1 and 0
    got = run(col, [(abi.AGG_COUNT, U)], key=key2)
    assert got == {2**64 - 1: [5000], 0: [5000]}


def test_bitmap_predicate_and_no_rows():
    n = 100_000
    col = ops.splitmix_column(1, 0, n)
    x = col.to_numpy()
    bm = ops.compare("<", col, 2**62)
    p = abi.fq_pred()
    p.kind = abi.PRED_BITMAP
    p.bitmap = bm.ptr
    key, _ = chain(U, [("%", 7)])
    got = run(col, [(abi.AGG_COUNT, U)], key=key, pred=p)
    m = x < np.uint64(2**62)
    exp = np_groupby((x % np.uint64(7))[m], [None], [abi.AGG_COUNT])
    compare(got, exp, [abi.AGG_COUNT], [U])
    none = predicate(U, [], ">", 2**64 - 1)
    assert run(col, [(abi.AGG_COUNT, U)], key=key, pred=none) == {}


def test_table_full_and_div_zero_are_reported():
    col = ops.numbers_column(0, 100_000)
    t = ops.GroupTable(64, [(abi.AGG_COUNT, U)])
    t.aggregate(col)  # 100k distinct keys into 64 slots
    with pytest.raises(ops.FQError) as ei:
        t.count()
    assert ei.value.status == abi.FQ_E_TABLE_FULL
    key, _ = chain(U, [("%", 2), ("/", 7, True)])  # 7 / (number % 2): zero on even rows
    t2 = ops.GroupTable(64, [(abi.AGG_COUNT, U)])
    t2.aggregate(col, key=key)
    with pytest.raises(ops.FQError) as ei:
        t2.count()
    assert str(ei.value) == "Internal Error: Divide by zero error"


def test_accumulates_across_blocks():
    # two device blocks into one table == one block over both
    a = ops.numbers_column(0, 600_000)
    b = ops.numbers_column(600_000, 400_001)
    key, _ = chain(U, [("%", 97)])
    aggs = [(abi.AGG_SUM, U), (abi.AGG_COUNT, U), (abi.AGG_MIN, U)]
    t = ops.GroupTable(256, aggs)
    t.aggregate(a, key=key)
    t.aggregate(b, key=key)
    keys, sts = t.extract()
    got = {int(k): [int(s[i]) for s in sts] for i, k in enumerate(keys)}
    x = np.arange(1_000_001, dtype=np.uint64)
    exp = np_groupby(x % np.uint64(97), [x, None, x], [abi.AGG_SUM, abi.AGG_COUNT, abi.AGG_MIN])
    compare(got, exp, [abi.AGG_SUM, abi.AGG_COUNT, abi.AGG_MIN], [U, U, U])


@pytest.mark.parametrize("mod,rows", [(20_000, 3_000_017), (300_000, 2_000_003), (5_000, 10_001)])
def test_partitioned_launches_after_the_table_fills(mod, rows):
    """Later launches into a table holding more groups than half an LDS table
    split the keys into partitions (each workgroup aggregates one partition
    and every row is read once per partition); the result must equal one
    numpy group-by over all blocks.  The last case has too few rows for a
    grid the partition count divides (falls back to one partition)."""
    aggs = [(abi.AGG_COUNT, U), (abi.AGG_SUM, U), (abi.AGG_MAX, U), (abi.AGG_MIN, F)]
    key, _ = chain(U, [("%", mod)])
    vf, _ = chain(U, [("*", 0.5)])
    t = ops.GroupTable(1 << 20, aggs)
    xs = []
    for i in range(3):
        col = ops.splitmix_column(0x9A + i, 0, rows)
        xs.append(col.to_numpy())
        t.aggregate(col, None, key, [None, None, None, vf])
    keys, states = t.extract()
    st = decode(states, [dt for _, dt in aggs])
    got = {int(k): [st[a][i] for a in range(len(aggs))] for i, k in enumerate(keys)}
    x = np.concatenate(xs)
    exp = np_groupby(x % np.uint64(mod), [None, x, x, x.astype(np.float64) * 0.5], [k for k, _ in aggs])
    compare(got, exp, [k for k, _ in aggs], [d for _, d in aggs])


# ---- GROUP BY through the SQL pipeline (GroupByPartial x P -> Merge -> Final) ----
import fq_ref as R  # noqa: E402


@pytest.fixture(scope="module")
def eng():
    from fq_amd.engine import Engine
    e = Engine()
    yield e
    e.close()


N = R.E_field("number")


def _c(v):
    return R.E_const(v)


@pytest.mark.parametrize("total", [100_000, 1_000_000, 4_000_000])
def test_sql_group_by_matches_oracle(eng, total):
    sql = ("SELECT number%%3, count(number), sum(number)/count(number), max(number+1), min(number) "
           "FROM system.numbers_mt(%d) WHERE (number%%8)<3 GROUP BY number%%3" % total)
    r = eng.execute(sql)
    exp = R.group_by_query(total, R.E_bin("%", N, _c(3)),
                           [R.E_fn("count", N), R.E_bin("/", R.E_fn("sum", N), R.E_fn("count", N)),
                            R.E_fn("max", R.E_bin("+", N, _c(1))), R.E_fn("min", N)],
                           where=R.E_bin("<", R.E_bin("%", N, _c(8)), _c(3)))
    assert r.rows == exp
    assert r.names == ["number % 3", "Count(number)", "Sum(number) / Count(number)", "Max(number + 1)",
                       "Min(number)"]


def test_sql_group_by_f64_and_keys_only(eng):
    r = eng.execute("SELECT number%5, sum(number*1.5) FROM system.numbers_mt(80000) GROUP BY number%5")
    exp = R.group_by_query(80000, R.E_bin("%", N, _c(5)), [R.E_fn("sum", R.E_bin("*", N, _c(1.5)))])
    assert [k for k, _ in r.rows] == [k for k, _ in exp]
    for (k, got), (_, e) in zip(r.rows, exp):
        assert abs(got - e) <= 1e-12 * abs(e)  # f64 sum: atomic add order unspecified
    r = eng.execute("SELECT number%7 FROM system.numbers_mt(1000) GROUP BY number%7")
    assert r.rows == [(k,) for k in range(7)]


def test_sql_group_by_sizes_distinct_keys(eng):
    # 160,000 distinct keys (GROUP BY number): the sample sees keys that keep
    # coming, the table is sized for every partition's
    r = eng.execute("SELECT number, count(number) FROM system.numbers_mt(160000) GROUP BY number")
    assert len(r.rows) == 160000 and r.rows[0] == (0, 1) and r.rows[-1] == (159999, 1)


def test_sql_group_by_grows_a_full_table(eng):
    # clustered keys: each partition repeats its own 25,000 keys, so the sample
    # sizes 131,072 slots for 200,000 groups -> TABLE_FULL -> re-run with 16x
    r = eng.execute("SELECT number/2, count(number), min(number) FROM system.numbers_mt(400000) GROUP BY number/2")
    assert len(r.rows) == 200000 and r.rows[0] == (0, 2, 0) and r.rows[-1] == (199999, 2, 399998)


def test_sql_group_by_limit_and_explain(eng):
    r = eng.execute("SELECT number%10, count(number) FROM system.numbers_mt(80000) GROUP BY number%10 LIMIT 3")
    assert r.rows == [(0, 8000), (1, 8000), (2, 8000)]
    txt = eng.explain("SELECT number%10, sum(number) FROM system.numbers_mt(80000) GROUP BY number%10")
    # plan_display.rs:43-49 prints the group list right after the aggregates
    assert "Aggregate: sum([number])(number % 10)" in txt or "Aggregate: sum([number])" in txt


def test_sql_group_by_errors(eng):
    from fq_amd import FQError  # noqa: F401
    with pytest.raises(Exception) as ei:
        eng.execute("SELECT number, number+1, sum(number) FROM system.numbers_mt(10) GROUP BY number%3")
    assert "Projection references non-aggregate values" in str(ei.value)


def test_sql_group_by_with_logic_predicate(eng):
    total = 1_000_000
    r = eng.execute("SELECT number%%4, count(number), max(number) FROM system.numbers_mt(%d) "
                    "WHERE number%%8 < 3 AND number > 100 GROUP BY number%%4" % total)
    w = R.E_bin("and", R.E_bin("<", R.E_bin("%", N, _c(8)), _c(3)), R.E_bin(">", N, _c(100)))
    exp = R.group_by_query(total, R.E_bin("%", N, _c(4)), [R.E_fn("count", N), R.E_fn("max", N)], where=w)
    assert r.rows == exp


# ---- radix-partitioned high-cardinality path (fq_group_aggregate_partitioned) ----

def run_parts(col, aggs, log2p, key=None, values=None, pred=None, key_dtype=U, capacity=1 << 12, blocks=1):
    t = ops.GroupTable(capacity, aggs, key_dtype)
    for _ in range(blocks):
        t.aggregate(col, pred, key, values, log2_parts=log2p)
    keys, states = t.extract()
    if key_dtype == I:
        keys = keys.view(np.int64)
    st = decode(states, [dt for _, dt in aggs])
    return {int(k): [st[a][i] for a in range(len(aggs))] for i, k in enumerate(keys)}


def run_parts_arrays(col, aggs, log2p, key=None, values=None, capacity=1 << 12, blocks=1):
    """-> (keys ascending, [decoded state array per aggregate]) of the table."""
    t = ops.GroupTable(capacity, aggs, U)
    for _ in range(blocks):
        t.aggregate(col, None, key, values, log2_parts=log2p)
    keys, states = t.extract()
    st = decode(states, [dt for _, dt in aggs])
    o = np.argsort(keys, kind="stable")
    return keys[o], [a[o] for a in st]


@pytest.mark.parametrize("mod,log2p", [(7, 1), (1000, 3), (65_536, 6), (100_000, 6), (2_000_000, 8), (None, 8)])
def test_partitioned_matches_numpy(mod, log2p):
    # 2 blocks into one table: rows of both, every group once, all aggregate kinds;
    # `% d` keys with d <= P * S take range bins (65,536: the `& mask` form),
    # 2,000,000 and the identity key hash bins
    n = 3_000_017
    col = ops.splitmix_column(0x5A, 3, n)
    x = col.to_numpy()
    key = chain(U, [("%", mod)])[0] if mod else None
    vf, _ = chain(U, [("*", 0.25)])
    aggs = [(abi.AGG_COUNT, U), (abi.AGG_SUM, U), (abi.AGG_MAX, U), (abi.AGG_MIN, U), (abi.AGG_SUM, F)]
    groups = min(n, mod or n)
    gk, gs = run_parts_arrays(col, aggs, log2p, key=key, values=[None, None, None, None, vf], capacity=4 * groups,
                              blocks=2)
    xx = np.concatenate([x, x])
    k = xx % np.uint64(mod) if mod else xx
    xf = xx.astype(np.float64) * 0.25
    ek, es = np_groupby_arrays(k, [None, xx, xx, xx, xf], [a for a, _ in aggs])
    assert np.array_equal(gk, ek), (len(gk), len(ek))
    for a in range(4):  # integer states bit for bit
        assert np.array_equal(gs[a], es[a]), a
    # f64 sums: atomic add order is unspecified -- 1e-12 relative per group
    assert np.all(np.abs(gs[4] - es[4]) <= 4e-12 * np.abs(es[4]) + 1e-9)


@pytest.mark.parametrize("steps,pred", [
    ([("/", 1_000_000_000)], False),   # hash bins, one key: every row in one bin
    ([("/", 5000), ("%", 3)], False),  # range bins, runs of 5,000 rows: a tile's rows mostly one bin
    ([("%", 2)], True),                # range bins, two keys, a predicate keeping 3/8 of the rows
])
def test_partitioned_skewed_bins(steps, pred):
    # block chains under skew: a tile's whole run in one bin spills into many
    # blocks at once; the workspace bound (full blocks but each chain's last)
    # holds; results equal numpy
    n = 3_000_017
    col = ops.numbers_column(0, n)
    x = np.arange(n, dtype=np.uint64)
    key, _ = chain(U, steps)
    aggs = [(abi.AGG_COUNT, U), (abi.AGG_SUM, U), (abi.AGG_MAX, U)]
    p = predicate(U, [("%", 8)], "<", 3) if pred else None
    got = run_parts(col, aggs, 8, key=key, pred=p, capacity=1 << 12)
    k = x
    for op, d in steps:
        k = k // np.uint64(d) if op == "/" else k % np.uint64(d)
    m = (x % np.uint64(8)) < 3 if pred else np.ones(n, dtype=bool)
    exp = np_groupby(k[m], [None, x[m], x[m]], [a for a, _ in aggs])
    compare(got, exp, [a for a, _ in aggs], [d for _, d in aggs])


@pytest.mark.parametrize("with_count", [True, False])
def test_partitioned_range_bins_with_and_without_count(with_count):
    # range bins: with a COUNT state the flush rebuilds each key from its bin
    # and LDS slot (no key written per row); without one the key is stored
    n = 2_000_003
    col = ops.splitmix_column(0x77, 1, n)
    x = col.to_numpy()
    key, _ = chain(U, [("%", 90_000)])
    aggs = ([(abi.AGG_COUNT, U)] if with_count else []) + [(abi.AGG_MAX, U), (abi.AGG_SUM, U)]
    got = run_parts(col, aggs, 7, key=key, capacity=1 << 18)
    exp = np_groupby(x % np.uint64(90_000), [None if a == abi.AGG_COUNT else x for a, _ in aggs],
                     [a for a, _ in aggs])
    compare(got, exp, [a for a, _ in aggs], [d for _, d in aggs])


def test_partitioned_equals_lds_path_bit_exact():
    # integer states: the partitioned path and the plain kernel agree exactly
    n = 5_000_003
    col = ops.splitmix_column(0x31, 0, n)
    key, _ = chain(U, [("%", 4096)])
    aggs = [(abi.AGG_COUNT, U), (abi.AGG_SUM, U), (abi.AGG_MIN, U)]
    a = run(col, aggs, key=key, capacity=1 << 14)
    b = run_parts(col, aggs, 4, key=key, capacity=1 << 14)
    assert a == b


def test_partitioned_predicates_and_misaligned_column():
    n = 1_000_001
    base = ops.numbers_column(0, n + 1)
    x = np.arange(1, n + 1, dtype=np.uint64)
    col = ops.DeviceColumn(base.buf, n, U, 8)  # rows 1..n: 8-byte aligned, not 16
    key, _ = chain(U, [("%", 50_000)])
    v, _ = chain(U, [("+", 1)])
    aggs = [(abi.AGG_MAX, U), (abi.AGG_COUNT, U)]
    pred = predicate(U, [("%", 8)], "<", 3)
    got = run_parts(col, aggs, 5, key=key, values=[v, None], pred=pred, capacity=1 << 17)
    m = (x % np.uint64(8)) < 3
    exp = np_groupby((x % np.uint64(50_000))[m], [(x + np.uint64(1))[m], None], [abi.AGG_MAX, abi.AGG_COUNT])
    compare(got, exp, [abi.AGG_MAX, abi.AGG_COUNT], [U, U])
    # bitmap predicate: rows by index
    bm = ops.compare("<", col, 700_000)
    p = abi.fq_pred()
    p.kind = abi.PRED_BITMAP
    p.bitmap = bm.ptr
    got = run_parts(col, [(abi.AGG_COUNT, U)], 5, key=key, pred=p, capacity=1 << 17)
    m = x < np.uint64(700_000)
    exp = np_groupby((x % np.uint64(50_000))[m], [None], [abi.AGG_COUNT])
    compare(got, exp, [abi.AGG_COUNT], [U])


def test_partitioned_signed_keys_small_inputs_and_errors():
    col = ops.numbers_column(0, 300_000)
    x = np.arange(300_000, dtype=np.int64)
    key, kdt = chain(U, [("-", (150_000, "Int64"))])  # negative and positive Int64 keys, all distinct
    aggs = [(abi.AGG_SUM, I), (abi.AGG_COUNT, U)]
    v, _ = chain(U, [("-", (7, "Int64"))])
    got = run_parts(col, aggs, 7, key=key, values=[v, None], key_dtype=I, capacity=1 << 20)
    assert len(got) == 300_000
    assert got[-150_000] == [-7, 1] and got[149_999] == [299_992, 1]
    for n in (0, 1, 63, 8191, 8193):  # fewer rows than one tile / than the workgroups
        c = ops.numbers_column(5, n)
        g = run_parts(c, [(abi.AGG_COUNT, U)], 2, capacity=1 << 14) if n else {}
        assert g == {5 + i: [1] for i in range(n)}
    key, _ = chain(U, [("%", 2), ("/", 7, True)])  # 7 / (number % 2): zero on even rows
    t = ops.GroupTable(64, [(abi.AGG_COUNT, U)])
    t.aggregate(col, key=key, log2_parts=3)
    with pytest.raises(ops.FQError) as ei:
        t.count()
    assert str(ei.value) == "Internal Error: Divide by zero error"
    with pytest.raises(ops.FQError):
        t.aggregate(col, key=key, log2_parts=9)


def test_sql_high_cardinality_group_by_takes_the_partitioned_path(eng):
    # 50,000 groups per partition: the engine's sample sees more groups than an
    # LDS table holds and launches the radix-partitioned kernels
    total = 2_400_000
    j0 = ops.jit_stats()["jit_launches"]
    r = eng.execute("SELECT number%%50000, count(number), max(number), sum(number) FROM system.numbers_mt(%d) "
                    "WHERE number%%3 < 2 GROUP BY number%%50000" % total)
    assert ops.jit_stats()["jit_launches"] - j0 >= 2 * 8  # gpart + bins per partition
    x = np.arange(total, dtype=np.uint64)
    x = x[x % np.uint64(3) < 2]
    exp = np_groupby(x % np.uint64(50000), [None, x, x], [abi.AGG_COUNT, abi.AGG_MAX, abi.AGG_SUM])
    assert len(r.rows) == len(exp)
    for k, cnt, mx, sm in r.rows:
        assert [cnt, mx, sm] == [int(v) for v in exp[k]]
    # keys only, every key distinct
    r = eng.execute("SELECT number FROM system.numbers_mt(400000) GROUP BY number")
    assert r.rows == [(i,) for i in range(400000)]


@pytest.mark.parametrize("chunk", [64 * 1001, 64 * 4096])
def test_sql_partitioned_group_by_in_chunks(chunk):
    # FQ_OPT_GROUP_CHUNK_ROWS: each partition's radix-partitioned launches go
    # over slices of the block; results equal the unchunked path (and numpy)
    from fq_amd._lib import FQError
    from fq_amd.engine import OPT_GROUP_CHUNK_ROWS, Engine
    total = 2_400_000
    sql = ("SELECT number%%50000, count(number), max(number), sum(number), min(number+7) "
           "FROM system.numbers_mt(%d) WHERE number%%3 < 2 GROUP BY number%%50000" % total)
    with Engine() as e:
        whole = e.execute(sql).rows
    with Engine() as e:
        e.set_option(OPT_GROUP_CHUNK_ROWS, chunk)
        j0 = ops.jit_stats()["jit_launches"]
        got = e.execute(sql).rows
        assert ops.jit_stats()["jit_launches"] - j0 >= 2 * 8 * 2  # gpart + bins, >= 2 chunks per partition
        with pytest.raises(FQError):
            e.set_option(OPT_GROUP_CHUNK_ROWS, 100)
    assert got == whole
    x = np.arange(total, dtype=np.uint64)
    x = x[x % np.uint64(3) < 2]
    exp = np_groupby(x % np.uint64(50000), [None, x, x, x + np.uint64(7)],
                     [abi.AGG_COUNT, abi.AGG_MAX, abi.AGG_SUM, abi.AGG_MIN])
    assert len(got) == len(exp)
    for k, *v in got:
        assert v == [int(t) for t in exp[k]]


@pytest.mark.parametrize("key_sql,key_steps,groups", [
    ("(number*7)%100003", [("*", 7), ("%", 100003)], 100003),  # hashed bins (64-bit magic key)
    ("number%65536", [("%", 65536)], 65536),                    # range bins (`& mask` form)
    ("(number/300)%5000", [("/", 300), ("%", 5000)], 5000),     # clustered runs, partitioned or LDS
])
def test_sql_group_by_matches_c_oracle_at_scale(eng, key_sql, key_steps, groups):
    # 4e7 rows through SQL (engine: sample -> LDS table or radix-partitioned
    # launches) against the C GROUP BY restatement (oracle/fq_oracle.c
    # fqo_numbers_group) over the same numbers_mt blocks
    import oracle_c
    total = 40_000_000
    r = eng.execute("SELECT %s, count(number), sum(number), max(number+1), min(number) FROM system.numbers_mt(%d) "
                    "WHERE number%%5 < 3 GROUP BY %s" % (key_sql, total, key_sql))
    key = chain(U, key_steps)[0]
    pred = predicate(U, [("%", 5)], "<", 3)
    aggs = [(abi.AGG_COUNT, U, None), (abi.AGG_SUM, U, None), (abi.AGG_MAX, U, chain(U, [("+", 1)])[0]),
            (abi.AGG_MIN, U, None)]
    keys, st = oracle_c.numbers_group(total, key, aggs, pred=pred, threads=8, cap_groups=2 * groups)
    o = np.argsort(keys)
    exp = [(int(k),) + tuple(int(x) for x in s) for k, s in zip(keys[o], st[o])]
    assert len(r.rows) == len(exp)
    assert [tuple(row) for row in r.rows] == exp


def test_table_merge_folds_exchanged_rows():
    # fq_group_table_merge (the cross-GPU GROUP BY final): three "ranks'"
    # extracted tables folded into one fresh table equal the group-by of all
    # rows; every kind and state type, repeated keys
    rng = np.random.default_rng(11)
    aggs = [(abi.AGG_COUNT, U), (abi.AGG_SUM, U), (abi.AGG_MAX, I), (abi.AGG_MIN, F), (abi.AGG_SUM, F)]
    parts = []
    for r in range(3):
        n = 200_000
        x = rng.integers(0, 1 << 62, n, dtype=np.uint64)
        col = ops.from_numpy(x)
        key, _ = chain(U, [("%", 5000)])
        vi, _ = chain(U, [("%", 1000), ("-", (500, "Int64"))])
        vf, _ = chain(U, [("%", 1000), ("*", 0.5)])
        t = ops.GroupTable(1 << 14, aggs)
        t.aggregate(col, key=key, values=[None, None, vi, vf, vf])
        parts.append((x, t.extract()))
    m = ops.GroupTable(1 << 14, aggs)
    for _, (k, st) in parts:
        m.merge(k, st)
    keys, states = m.extract()
    got = {int(k): [s[i] for s in decode(states, [d for _, d in aggs])] for i, k in enumerate(keys)}
    allx = np.concatenate([x for x, _ in parts])
    k = allx % np.uint64(5000)
    xi = (allx % np.uint64(1000)).astype(np.int64) - 500
    xf = (allx % np.uint64(1000)).astype(np.float64) * 0.5
    exp = np_groupby(k, [None, allx, xi, xf, xf], [a for a, _ in aggs])
    bound = {g: 1e-9 * abs(e[4]) + 1e-9 for g, e in exp.items()}
    compare(got, exp, [a for a, _ in aggs], [d for _, d in aggs], bound)
    # a table too small for the merged keys reports TABLE_FULL
    tiny = ops.GroupTable(64, aggs)
    tiny.merge(parts[0][1][0], parts[0][1][1])
    with pytest.raises(ops.FQError):
        tiny.count()


@pytest.mark.parametrize("log2p", [0, 4])
def test_aggregate_merge_aggregate_into_one_table(log2p):
    # fq_group_aggregate(_partitioned) and fq_group_table_merge into the SAME
    # table, in both orders: every key must reach its one slot (both inserts
    # start probing at the same home slot), so keys stay unique and the states
    # fold across the writers
    rng = np.random.default_rng(23)
    aggs = [(abi.AGG_COUNT, U), (abi.AGG_SUM, U), (abi.AGG_MAX, U)]
    key, _ = chain(U, [("%", 3000)])
    xs = [rng.integers(0, 1 << 62, 300_000, dtype=np.uint64) for _ in range(3)]
    src = ops.GroupTable(1 << 13, aggs)
    src.aggregate(ops.from_numpy(xs[1]), key=key, values=[None, None, None])
    mk, ms = src.extract()
    t = ops.GroupTable(1 << 13, aggs)
    t.aggregate(ops.from_numpy(xs[0]), key=key, values=[None, None, None], log2_parts=log2p)
    t.merge(mk, ms)
    t.aggregate(ops.from_numpy(xs[2]), key=key, values=[None, None, None], log2_parts=log2p)
    t.merge(mk, ms)  # and the merged rows once more, after the second aggregate
    keys, states = t.extract()
    assert len(np.unique(keys)) == len(keys) == 3000
    got = {int(k): [s[i] for s in decode(states, [d for _, d in aggs])] for i, k in enumerate(keys)}
    allx = np.concatenate([xs[0], xs[1], xs[2], xs[1]])
    exp = np_groupby(allx % np.uint64(3000), [None, allx, allx], [a for a, _ in aggs])
    compare(got, exp, [a for a, _ in aggs], [d for _, d in aggs])


@pytest.mark.parametrize("mod,log2p,pred", [(100_000, 6, False), (None, 8, False), (5000, 4, True)])
def test_narrow_partition_rows_match_wide(mod, log2p, pred):
    # FQ_GROUP_NARROW_ROWS (4-byte offsets from col[0] - 2^31 in the blocks):
    # the same table as the 8-byte rows over a numbers_mt-like block, with
    # range bins, hash bins and a predicate, first values near 2^40 (offsets
    # wrap through 0) and near 2^64 - 2^31 (the base wraps)
    for first in (2**40 - 1000, 2**64 - 2**31 + 77):
        n = 2_000_003
        col = ops.numbers_column(first, n)
        key = chain(U, [("%", mod)])[0] if mod else None
        p = predicate(U, [("%", 8)], "<", 3) if pred else None
        aggs = [(abi.AGG_COUNT, U), (abi.AGG_SUM, U), (abi.AGG_MAX, U), (abi.AGG_MIN, U)]
        res = []
        for narrow in (False, True):
            t = ops.GroupTable(4 * min(n, mod or n), aggs)
            t.aggregate(col, p, key, [None] * 4, log2_parts=log2p, narrow=narrow)
            keys, st = t.extract()
            o = np.argsort(keys, kind="stable")
            res.append((keys[o], [x[o] for x in st]))
        assert np.array_equal(res[0][0], res[1][0]) and len(res[0][0]) > 0
        for a in range(4):
            assert np.array_equal(res[0][1][a], res[1][1][a]), (first, a)


@pytest.mark.parametrize("mod,log2p", [(7, 4), (99_991, 5), (1_000_000, 8)])
def test_narrow_range_bin_key_from_row_offset(mod, log2p):
    # range bins over 4-byte rows compute `number % d` from the row's 32-bit
    # offset (fq_jit_gpart GP_MOD32): blocks starting below 2^31 (the offset
    # base would wrap, so the values themselves are the offsets), at 2^31 - 10
    # (crossing 2^31) and above 2^32, against numpy
    aggs = [(abi.AGG_COUNT, U), (abi.AGG_SUM, U), (abi.AGG_MAX, U)]
    for first in (0, 2**31 - 10, 2**33 + 5):
        n = 1_500_007
        x = np.arange(first, first + n, dtype=np.uint64)
        t = ops.GroupTable(4 * min(n, mod), aggs)
        t.aggregate(ops.numbers_column(first, n), None, chain(U, [("%", mod)])[0], [None] * 3,
                    log2_parts=log2p, narrow=True)
        keys, states = t.extract()
        got = {int(k): [s[i] for s in decode(states, [d for _, d in aggs])] for i, k in enumerate(keys)}
        exp = np_groupby(x % np.uint64(mod), [None, x, x], [a for a, _ in aggs])
        compare(got, exp, [a for a, _ in aggs], [d for _, d in aggs])


def test_narrow_partition_rows_refuse_values_out_of_range():
    # a value more than 2^31 from col[0]: reported, never aggregated wrongly
    x = np.arange(100_000, dtype=np.uint64)
    x[77_777] += np.uint64(2**33)
    col = ops.from_numpy(x)
    t = ops.GroupTable(1 << 18, [(abi.AGG_COUNT, U)])
    t.aggregate(col, None, chain(U, [("%", 1000)])[0], [None], log2_parts=4, narrow=True)
    with pytest.raises(ops.FQError, match="narrow rows"):
        t.count()


def test_table_merge_sentinel_key_and_empty_input():
    # the all-ones key (the table's EMPTY marker) has its own slot
    aggs = [(abi.AGG_COUNT, U), (abi.AGG_MAX, U)]
    m = ops.GroupTable(64, aggs)
    E1 = 0xFFFFFFFFFFFFFFFF
    m.merge(np.array([E1, 7, E1], dtype=np.uint64), [np.array([2, 1, 3], dtype=np.uint64),
                                                     np.array([10, 4, 30], dtype=np.uint64)])
    m.merge(np.array([], dtype=np.uint64), [np.array([], dtype=np.uint64)] * 2)
    keys, states = m.extract()
    got = {int(k): [int(states[0][i]), int(states[1][i])] for i, k in enumerate(keys)}
    assert got == {E1: [5, 30], 7: [1, 4]}
