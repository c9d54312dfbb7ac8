/*
 * fq_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 * See fq_oracle.h for what it restates and why its structure is kept slow on
 * purpose.  Every function cites the reference file:line it follows.
 */
#define _GNU_SOURCE
#include "fq_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define BLOCK_SIZE 10000 /* numbers_stream.rs:29 */

/* ------------------------------------------------------------------ */
/* numbers_mt partitioning                                              */
/* ------------------------------------------------------------------ */

/* NumbersTable::generate_parts (numbers_table.rs:29-55) */
int32_t fqo_num_partitions(uint64_t total) { return total / 8 == 0 ? 1 : 8; }

void fqo_partition_range(uint64_t total, int32_t p, uint64_t *begin, uint64_t *end) {
    const uint64_t workers = 8, chunk = total / workers;
    if (chunk == 0) {
        *begin = 0;
        *end = total - 1; /* total == 0 wraps in release: unsupported, see DESIGN.md */
        return;
    }
    *begin = (uint64_t)p * chunk;
    *end = ((uint64_t)p + 1) * chunk - 1;
    if (p == (int32_t)workers - 1) *end += total % workers;
}

/* NumbersStream::create (numbers_stream.rs:27-62): the partition's block list.
 * Calls fn(begin, end_inclusive) for every block in order. */
typedef int (*block_fn)(void *ctx, uint64_t b, uint64_t e);
static int numbers_blocks(uint64_t begin, uint64_t end, block_fn fn, void *ctx) {
    const uint64_t count = end - begin + 1;
    const uint64_t nblocks = count / BLOCK_SIZE, remain = count % BLOCK_SIZE;
    if (nblocks > 0) {
        for (uint64_t i = 0; i < nblocks; ++i) {
            const uint64_t bb = begin + BLOCK_SIZE * i;
            uint64_t be = begin + BLOCK_SIZE * (i + 1) - 1;
            if (i == nblocks - 1 && remain > 0) be = bb + remain; /* the quirk: rows dropped */
            int rc = fn(ctx, bb, be);
            if (rc) return rc;
        }
        return 0;
    }
    return fn(ctx, begin, end);
}

static int count_rows_fn(void *ctx, uint64_t b, uint64_t e) {
    *(uint64_t *)ctx += e - b + 1;
    return 0;
}

uint64_t fqo_partition_rows(uint64_t total, int32_t p) {
    uint64_t b, e, rows = 0;
    fqo_partition_range(total, p, &b, &e);
    numbers_blocks(b, e, count_rows_fn, &rows);
    return rows;
}

uint64_t fqo_splitmix64(uint64_t seed, uint64_t i) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* ------------------------------------------------------------------ */
/* arrays (arrow PrimitiveArray restated as bits + dtype)               */
/* ------------------------------------------------------------------ */
typedef struct {
    uint64_t *v;
    int64_t n;
    int32_t dtype;
} arr_t;

typedef struct {
    int status; /* fq_status */
    char msg[256];
} err_t;

static int set_err(err_t *e, int st, const char *m) {
    if (!e->status) {
        e->status = st;
        snprintf(e->msg, sizeof(e->msg), "%s", m);
    }
    return st;
}

static double as_f(uint64_t b) {
    double d;
    memcpy(&d, &b, 8);
    return d;
}
static uint64_t of_f(double d) {
    uint64_t b;
    memcpy(&b, &d, 8);
    return b;
}

static arr_t arr_new(int64_t n, int32_t dt) {
    arr_t a;
    a.v = (uint64_t *)malloc((size_t)(n > 0 ? n : 1) * 8);
    a.n = n;
    a.dtype = dt;
    return a;
}
static void arr_free(arr_t *a) {
    free(a->v);
    a->v = NULL;
}

/* arrow::compute::cast between the 64-bit types (num-traits NumCast); a value
 * that does not fit becomes null in the reference.  Nulls are outside this
 * restatement's scope: reported as FQ_E_UNSUPPORTED "cast produced nulls"
 * (the device path reports the same; documented in DESIGN.md). */
static int cast_arr(const arr_t *in, int32_t to, arr_t *out, err_t *err) {
    *out = arr_new(in->n, to);
    for (int64_t i = 0; i < in->n; ++i) {
        const uint64_t x = in->v[i];
        if (in->dtype == to) {
            out->v[i] = x;
        } else if (to == FQ_DT_FLOAT64) {
            out->v[i] = of_f(in->dtype == FQ_DT_INT64 ? (double)(int64_t)x : (double)x);
        } else if (in->dtype == FQ_DT_UINT64 && to == FQ_DT_INT64) {
            if (x >> 63) return set_err(err, FQ_E_UNSUPPORTED, "cast produced nulls");
            out->v[i] = x;
        } else {
            return set_err(err, FQ_E_UNSUPPORTED, "cast not covered by the oracle");
        }
    }
    return 0;
}

/* DataValue::to_array(size): materialised constant broadcast (data_value.rs:77-111) */
static arr_t broadcast(uint64_t bits, int32_t dt, int64_t n) {
    arr_t a = arr_new(n, dt);
    for (int64_t i = 0; i < n; ++i) a.v[i] = bits;
    return a;
}

/* arrow add/subtract/multiply/divide (+ '%' extension) on same-typed arrays
 * (data_array_arithmetic.rs:42-54).  Release build: integer wrap.  Divide
 * checks every divisor first and fails with DivideByZero. */
static int arith_arr(int32_t op, const arr_t *l, const arr_t *r, arr_t *out, err_t *err) {
    const int32_t dt = l->dtype;
    const int64_t n = l->n;
    if (op == FQ_OP_DIV || op == FQ_OP_MOD) {
        for (int64_t i = 0; i < n; ++i) {
            const int zero = dt == FQ_DT_FLOAT64 ? as_f(r->v[i]) == 0.0 : r->v[i] == 0;
            if (zero) return set_err(err, FQ_E_DIVIDE_BY_ZERO, "Internal Error: Divide by zero error");
        }
    }
    *out = arr_new(n, dt);
    for (int64_t i = 0; i < n; ++i) {
        const uint64_t a = l->v[i], b = r->v[i];
        uint64_t z = 0;
        if (dt == FQ_DT_FLOAT64) {
            const double fa = as_f(a), fb = as_f(b);
            double fz = 0;
            switch (op) {
                case FQ_OP_ADD: fz = fa + fb; break;
                case FQ_OP_SUB: fz = fa - fb; break;
                case FQ_OP_MUL: fz = fa * fb; break;
                case FQ_OP_DIV: fz = fa / fb; break;
                default: fz = fmod(fa, fb); break;
            }
            z = of_f(fz);
        } else if (dt == FQ_DT_INT64) {
            const int64_t sa = (int64_t)a, sb = (int64_t)b;
            switch (op) {
                case FQ_OP_ADD: z = a + b; break;
                case FQ_OP_SUB: z = a - b; break;
                case FQ_OP_MUL: z = a * b; break;
                case FQ_OP_DIV: z = sb == -1 ? (uint64_t)0 - a : (uint64_t)(sa / sb); break;
                default: z = sb == -1 ? 0 : (uint64_t)(sa % sb); break;
            }
        } else {
            switch (op) {
                case FQ_OP_ADD: z = a + b; break;
                case FQ_OP_SUB: z = a - b; break;
                case FQ_OP_MUL: z = a * b; break;
                case FQ_OP_DIV: z = a / b; break;
                default: z = a % b; break;
            }
        }
        out->v[i] = z;
    }
    return 0;
}

/* operand of a step: constant broadcast or the block's column cast to dtype */
static int operand_arr(int32_t operand, uint64_t bits, int32_t dt, const arr_t *x, arr_t *out, err_t *err) {
    if (operand == FQ_OPERAND_CONST) {
        *out = broadcast(bits, dt, x->n);
        return 0;
    }
    return cast_arr(x, dt, out, err);
}

/* Function::eval of an ArithmeticFunction chain (function_arithmetic.rs:64-72):
 * each level evaluates its children to arrays, casts both to the coercion
 * type (data_array_arithmetic.rs:34-40) and runs one arrow kernel. */
/* Expression trees (FQ_OP_PUSH / FQ_OPERAND_STACK): a pushed array is the
 * evaluated left child of a node whose right child is evaluated next; the
 * node casts both to its coercion type (the left one first, as the
 * reference evaluates left_->eval before right_->eval). */
static int eval_chain(const fq_expr *e, const arr_t *x, arr_t *out, err_t *err) {
    arr_t acc = arr_new(x->n, x->dtype);
    memcpy(acc.v, x->v, (size_t)x->n * 8);
    arr_t stack[FQ_MAX_STACK];
    int depth = 0;
    for (int s = 0; s < e->n_steps; ++s) {
        const fq_step *st = &e->steps[s];
        arr_t accc, opnd, res;
        if (st->op == FQ_OP_PUSH) {
            if (depth >= FQ_MAX_STACK) {
                arr_free(&acc);
                while (depth > 0) arr_free(&stack[--depth]);
                return set_err(err, FQ_E_UNSUPPORTED, "expression tree too deep");
            }
            stack[depth++] = acc;
            acc = arr_new(x->n, x->dtype);
            memcpy(acc.v, x->v, (size_t)x->n * 8);
            continue;
        }
        if (st->operand == FQ_OPERAND_STACK) {
            arr_t left = stack[--depth];
            int rc = cast_arr(&left, st->dtype, &opnd, err);
            arr_free(&left);
            if (rc) {
                arr_free(&acc);
                while (depth > 0) arr_free(&stack[--depth]);
                return err->status;
            }
            if (cast_arr(&acc, st->dtype, &accc, err)) {
                arr_free(&acc);
                arr_free(&opnd);
                while (depth > 0) arr_free(&stack[--depth]);
                return err->status;
            }
            arr_free(&acc);
            rc = st->reversed ? arith_arr(st->op, &opnd, &accc, &res, err) : arith_arr(st->op, &accc, &opnd, &res, err);
            arr_free(&accc);
            arr_free(&opnd);
            if (rc) {
                while (depth > 0) arr_free(&stack[--depth]);
                return rc;
            }
            acc = res;
            continue;
        }
        if (cast_arr(&acc, st->dtype, &accc, err)) {
            arr_free(&acc);
            while (depth > 0) arr_free(&stack[--depth]);
            return err->status;
        }
        arr_free(&acc);
        if (operand_arr(st->operand, st->bits, st->dtype, x, &opnd, err)) {
            arr_free(&accc);
            while (depth > 0) arr_free(&stack[--depth]);
            return err->status;
        }
        int rc = st->reversed ? arith_arr(st->op, &opnd, &accc, &res, err) : arith_arr(st->op, &accc, &opnd, &res, err);
        arr_free(&accc);
        arr_free(&opnd);
        if (rc) {
            while (depth > 0) arr_free(&stack[--depth]);
            return rc;
        }
        acc = res;
    }
    *out = acc;
    return 0;
}

static int cmp1(int32_t cmp, int32_t dt, uint64_t a, uint64_t b) {
    if (dt == FQ_DT_FLOAT64) {
        const double x = as_f(a), y = as_f(b);
        switch (cmp) {
            case FQ_CMP_EQ: return x == y;
            case FQ_CMP_LT: return x < y;
            case FQ_CMP_LTEQ: return x <= y;
            case FQ_CMP_GT: return x > y;
            default: return x >= y;
        }
    }
    if (dt == FQ_DT_INT64) {
        const int64_t x = (int64_t)a, y = (int64_t)b;
        switch (cmp) {
            case FQ_CMP_EQ: return x == y;
            case FQ_CMP_LT: return x < y;
            case FQ_CMP_LTEQ: return x <= y;
            case FQ_CMP_GT: return x > y;
            default: return x >= y;
        }
    }
    switch (cmp) {
        case FQ_CMP_EQ: return a == b;
        case FQ_CMP_LT: return a < b;
        case FQ_CMP_LTEQ: return a <= b;
        case FQ_CMP_GT: return a > b;
        default: return a >= b;
    }
}

/* FilterTransform::expression_executor (transform_filter.rs:38-55): evaluate
 * the ComparisonFunction to a BooleanArray, then filter_record_batch. */
static int filter_block(const fq_pred *p, const arr_t *x, arr_t *out, err_t *err) {
    arr_t l, lc, r;
    if (eval_chain(&p->lhs, x, &l, err)) return err->status;
    if (cast_arr(&l, p->cmp_dtype, &lc, err)) {
        arr_free(&l);
        return err->status;
    }
    arr_free(&l);
    if (operand_arr(p->rhs_operand, p->rhs_bits, p->cmp_dtype, x, &r, err)) {
        arr_free(&lc);
        return err->status;
    }
    unsigned char *mask = (unsigned char *)malloc((size_t)(x->n > 0 ? x->n : 1));
    for (int64_t i = 0; i < x->n; ++i) mask[i] = (unsigned char)cmp1(p->cmp, p->cmp_dtype, lc.v[i], r.v[i]);
    arr_free(&lc);
    arr_free(&r);
    int64_t k = 0;
    for (int64_t i = 0; i < x->n; ++i) k += mask[i];
    *out = arr_new(k, x->dtype);
    k = 0;
    for (int64_t i = 0; i < x->n; ++i)
        if (mask[i]) out->v[k++] = x->v[i];
    free(mask);
    return 0;
}

/* ------------------------------------------------------------------ */
/* DataValue state machine                                              */
/* ------------------------------------------------------------------ */

/* data_value_arithmetic_op(Add, state, delta) (data_value_arithmetic.rs:10-27):
 * Null absorbs; otherwise both sides go through to_array(1), which fails on
 * X(None) with "DataValue to array cannot be NONE NULL". */
static int state_add(fqo_state *s, fqo_state d, err_t *err) {
    if (s->kind == FQO_NULL) {
        *s = d;
        return 0;
    }
    if (d.kind == FQO_NULL) return 0;
    if (s->kind == FQO_NONE || d.kind == FQO_NONE)
        return set_err(err, FQ_E_INTERNAL, "Internal Error: DataValue to array cannot be NONE NULL");
    if (s->dtype == FQ_DT_FLOAT64) s->bits = of_f(as_f(s->bits) + as_f(d.bits));
    else s->bits = s->bits + d.bits; /* release-build wrap */
    return 0;
}

/* data_value_aggregate_op(Min|Max, state, delta) (data_value_aggregate.rs:8-101 +
 * typed_data_value_min_max, macros.rs:179-188): None-aware, uses Ord/f64::min. */
static void state_minmax(fqo_state *s, fqo_state d, int is_max) {
    if (s->kind == FQO_NULL) {
        *s = d;
        return;
    }
    if (d.kind == FQO_NULL || d.kind == FQO_NONE) return;
    if (s->kind == FQO_NONE) {
        *s = d;
        return;
    }
    const uint64_t a = s->bits, b = d.bits;
    int take_b;
    if (s->dtype == FQ_DT_FLOAT64) {
        const double x = as_f(a), y = as_f(b);
        if (x != x) take_b = 1;       /* f64::max/min ignore NaN */
        else if (y != y) take_b = 0;
        else take_b = is_max ? y > x : y < x;
    } else if (s->dtype == FQ_DT_INT64) {
        take_b = is_max ? (int64_t)b > (int64_t)a : (int64_t)b < (int64_t)a;
    } else {
        take_b = is_max ? b > a : b < a;
    }
    if (take_b) s->bits = b;
}

/* data_array_aggregate_op (data_array_aggregate.rs:14-163) over one block. */
static fqo_state block_agg(int32_t op, const arr_t *v) {
    fqo_state r;
    r.dtype = v->dtype;
    r.bits = 0;
    if (v->n == 0) { /* arrow returns None when null_count == len */
        r.kind = FQO_NONE;
        return r;
    }
    r.kind = FQO_SOME;
    if (op == FQ_AGG_SUM) {
        if (v->dtype == FQ_DT_FLOAT64) {
            double s = 0;
            for (int64_t i = 0; i < v->n; ++i) s += as_f(v->v[i]);
            r.bits = of_f(s);
        } else {
            uint64_t s = 0;
            for (int64_t i = 0; i < v->n; ++i) s += v->v[i];
            r.bits = s;
        }
        return r;
    }
    /* min_max_helper: n = fold(m[0], |n, item| if cmp(n, item) {item} else {n}) */
    uint64_t n = v->v[0];
    for (int64_t i = 1; i < v->n; ++i) {
        const uint64_t it = v->v[i];
        int take;
        if (v->dtype == FQ_DT_FLOAT64) take = op == FQ_AGG_MAX ? as_f(n) < as_f(it) : as_f(n) > as_f(it);
        else if (v->dtype == FQ_DT_INT64) take = op == FQ_AGG_MAX ? (int64_t)n < (int64_t)it : (int64_t)n > (int64_t)it;
        else take = op == FQ_AGG_MAX ? n < it : n > it;
        if (take) n = it;
    }
    r.bits = n;
    return r;
}

/* ------------------------------------------------------------------ */
/* AggregatePartialTransform over one block stream                      */
/* ------------------------------------------------------------------ */
typedef struct {
    int32_t src, col_dtype;
    uint64_t seed;
    const void *host_col; /* for fqo_column_partial */
    const fq_pred *pred;
    int32_t n_aggs;
    const int32_t *agg_ops;
    const fq_expr *agg_args;
    fqo_state *states; /* [n_aggs] */
    err_t err;
} task_t;

/* one block: materialise (numbers_stream.rs:76), filter, accumulate every func */
static int process_block(task_t *t, const arr_t *blk) {
    arr_t filtered;
    const arr_t *x = blk;
    if (t->pred && t->pred->kind == FQ_PRED_EXPR) {
        if (filter_block(t->pred, blk, &filtered, &t->err)) return t->err.status;
        x = &filtered;
    }
    for (int a = 0; a < t->n_aggs; ++a) {
        arr_t val;
        /* AggregatorFunction::accumulate: val = arg.eval(block) for every op */
        if (eval_chain(&t->agg_args[a], x, &val, &t->err)) break;
        const int32_t op = t->agg_ops[a];
        if (op == FQ_AGG_COUNT) {
            fqo_state d = {FQO_SOME, FQ_DT_UINT64, (uint64_t)x->n};
            state_add(&t->states[a], d, &t->err);
        } else if (op == FQ_AGG_SUM) {
            state_add(&t->states[a], block_agg(op, &val), &t->err);
        } else {
            state_minmax(&t->states[a], block_agg(op, &val), op == FQ_AGG_MAX);
        }
        arr_free(&val);
        if (t->err.status) break;
    }
    if (x == &filtered) arr_free(&filtered);
    return t->err.status;
}

static int numbers_block_fn(void *ctx, uint64_t b, uint64_t e) {
    task_t *t = (task_t *)ctx;
    arr_t blk = arr_new((int64_t)(e - b + 1), FQ_DT_UINT64);
    for (uint64_t i = b; i <= e; ++i)
        blk.v[i - b] = t->src == FQO_SRC_SPLITMIX ? fqo_splitmix64(t->seed, i) : i;
    int rc = process_block(t, &blk);
    arr_free(&blk);
    return rc;
}

typedef struct {
    task_t task;
    uint64_t total;
    int32_t part;
} part_job_t;

static void *part_thread(void *arg) {
    part_job_t *j = (part_job_t *)arg;
    uint64_t b, e;
    fqo_partition_range(j->total, j->part, &b, &e);
    numbers_blocks(b, e, numbers_block_fn, &j->task);
    return NULL;
}

static void init_states(fqo_state *s, int n) {
    for (int i = 0; i < n; ++i) {
        s[i].kind = FQO_NULL;
        s[i].dtype = FQ_DT_NULL;
        s[i].bits = 0;
    }
}

int32_t fqo_numbers_partial(uint64_t total, int32_t src, uint64_t seed, int32_t p0, int32_t p1,
                            const fq_pred *pred, int32_t n_aggs, const int32_t *agg_ops,
                            const fq_expr *agg_args, int32_t n_threads, fqo_state *out_states,
                            int32_t *part_status, char *errbuf, int32_t errlen) {
    const int32_t np = p1 - p0;
    if (np <= 0) return 0;
    part_job_t *jobs = (part_job_t *)calloc((size_t)np, sizeof(part_job_t));
    for (int32_t i = 0; i < np; ++i) {
        jobs[i].total = total;
        jobs[i].part = p0 + i;
        jobs[i].task.src = src;
        jobs[i].task.col_dtype = FQ_DT_UINT64;
        jobs[i].task.seed = seed;
        jobs[i].task.pred = pred;
        jobs[i].task.n_aggs = n_aggs;
        jobs[i].task.agg_ops = agg_ops;
        jobs[i].task.agg_args = agg_args;
        jobs[i].task.states = out_states + (size_t)i * n_aggs;
        init_states(jobs[i].task.states, n_aggs);
    }
    if (n_threads <= 0 || n_threads > np) n_threads = np;
    /* waves of n_threads threads, partition order (one tokio task per source) */
    pthread_t *th = (pthread_t *)calloc((size_t)n_threads, sizeof(pthread_t));
    for (int32_t w = 0; w < np; w += n_threads) {
        const int32_t k = (np - w) < n_threads ? (np - w) : n_threads;
        for (int32_t i = 0; i < k; ++i) pthread_create(&th[i], NULL, part_thread, &jobs[w + i]);
        for (int32_t i = 0; i < k; ++i) pthread_join(th[i], NULL);
    }
    free(th);
    int32_t rc = 0;
    for (int32_t i = 0; i < np; ++i) {
        part_status[i] = jobs[i].task.err.status;
        if (jobs[i].task.err.status && !rc) {
            rc = jobs[i].task.err.status;
            if (errbuf && errlen > 0) snprintf(errbuf, (size_t)errlen, "%s", jobs[i].task.err.msg);
        }
    }
    free(jobs);
    return rc;
}

/* The same work cut finer than the reference can (BASELINE.md 2's all-cores
 * leg): generate_parts always makes 8 partitions (numbers_table.rs:29-55), so
 * the reference never runs more than 8 tasks.  Here every partition's block
 * list is cut into `slices` runs of whole blocks, each its own task with its
 * own partial states (out_states: [8 * slices][n_aggs], partition-major), run
 * in waves of n_threads; AggregateFinal's merge of the rows gives the
 * reference's result (sums add, min/max and counts commute). */
typedef struct {
    block_fn fn;
    void *ctx;
    uint64_t idx, lo, hi;
} window_t;

static int window_fn(void *c, uint64_t b, uint64_t e) {
    window_t *w = (window_t *)c;
    int rc = 0;
    if (w->idx >= w->lo && w->idx < w->hi) rc = w->fn(w->ctx, b, e);
    w->idx++;
    return rc;
}

typedef struct {
    task_t task;
    uint64_t total;
    int32_t part, slice, slices;
} slice_job_t;

static int count_blocks_fn(void *ctx, uint64_t b, uint64_t e) {
    (void)b;
    (void)e;
    ++*(uint64_t *)ctx;
    return 0;
}

static void *slice_thread(void *arg) {
    slice_job_t *j = (slice_job_t *)arg;
    uint64_t b, e, nb = 0;
    fqo_partition_range(j->total, j->part, &b, &e);
    numbers_blocks(b, e, count_blocks_fn, &nb);
    window_t w = {numbers_block_fn, &j->task, 0, nb * (uint64_t)j->slice / (uint64_t)j->slices,
                  nb * (uint64_t)(j->slice + 1) / (uint64_t)j->slices};
    numbers_blocks(b, e, window_fn, &w);
    return NULL;
}

int32_t fqo_numbers_partial_split(uint64_t total, const fq_pred *pred, int32_t n_aggs, const int32_t *agg_ops,
                                  const fq_expr *agg_args, int32_t n_threads, int32_t slices,
                                  fqo_state *out_states, char *errbuf, int32_t errlen) {
    const int32_t np = fqo_num_partitions(total);
    if (np <= 0 || slices < 1) return 0;
    const int32_t nj = np * slices;
    slice_job_t *jobs = (slice_job_t *)calloc((size_t)nj, sizeof(slice_job_t));
    for (int32_t i = 0; i < nj; ++i) {
        jobs[i].total = total;
        jobs[i].part = i / slices;
        jobs[i].slice = i % slices;
        jobs[i].slices = slices;
        jobs[i].task.src = FQO_SRC_NUMBERS;
        jobs[i].task.col_dtype = FQ_DT_UINT64;
        jobs[i].task.pred = pred;
        jobs[i].task.n_aggs = n_aggs;
        jobs[i].task.agg_ops = agg_ops;
        jobs[i].task.agg_args = agg_args;
        jobs[i].task.states = out_states + (size_t)i * n_aggs;
        init_states(jobs[i].task.states, n_aggs);
    }
    if (n_threads <= 0 || n_threads > nj) n_threads = nj;
    pthread_t *th = (pthread_t *)calloc((size_t)n_threads, sizeof(pthread_t));
    for (int32_t w = 0; w < nj; w += n_threads) {
        const int32_t k = (nj - w) < n_threads ? (nj - w) : n_threads;
        for (int32_t i = 0; i < k; ++i) pthread_create(&th[i], NULL, slice_thread, &jobs[w + i]);
        for (int32_t i = 0; i < k; ++i) pthread_join(th[i], NULL);
    }
    free(th);
    int32_t rc = 0;
    for (int32_t i = 0; i < nj && !rc; ++i)
        if (jobs[i].task.err.status) {
            rc = jobs[i].task.err.status;
            if (errbuf && errlen > 0) snprintf(errbuf, (size_t)errlen, "%s", jobs[i].task.err.msg);
        }
    free(jobs);
    return rc;
}

int32_t fqo_column_partial(const void *col, int32_t col_dtype, int64_t len, int64_t block_rows,
                           const fq_pred *pred, int32_t n_aggs, const int32_t *agg_ops,
                           const fq_expr *agg_args, fqo_state *out_states, char *errbuf,
                           int32_t errlen) {
    task_t t;
    memset(&t, 0, sizeof(t));
    t.col_dtype = col_dtype;
    t.host_col = col;
    t.pred = pred;
    t.n_aggs = n_aggs;
    t.agg_ops = agg_ops;
    t.agg_args = agg_args;
    t.states = out_states;
    init_states(out_states, n_aggs);
    if (block_rows <= 0) block_rows = len > 0 ? len : 1;
    const uint64_t *c = (const uint64_t *)col;
    for (int64_t s = 0; s < len; s += block_rows) {
        const int64_t n = (s + block_rows < len) ? block_rows : len - s;
        arr_t blk = arr_new(n, col_dtype);
        memcpy(blk.v, c + s, (size_t)n * 8);
        const int rc = process_block(&t, &blk);
        arr_free(&blk);
        if (rc) break;
    }
    if (t.err.status && errbuf && errlen > 0) snprintf(errbuf, (size_t)errlen, "%s", t.err.msg);
    return t.err.status;
}

/* ------------------------------------------------------------------ */
/* GROUP BY (no reference transform: plan_parser.rs:284-308 plans       */
/* group_expr, pipeline_builder.rs:50-66 ignores it).  The semantics are */
/* the ungrouped path's per group (fq_ref.py group_by_query states them); */
/* here a plain CPU hash aggregation over the same 10,000-row blocks:     */
/* per block materialise, filter, key = key.eval(block), every argument   */
/* .eval(block), then one open-addressing table insert per row; one      */
/* table per partition thread, merged after the join.  CPU baseline of    */
/* the device GROUP BY (bench.py --query g1/g2) and a large-N checker.   */
/* ------------------------------------------------------------------ */
#define GEMPTY 0xffffffffffffffffull
typedef struct {
    uint64_t *keys;   /* cap slots, GEMPTY = free */
    uint64_t *st;     /* cap * n_aggs state bits */
    uint64_t *cnt;    /* rows per group (COUNT states and "seen") */
    uint64_t cap, used;
    int has_empty_key; /* the GEMPTY key itself, kept aside */
    uint64_t empty_cnt, *empty_st;
} gtab_t;

static uint64_t gmix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static uint64_t gident(int32_t op, int32_t dt) {
    if (op == FQ_AGG_COUNT || op == FQ_AGG_SUM) return 0;
    if (dt == FQ_DT_FLOAT64) return op == FQ_AGG_MAX ? 0xfff0000000000000ull : 0x7ff0000000000000ull;
    if (dt == FQ_DT_INT64) return op == FQ_AGG_MAX ? 0x8000000000000000ull : 0x7fffffffffffffffull;
    return op == FQ_AGG_MAX ? 0ull : ~0ull;
}

static void gupdate(uint64_t *s, int32_t op, int32_t dt, uint64_t v) {
    if (op == FQ_AGG_SUM) {
        *s = dt == FQ_DT_FLOAT64 ? of_f(as_f(*s) + as_f(v)) : *s + v; /* u64/i64 wrap (macros.rs:174) */
    } else if (op == FQ_AGG_MAX || op == FQ_AGG_MIN) {
        const int mx = op == FQ_AGG_MAX;
        int take;
        if (dt == FQ_DT_FLOAT64) take = mx ? as_f(v) > as_f(*s) : as_f(v) < as_f(*s);
        else if (dt == FQ_DT_INT64) take = mx ? (int64_t)v > (int64_t)*s : (int64_t)v < (int64_t)*s;
        else take = mx ? v > *s : v < *s;
        if (take) *s = v;
    }
}

static int gtab_init(gtab_t *t, uint64_t cap, int32_t n_aggs) {
    memset(t, 0, sizeof(*t));
    uint64_t c = 1024;
    while (c < cap) c <<= 1;
    t->cap = c;
    t->keys = (uint64_t *)malloc(c * 8);
    t->st = (uint64_t *)malloc(c * 8 * (size_t)(n_aggs > 0 ? n_aggs : 1));
    t->cnt = (uint64_t *)calloc(c, 8);
    t->empty_st = (uint64_t *)malloc(8 * (size_t)(n_aggs > 0 ? n_aggs : 1));
    if (!t->keys || !t->st || !t->cnt || !t->empty_st) return -1;
    memset(t->keys, 0xff, c * 8);
    return 0;
}

static void gtab_free(gtab_t *t) {
    free(t->keys);
    free(t->st);
    free(t->cnt);
    free(t->empty_st);
}

/* slot of key k (claimed if new); NULL when the table is full */
static uint64_t *gtab_slot(gtab_t *t, uint64_t k, int32_t n_aggs, const int32_t *ops, const int32_t *dts,
                           uint64_t **cnt) {
    if (k == GEMPTY) {
        if (!t->has_empty_key) {
            t->has_empty_key = 1;
            for (int a = 0; a < n_aggs; ++a) t->empty_st[a] = gident(ops[a], dts[a]);
        }
        *cnt = &t->empty_cnt;
        return t->empty_st;
    }
    uint64_t h = gmix(k) & (t->cap - 1);
    for (uint64_t p = 0; p < t->cap; ++p) {
        if (t->keys[h] == k) break;
        if (t->keys[h] == GEMPTY) {
            if ((t->used + 1) * 4 > t->cap * 3) return NULL;
            t->keys[h] = k;
            t->used++;
            for (int a = 0; a < n_aggs; ++a) t->st[h * (uint64_t)n_aggs + (uint64_t)a] = gident(ops[a], dts[a]);
            break;
        }
        h = (h + 1) & (t->cap - 1);
    }
    *cnt = &t->cnt[h];
    return &t->st[h * (uint64_t)n_aggs];
}

typedef struct {
    uint64_t total;
    int32_t part, src, n_aggs;
    uint64_t seed;
    const fq_pred *pred;
    const fq_expr *key;
    const int32_t *ops, *dts;
    const fq_expr *args;
    gtab_t tab;
    err_t err;
} gjob_t;

static int group_block_fn(void *ctx, uint64_t b, uint64_t e) {
    gjob_t *j = (gjob_t *)ctx;
    arr_t blk = arr_new((int64_t)(e - b + 1), FQ_DT_UINT64), filtered, key;
    arr_t vals[FQ_MAX_GROUP_AGGS];
    key.v = NULL;
    for (int a = 0; a < FQ_MAX_GROUP_AGGS; ++a) vals[a].v = NULL;
    for (uint64_t i = b; i <= e; ++i) blk.v[i - b] = j->src == FQO_SRC_SPLITMIX ? fqo_splitmix64(j->seed, i) : i;
    const arr_t *x = &blk;
    int rc = 0;
    if (j->pred && j->pred->kind == FQ_PRED_EXPR) {
        if (filter_block(j->pred, &blk, &filtered, &j->err)) rc = j->err.status;
        else x = &filtered;
    }
    if (!rc && eval_chain(j->key, x, &key, &j->err)) rc = j->err.status;
    for (int a = 0; !rc && a < j->n_aggs; ++a)
        if (eval_chain(&j->args[a], x, &vals[a], &j->err)) rc = j->err.status;
    for (int64_t i = 0; !rc && i < x->n; ++i) {
        uint64_t *cnt;
        uint64_t *s = gtab_slot(&j->tab, key.v[i], j->n_aggs, j->ops, j->dts, &cnt);
        if (!s) {
            rc = set_err(&j->err, FQ_E_TABLE_FULL, "GROUP BY: CPU table full");
            break;
        }
        *cnt += 1;
        for (int a = 0; a < j->n_aggs; ++a)
            if (j->ops[a] == FQ_AGG_COUNT) s[a] += 1;
            else gupdate(&s[a], j->ops[a], j->dts[a], vals[a].v[i]);
    }
    for (int a = 0; a < FQ_MAX_GROUP_AGGS; ++a)
        if (vals[a].v) arr_free(&vals[a]);
    if (key.v) arr_free(&key);
    if (x == &filtered) arr_free(&filtered);
    arr_free(&blk);
    return rc;
}

static void *group_thread(void *arg) {
    gjob_t *j = (gjob_t *)arg;
    uint64_t b, e;
    fqo_partition_range(j->total, j->part, &b, &e);
    numbers_blocks(b, e, group_block_fn, j);
    return NULL;
}

int32_t fqo_numbers_group(uint64_t total, int32_t src, uint64_t seed, const fq_pred *pred, const fq_expr *key,
                          int32_t n_aggs, const int32_t *agg_ops, const int32_t *agg_dtypes, const fq_expr *agg_args,
                          int32_t n_threads, uint64_t cap_groups, uint64_t *out_keys, uint64_t *out_states,
                          uint64_t *out_groups, char *errbuf, int32_t errlen) {
    const int32_t np = fqo_num_partitions(total);
    *out_groups = 0;
    if (n_aggs < 1 || n_aggs > FQ_MAX_GROUP_AGGS) return FQ_E_INVALID;
    gjob_t *jobs = (gjob_t *)calloc((size_t)np, sizeof(gjob_t));
    int32_t rc = 0;
    for (int32_t i = 0; i < np && !rc; ++i) {
        jobs[i].total = total;
        jobs[i].part = i;
        jobs[i].src = src;
        jobs[i].seed = seed;
        jobs[i].pred = pred;
        jobs[i].key = key;
        jobs[i].n_aggs = n_aggs;
        jobs[i].ops = agg_ops;
        jobs[i].dts = agg_dtypes;
        jobs[i].args = agg_args;
        if (gtab_init(&jobs[i].tab, cap_groups * 2, n_aggs)) rc = FQ_E_INTERNAL;
    }
    if (n_threads <= 0 || n_threads > np) n_threads = np;
    pthread_t *th = (pthread_t *)calloc((size_t)n_threads, sizeof(pthread_t));
    for (int32_t w = 0; !rc && w < np; w += n_threads) {
        const int32_t k = (np - w) < n_threads ? (np - w) : n_threads;
        for (int32_t i = 0; i < k; ++i) pthread_create(&th[i], NULL, group_thread, &jobs[w + i]);
        for (int32_t i = 0; i < k; ++i) pthread_join(th[i], NULL);
    }
    free(th);
    for (int32_t i = 0; i < np && !rc; ++i)
        if (jobs[i].err.status) {
            rc = jobs[i].err.status;
            if (errbuf && errlen > 0) snprintf(errbuf, (size_t)errlen, "%s", jobs[i].err.msg);
        }
    /* merge the partition tables in partition order into table 0 */
    for (int32_t i = 1; i < np && !rc; ++i) {
        gtab_t *t = &jobs[i].tab;
        for (uint64_t h = 0; h <= t->cap && !rc; ++h) {
            const int empty_key = h == t->cap;
            if (empty_key ? !t->has_empty_key : t->keys[h] == GEMPTY) continue;
            const uint64_t k = empty_key ? GEMPTY : t->keys[h];
            const uint64_t *src_st = empty_key ? t->empty_st : &t->st[h * (uint64_t)n_aggs];
            uint64_t *cnt;
            uint64_t *s = gtab_slot(&jobs[0].tab, k, n_aggs, agg_ops, agg_dtypes, &cnt);
            if (!s) {
                rc = FQ_E_TABLE_FULL;
                break;
            }
            *cnt += empty_key ? t->empty_cnt : t->cnt[h];
            for (int a = 0; a < n_aggs; ++a)
                if (agg_ops[a] == FQ_AGG_COUNT) s[a] += src_st[a];
                else gupdate(&s[a], agg_ops[a], agg_dtypes[a], src_st[a]);
        }
    }
    if (!rc) {
        gtab_t *t = &jobs[0].tab;
        uint64_t g = 0;
        for (uint64_t h = 0; h <= t->cap; ++h) {
            const int empty_key = h == t->cap;
            if (empty_key ? !t->has_empty_key : t->keys[h] == GEMPTY) continue;
            if (g >= cap_groups) {
                rc = FQ_E_TABLE_FULL;
                break;
            }
            out_keys[g] = empty_key ? GEMPTY : t->keys[h];
            memcpy(&out_states[g * (uint64_t)n_aggs], empty_key ? t->empty_st : &t->st[h * (uint64_t)n_aggs],
                   8 * (size_t)n_aggs);
            ++g;
        }
        *out_groups = g;
    }
    for (int32_t i = 0; i < np; ++i) gtab_free(&jobs[i].tab);
    free(jobs);
    return rc;
}

/* ------------------------------------------------------------------ */
/* FilterTransform -> ProjectionTransform over numbers_mt               */
/* (transform_filter.rs:38-55, transform_projection.rs:45-56): per      */
/* 10,000-row block materialise, filter_record_batch (compaction), then */
/* every projected expression evaluated into its own array.  The arrays */
/* are folded into per-output wrapping sums of the value bits (the      */
/* result would be 16 B per kept row: the checker compares sums and the */
/* kept count with closed forms).  CPU baseline of bench.py --query p1.  */
/* ------------------------------------------------------------------ */
typedef struct {
    uint64_t total;
    int32_t part, n_out;
    const fq_pred *pred;
    const fq_expr *outs;
    uint64_t kept, sums[FQ_MAX_PROJECT];
    err_t err;
} pjob_t;

static int project_block_fn(void *ctx, uint64_t b, uint64_t e) {
    pjob_t *j = (pjob_t *)ctx;
    arr_t blk = arr_new((int64_t)(e - b + 1), FQ_DT_UINT64), filtered;
    for (uint64_t i = b; i <= e; ++i) blk.v[i - b] = i;
    const arr_t *x = &blk;
    int rc = 0;
    if (j->pred && j->pred->kind == FQ_PRED_EXPR) {
        if (filter_block(j->pred, &blk, &filtered, &j->err)) rc = j->err.status;
        else x = &filtered;
    }
    if (!rc) j->kept += (uint64_t)x->n;
    for (int o = 0; !rc && o < j->n_out; ++o) {
        arr_t v;
        if (eval_chain(&j->outs[o], x, &v, &j->err)) {
            rc = j->err.status;
            break;
        }
        uint64_t s = 0;
        for (int64_t i = 0; i < v.n; ++i) s += v.v[i];
        j->sums[o] += s;
        arr_free(&v);
    }
    if (x == &filtered) arr_free(&filtered);
    arr_free(&blk);
    return rc;
}

static void *project_thread(void *arg) {
    pjob_t *j = (pjob_t *)arg;
    uint64_t b, e;
    fqo_partition_range(j->total, j->part, &b, &e);
    numbers_blocks(b, e, project_block_fn, j);
    return NULL;
}

int32_t fqo_numbers_project(uint64_t total, const fq_pred *pred, int32_t n_out, const fq_expr *outs,
                            int32_t n_threads, uint64_t *out_kept, uint64_t *out_sums, char *errbuf, int32_t errlen) {
    const int32_t np = fqo_num_partitions(total);
    if (n_out < 1 || n_out > FQ_MAX_PROJECT) return FQ_E_INVALID;
    pjob_t *jobs = (pjob_t *)calloc((size_t)np, sizeof(pjob_t));
    for (int32_t i = 0; i < np; ++i) {
        jobs[i].total = total;
        jobs[i].part = i;
        jobs[i].n_out = n_out;
        jobs[i].pred = pred;
        jobs[i].outs = outs;
    }
    if (n_threads <= 0 || n_threads > np) n_threads = np;
    pthread_t *th = (pthread_t *)calloc((size_t)n_threads, sizeof(pthread_t));
    for (int32_t w = 0; w < np; w += n_threads) {
        const int32_t k = (np - w) < n_threads ? (np - w) : n_threads;
        for (int32_t i = 0; i < k; ++i) pthread_create(&th[i], NULL, project_thread, &jobs[w + i]);
        for (int32_t i = 0; i < k; ++i) pthread_join(th[i], NULL);
    }
    free(th);
    int32_t rc = 0;
    *out_kept = 0;
    for (int o = 0; o < n_out; ++o) out_sums[o] = 0;
    for (int32_t i = 0; i < np; ++i) {
        if (jobs[i].err.status && !rc) {
            rc = jobs[i].err.status;
            if (errbuf && errlen > 0) snprintf(errbuf, (size_t)errlen, "%s", jobs[i].err.msg);
        }
        *out_kept += jobs[i].kept;
        for (int o = 0; o < n_out; ++o) out_sums[o] += jobs[i].sums[o];
    }
    free(jobs);
    return rc;
}
