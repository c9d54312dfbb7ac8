/* A plain C host of the drop-in boundary: what the Rust FFI of INTEGRATION.md
 * does, without Python or torch in the process.  Links libfq_amd.so and the
 * HIP runtime only (tests/native/Makefile; tests/test_c_client_gpu.py runs it
 * on the GPU box).
 *
 *  1. kernel ABI: hipMalloc a numbers_mt partition, fq_fill_numbers_u64
 *     (NumbersStream::poll_next, numbers_stream.rs:65-83), one fused
 *     fq_aggregate (AggregatorFunction::accumulate for sum/count/max/min,
 *     function_aggregator.rs:57-100) -> fq_agg_state, checked against the
 *     closed forms of begin..begin+n-1;
 *  2. error texts through fq_last_error (a NULL column);
 *  3. engine ABI: fq_engine_create -> materialise numbers_mt(N) -> the C3
 *     statement through fq_engine_execute -> fq_result values, checked
 *     against the closed forms.
 * Prints one "OK ..." line per check; exits non-zero on the first failure.
 *
 * `fq_c_client --bench STEPS TOTAL [WARMUP]`: the timed drop-in stack (C, the
 * /opt/rocm runtime, no torch): materialise numbers_mt(TOTAL) in HBM, then
 * STEPS x the C3 statement through fq_engine_execute with the engine's scan
 * timing on (FQ_OPT_PROFILE 2: one HIP-event span per query, first scan start
 * to last scan end -- bench.py's setting), every result checked against the
 * closed form; prints one JSON line (rows/s, ms per step, the scan kernel's
 * average time per launch and its fraction of the 8 TB/s HBM peak).      */
#define _POSIX_C_SOURCE 199309L /* clock_gettime under -std=c11 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <hip/hip_runtime_api.h>

#include "fq_engine.h"
#include "fq_gpu.h"

#define CHECK(cond, ...)                           \
    do {                                           \
        if (!(cond)) {                             \
            fprintf(stderr, "FAIL: " __VA_ARGS__); \
            fprintf(stderr, "\n");                 \
            exit(1);                               \
        }                                          \
    } while (0)

static void kernel_abi(uint64_t begin, uint64_t n) {
    hipStream_t st;
    CHECK(hipStreamCreate(&st) == hipSuccess, "hipStreamCreate");
    uint64_t *col = NULL;
    fq_agg_state *d_state = NULL;
    void *ws = NULL;
    const size_t ws_bytes = fq_aggregate_workspace_bytes((int64_t)n);
    CHECK(hipMalloc((void **)&col, n * 8) == hipSuccess, "hipMalloc column");
    CHECK(hipMalloc((void **)&d_state, sizeof(fq_agg_state)) == hipSuccess, "hipMalloc state");
    CHECK(hipMalloc(&ws, ws_bytes) == hipSuccess, "hipMalloc workspace");
    CHECK(fq_fill_numbers_u64(col, begin, n, st) == FQ_OK, "fill: %s", fq_last_error());
    fq_col c = {col, (int64_t)n, FQ_DT_UINT64, 0};
    const uint32_t mask = FQ_AGG_SUM | FQ_AGG_COUNT | FQ_AGG_MAX | FQ_AGG_MIN;
    CHECK(fq_aggregate(&c, 10000, NULL, NULL, mask, d_state, ws, ws_bytes, st) == FQ_OK, "aggregate: %s",
          fq_last_error());
    fq_agg_state s;
    CHECK(hipMemcpyAsync(&s, d_state, sizeof s, hipMemcpyDeviceToHost, st) == hipSuccess, "copy state");
    CHECK(hipStreamSynchronize(st) == hipSuccess, "sync");
    /* sum of begin .. begin+n-1, wrapping mod 2^64 */
    const unsigned __int128 last = (unsigned __int128)begin + n - 1;
    const uint64_t sum = (uint64_t)(((unsigned __int128)begin + last) * n / 2);
    CHECK(s.sum == sum && s.count == n && s.max == begin + n - 1 && s.min == begin,
          "state %llu/%llu/%llu/%llu", (unsigned long long)s.sum, (unsigned long long)s.count,
          (unsigned long long)s.max, (unsigned long long)s.min);
    printf("OK kernel abi: fq_fill_numbers_u64 + fq_aggregate over %llu rows from %llu: sum %llu count %llu "
           "max %llu min %llu\n",
           (unsigned long long)n, (unsigned long long)begin, (unsigned long long)s.sum, (unsigned long long)s.count,
           (unsigned long long)s.max, (unsigned long long)s.min);
    /* error path: a NULL column is rejected with a message */
    CHECK(fq_aggregate(NULL, 10000, NULL, NULL, mask, d_state, ws, ws_bytes, st) != FQ_OK &&
              strlen(fq_last_error()) > 0,
          "NULL column accepted");
    printf("OK error text: %s\n", fq_last_error());
    (void)hipFree(ws);
    (void)hipFree(d_state);
    (void)hipFree(col);
    (void)hipStreamDestroy(st);
}

static uint64_t value_u64(const fq_result *r, int32_t col) {
    fq_value v;
    CHECK(fq_result_value(r, 0, col, &v) == FQ_OK && v.is_some && v.dtype == FQ_DT_UINT64, "result value %d", col);
    return v.bits;
}

static void engine_abi(uint64_t total) {
    fq_engine *e = NULL;
    CHECK(fq_engine_create(0, &e) == FQ_OK, "engine: %s", fq_last_error());
    CHECK(fq_engine_materialize_numbers(e, total, 0, 1) == FQ_OK, "materialise: %s", fq_last_error());
    char sql[256];
    snprintf(sql, sizeof sql,
             "SELECT sum(number)/count(number), max(number), min(number) FROM system.numbers_mt(%llu)",
             (unsigned long long)total);
    fq_result *r = NULL;
    CHECK(fq_engine_execute(e, sql, &r) == FQ_OK, "execute: %s", fq_last_error());
    CHECK(fq_result_num_rows(r) == 1 && fq_result_num_columns(r) == 3, "result shape");
    const uint64_t sum = (uint64_t)((unsigned __int128)total * (total - 1) / 2);
    const uint64_t avg = value_u64(r, 0), mx = value_u64(r, 1), mn = value_u64(r, 2);
    CHECK(avg == sum / total && mx == total - 1 && mn == 0, "C3 = %llu %llu %llu", (unsigned long long)avg,
          (unsigned long long)mx, (unsigned long long)mn);
    printf("OK engine abi: %s -> [%s = %llu, %s = %llu, %s = %llu]\n", sql, fq_result_column_name(r, 0),
           (unsigned long long)avg, fq_result_column_name(r, 1), (unsigned long long)mx,
           fq_result_column_name(r, 2), (unsigned long long)mn);
    fq_result_free(r);
    /* the reference's error for an unknown function, through the same ABI */
    CHECK(fq_engine_execute(e, "SELECT foo(number) FROM system.numbers_mt(10)", &r) != FQ_OK, "unknown function");
    printf("OK engine error: %s\n", fq_last_error());
    fq_engine_destroy(e);
}

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + (double)t.tv_nsec * 1e-9;
}

static void c3_row(fq_engine *e, const char *sql, uint64_t out[3]) {
    fq_value row[3];
    int32_t n = 0;
    CHECK(fq_engine_execute_row(e, sql, row, 3, &n) == FQ_OK && n == 3, "execute_row: %s", fq_last_error());
    for (int c = 0; c < 3; ++c) {
        CHECK(row[c].is_some && row[c].dtype == FQ_DT_UINT64, "column %d is not a UInt64 value", c);
        out[c] = row[c].bits;
    }
}

static int bench(int steps, uint64_t total, int warmup) {
    fq_engine *e = NULL;
    CHECK(fq_engine_create(0, &e) == FQ_OK, "engine: %s", fq_last_error());
    CHECK(fq_engine_set_option(e, FQ_OPT_PROFILE, 2) == FQ_OK, "profile: %s", fq_last_error());
    CHECK(fq_engine_materialize_numbers(e, total, 0, 1) == FQ_OK, "materialise: %s", fq_last_error());
    char sql[256];
    snprintf(sql, sizeof sql,
             "SELECT sum(number)/count(number), max(number), min(number) FROM system.numbers_mt(%llu)",
             (unsigned long long)total);
    const uint64_t sum = (uint64_t)((unsigned __int128)total * (total - 1) / 2);
    const uint64_t expect[3] = {sum / total, total - 1, 0};
    uint64_t got[3];
    /* untimed steps for ~2 s first: HBM another process freed is cleared by
     * the driver in the background for a few seconds and slows the scans
     * (bench.py settle, profiles/r05_j_reclaim_probe/) */
    int settle = 0;
    for (const double s0 = now_s(); now_s() - s0 < 2.0; ++settle) c3_row(e, sql, got);
    for (int i = 0; i < (warmup > 0 ? warmup : 1); ++i) c3_row(e, sql, got);
    CHECK(memcmp(got, expect, sizeof got) == 0, "C3 = %llu %llu %llu", (unsigned long long)got[0],
          (unsigned long long)got[1], (unsigned long long)got[2]);
    CHECK(fq_engine_reset_stats(e) == FQ_OK, "reset stats");
    CHECK(hipDeviceSynchronize() == hipSuccess, "sync");
    int bad = 0;
    const double t0 = now_s();
    for (int i = 0; i < steps; ++i) {
        c3_row(e, sql, got);  /* the result row is on the host when execute returns */
        bad |= memcmp(got, expect, sizeof got) != 0;
    }
    CHECK(hipDeviceSynchronize() == hipSuccess, "sync");
    const double dt = now_s() - t0;
    CHECK(!bad, "a timed step returned another result");
    fq_engine_stats st;
    CHECK(fq_engine_get_stats(e, &st) == FQ_OK, "stats");
    const double launches = st.scan_launches ? (double)st.scan_launches : 1.0;
    const double kms = st.scan_ms / launches, bytes = (double)st.scan_bytes / launches;
    const double gbps = bytes / (kms * 1e-3) / 1e9;
    printf("{\"path\": \"fq_c_client (C host, libfq_amd.so + /opt/rocm libamdhip64, no torch): fq_engine_execute "
           "of the C3 statement\", \"workload\": \"%s\", \"steps\": %d, \"warmup\": %d, \"value\": %.6g, "
           "\"settle_steps\": %d, \"unit\": \"rows/s\", \"ms_per_step\": %.6g, \"scan_launches_per_step\": %.6g, "
           "\"kernel_ms_per_launch\": %.6g, \"bytes_per_launch\": %.6g, \"achieved_hbm_gbps\": %.6g, "
           "\"frac\": %.6g, \"step_over_scans\": %.6g, \"host_ms_per_step\": {\"plan\": %.6g, "
           "\"first_launch\": %.6g, \"exec\": %.6g, \"tail\": %.6g, \"tail_states\": %.6g, \"outside_exec\": %.6g}, "
           "\"result\": [%llu, %llu, %llu]}\n",
           sql, steps, warmup, (double)total * steps / dt, settle, dt / steps * 1e3, (double)st.scan_launches / steps, kms,
           bytes, gbps, gbps / 8000.0, (dt * 1e3) / (st.scan_ms > 0 ? st.scan_ms : 1.0), st.plan_ms / steps,
           st.first_launch_ms / steps, st.exec_ms / steps, st.tail_ms / steps, st.complete_ms / steps,
           (dt * 1e3 - st.plan_ms - st.exec_ms) / steps, (unsigned long long)got[0], (unsigned long long)got[1], (unsigned long long)got[2]);
    fq_engine_destroy(e);
    return 0;
}

/* ---- the Function-handle boundary, timed (`--handles STEPS TOTAL [WARMUP]`) ----
 * What a Rust host that keeps the reference's own transforms does with the C3
 * statement: its AggregatePartialTransform per partition pipe
 * (transform_aggregate_partial.rs:50-78) over the 3 Functions of the plan --
 * Sum/Count under an Arithmetic '/', Max, Min: 4 aggregator leaves -- with its
 * own Arrow-layout column per partition in HBM, then AggregateFinal's
 * merge_state / merge_result (transform_aggregate_final.rs:50-78).  One
 * fq_functions_accumulate call per partition: the block spans the partition's
 * 10,000-row reference blocks (block_rows) and the 4 leaves share one scan. */
static fq_function *fn_create(const char *name, fq_function *a, fq_function *b) {
    fq_function *args[2] = {a, b}, *out = NULL;
    CHECK(fq_function_create(name, args, b ? 2 : 1, &out) == FQ_OK, "create %s: %s", name, fq_last_error());
    return out;
}

static int handles(int steps, uint64_t total, int warmup) {
    CHECK(total % 80000 == 0, "--handles needs numbers_mt(N) with whole 10,000-row blocks per partition");
    fq_engine *e = NULL;
    CHECK(fq_engine_create(0, &e) == FQ_OK, "engine: %s", fq_last_error());
    CHECK(fq_engine_set_option(e, FQ_OPT_PROFILE, 1) == FQ_OK, "profile: %s", fq_last_error());
    /* the host's own partitions: numbers_mt's 8 ranges (numbers_table.rs:29-55) */
    enum { P = 8 };
    const uint64_t chunk = total / P;
    uint64_t *cols[P];
    fq_col fc[P];
    const char *names[1] = {"number"};
    for (int p = 0; p < P; ++p) {
        CHECK(hipMalloc((void **)&cols[p], chunk * 8) == hipSuccess, "hipMalloc partition %d", p);
        CHECK(fq_fill_numbers_u64(cols[p], (uint64_t)p * chunk, chunk, NULL) == FQ_OK, "fill: %s", fq_last_error());
        fc[p] = (fq_col){cols[p], (int64_t)chunk, FQ_DT_UINT64, 0};
    }
    CHECK(hipDeviceSynchronize() == hipSuccess, "sync");
    /* the plan's functions (plan_expression.rs:40-75): sum(number)/count(number), max(number), min(number) */
    fq_function *num = NULL;
    CHECK(fq_function_field("number", &num) == FQ_OK, "field");
    fq_function *tmpl[3];
    tmpl[0] = fn_create("/", fn_create("sum", num, NULL), fn_create("count", num, NULL));
    tmpl[1] = fn_create("max", num, NULL);
    tmpl[2] = fn_create("min", num, NULL);
    for (int i = 0; i < 3; ++i) CHECK(fq_function_set_depth(tmpl[i], 0) == FQ_OK, "depth");
    const uint64_t sum = (uint64_t)((unsigned __int128)total * (total - 1) / 2);
    const uint64_t expect[3] = {sum / total, total - 1, 0};
    uint64_t got[3] = {0, 0, 0};
    int bad = 0;
    double t0 = 0;
    /* untimed: the warmup steps, and steps for at least ~2 s (as --bench) */
    const int w = warmup > 0 ? warmup : 1;
    const double s0 = now_s();
    int first = -1;
    for (int it = 0; first < 0 || it < first + steps; ++it) {
        if (first < 0 && it >= w && now_s() - s0 >= 2.0) {
            first = it;
            CHECK(fq_engine_reset_stats(e) == FQ_OK, "reset stats");
            t0 = now_s();
        }
        fq_function *fin[3];
        for (int i = 0; i < 3; ++i) CHECK(fq_function_clone(tmpl[i], &fin[i]) == FQ_OK, "clone");
        for (int p = 0; p < P; ++p) {
            fq_function *part[3];
            for (int i = 0; i < 3; ++i) CHECK(fq_function_clone(tmpl[i], &part[i]) == FQ_OK, "clone");
            const fq_block blk = {1, names, &fc[p], 10000, NULL};
            CHECK(fq_functions_accumulate(e, part, 3, &blk) == FQ_OK, "accumulate: %s", fq_last_error());
            for (int i = 0; i < 3; ++i) {  /* the partial's state row -> AggregateFinal */
                fq_scalar st[4];
                size_t n = 0;
                CHECK(fq_function_accumulate_result(part[i], st, 4, &n) == FQ_OK, "accumulate_result");
                CHECK(fq_function_merge_state(fin[i], st, n) == FQ_OK, "merge_state: %s", fq_last_error());
                fq_function_free(part[i]);
            }
        }
        for (int i = 0; i < 3; ++i) {
            fq_scalar v;
            CHECK(fq_function_merge_result(fin[i], &v) == FQ_OK && v.kind == FQ_SCALAR_SOME, "merge_result");
            got[i] = v.bits;
            fq_function_free(fin[i]);
        }
        bad |= memcmp(got, expect, sizeof got) != 0;
    }
    const double dt = now_s() - t0;
    CHECK(!bad, "C3 through handles = %llu %llu %llu", (unsigned long long)got[0], (unsigned long long)got[1],
          (unsigned long long)got[2]);
    fq_engine_stats st;
    CHECK(fq_engine_get_stats(e, &st) == FQ_OK, "stats");
    const double launches = st.scan_launches ? (double)st.scan_launches : 1.0;
    const double kms = st.scan_ms / launches, bytes = (double)st.scan_bytes / launches;
    const double gbps = bytes / (kms * 1e-3) / 1e9;
    printf("{\"path\": \"fq_c_client --handles: 8 partitions x fq_functions_accumulate over the plan's 3 Function "
           "handles (4 aggregator leaves, one fused scan), block_rows 10000, then merge_state / merge_result\", "
           "\"total\": %llu, \"steps\": %d, \"value\": %.6g, \"unit\": \"rows/s\", \"ms_per_step\": %.6g, "
           "\"scan_launches_per_step\": %.6g, \"kernel_ms_per_launch\": %.6g, \"bytes_per_launch\": %.6g, "
           "\"achieved_hbm_gbps\": %.6g, \"frac\": %.6g, \"result\": [%llu, %llu, %llu]}\n",
           (unsigned long long)total, steps, (double)total * steps / dt, dt / steps * 1e3,
           (double)st.scan_launches / steps, kms, bytes, gbps, gbps / 8000.0, (unsigned long long)got[0],
           (unsigned long long)got[1], (unsigned long long)got[2]);
    for (int i = 0; i < 3; ++i) fq_function_free(tmpl[i]);
    fq_function_free(num);
    for (int p = 0; p < P; ++p) (void)hipFree(cols[p]);
    fq_engine_destroy(e);
    return 0;
}

int main(int argc, char **argv) {
    if (argc > 1 && strcmp(argv[1], "--handles") == 0) {
        const int steps = argc > 2 ? atoi(argv[2]) : 10;
        const uint64_t total = argc > 3 ? strtoull(argv[3], NULL, 10) : 10000000000ull;
        const int warmup = argc > 4 ? atoi(argv[4]) : 2;
        CHECK(steps > 0, "usage: fq_c_client --handles STEPS TOTAL [WARMUP]");
        return handles(steps, total, warmup);
    }
    if (argc > 1 && strcmp(argv[1], "--bench") == 0) {
        const int steps = argc > 2 ? atoi(argv[2]) : 20;
        const uint64_t total = argc > 3 ? strtoull(argv[3], NULL, 10) : 10000000000ull;
        const int warmup = argc > 4 ? atoi(argv[4]) : 3;
        CHECK(steps > 0 && total >= 8, "usage: fq_c_client --bench STEPS TOTAL [WARMUP]");
        return bench(steps, total, warmup);
    }
    const uint64_t n = argc > 1 ? strtoull(argv[1], NULL, 10) : 100000003ull;
    const uint64_t total = argc > 2 ? strtoull(argv[2], NULL, 10) : 1000000000ull;
    int32_t devices = 0;
    CHECK(fq_abi_version() > 0 && fq_device_count(&devices) == FQ_OK && devices > 0, "abi version / devices: %s",
          fq_last_error());
    printf("OK abi version %d, %d device(s)\n", fq_abi_version(), devices);
    kernel_abi(1250000000ull, n);
    engine_abi(total);
    return 0;
}
