// Host-side check of the C ABI under AddressSanitizer + UBSan (and, built
// with `make tsan`, ThreadSanitizer): the parts of libfq_amd that run on the
// CPU -- SQL planner / EXPLAIN, the AggregateFinal merge of exchanged states,
// the cross-rank exchange protocol (3 threads as 3 ranks through an
// in-process all-reduce), scalar state merge, coercion -- and a deterministic
// mutation fuzz of the planner.  No GPU is touched (host-only engine).
//
// Test infrastructure (tests/test_host_sanitized.py drives it): reads a
// script on stdin, one command per line, and prints one result line each.
//   EXPLAIN <sql>                  -> OK <escaped text> | ERR <status> <message>
//   FINAL <world> <hex>... <sql>   -> OK <row;row...>   | ERR <status> <message>
//   EXCHANGE <len0> <len1> ...     -> OK | FAIL <why>
//   XSIZED <cap> <len0> <len1> ... -> OK | FAIL <why>  (fq_exchange_states_sized)
//   XERRORS <world> <sql>          -> OK | FAIL <why>  (error records through fq_engine_execute_exchange)
//   FUZZ <seed> <count>            -> OK <n_ok> <n_err> (mutations of every EXPLAIN sql seen)
//   MERGE                          -> OK | FAIL <why>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <condition_variable>
#include <iostream>
#include <mutex>
#include <random>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "fq_comm.h"
#include "fq_engine.h"
#include "fq_gpu.h"

namespace {

std::string esc(const std::string &s) {
    std::string o;
    for (char c : s) {
        if (c == '\n') o += "\\n";
        else if (c == '\\') o += "\\\\";
        else o += c;
    }
    return o;
}

std::vector<uint8_t> unhex(const std::string &h) {
    std::vector<uint8_t> out(h.size() / 2);
    for (size_t i = 0; i < out.size(); ++i) out[i] = (uint8_t)std::stoi(h.substr(2 * i, 2), nullptr, 16);
    return out;
}

std::string explain(fq_engine *e, const std::string &sql, fq_status *st_out = nullptr) {
    size_t n = 0;
    fq_status st = fq_engine_explain(e, sql.c_str(), nullptr, 0, &n);
    if (st_out) *st_out = st;
    if (st != FQ_OK) return "ERR " + std::to_string(st) + " " + esc(fq_last_error());
    std::string buf(n + 1, '\0');
    st = fq_engine_explain(e, sql.c_str(), &buf[0], buf.size(), &n);
    if (st_out) *st_out = st;
    if (st != FQ_OK) return "ERR " + std::to_string(st) + " " + esc(fq_last_error());
    buf.resize(n);
    return "OK " + esc(buf);
}

std::string final_merge(fq_engine *e, const std::string &sql, const std::vector<std::vector<uint8_t>> &states) {
    size_t stride = 0;
    for (auto &s : states) stride = std::max(stride, s.size());
    std::vector<uint8_t> blob(stride * states.size(), 0);
    for (size_t r = 0; r < states.size(); ++r) memcpy(&blob[r * stride], states[r].data(), states[r].size());
    fq_result *res = nullptr;
    fq_status st = fq_engine_execute_final(e, sql.c_str(), blob.data(), stride, (int32_t)states.size(), &res);
    if (st != FQ_OK) return "ERR " + std::to_string(st) + " " + esc(fq_last_error());
    std::string o = "OK ";
    const int64_t rows = fq_result_num_rows(res);
    const int32_t cols = fq_result_num_columns(res);
    for (int64_t r = 0; r < rows; ++r) {
        if (r) o += ";";
        for (int32_t c = 0; c < cols; ++c) {
            if (c) o += ",";
            const char *t = fq_result_text(res, r, c);
            o += t ? t : "NULL";
        }
    }
    fq_result_free(res);
    return o;
}

// An in-process all-reduce over `world` threads: each rank adds its words
// into a shared accumulator, the last one in publishes, everyone copies out.
struct LocalAllReduce {
    int world;
    std::mutex mu;
    std::condition_variable cv;
    std::vector<uint64_t> acc, out;  // out: the last round's result (acc may already hold the next one)
    int arrived = 0;
    uint64_t generation = 0;

    static fq_status call(uint64_t *buf, int64_t n, void *user) {
        auto *self = (LocalAllReduce *)user;
        std::unique_lock<std::mutex> lk(self->mu);
        const uint64_t gen = self->generation;
        if (self->arrived == 0) self->acc.assign((size_t)n, 0);
        if ((int64_t)self->acc.size() != n) return FQ_E_INVALID;  // ranks disagree on the size
        for (int64_t i = 0; i < n; ++i) self->acc[(size_t)i] += buf[i];
        if (++self->arrived == self->world) {
            self->arrived = 0;
            self->out = self->acc;
            self->generation++;
            self->cv.notify_all();
        } else {
            self->cv.wait(lk, [&] { return self->generation != gen; });
        }
        memcpy(buf, self->out.data(), (size_t)n * 8);
        return FQ_OK;
    }
};

std::string run_exchange(const std::vector<size_t> &lens, long cap = -1) {
    const int world = (int)lens.size();
    LocalAllReduce ar;
    ar.world = world;
    std::vector<std::string> why((size_t)world);
    auto payload = [](int r, size_t i) { return (uint8_t)((r * 31 + (int)i) % 251 + 1); };
    std::vector<std::thread> ts;
    for (int r = 0; r < world; ++r)
        ts.emplace_back([&, r] {
            std::vector<uint8_t> mine(lens[(size_t)r]);
            for (size_t i = 0; i < mine.size(); ++i) mine[i] = payload(r, i);
            const void *rows = nullptr;
            size_t stride = 0;
            const fq_status st =
                cap < 0 ? fq_exchange_states(mine.data(), mine.size(), r, world, LocalAllReduce::call, &ar, &rows, &stride)
                        : fq_exchange_states_sized(mine.data(), mine.size(), (size_t)cap, r, world, LocalAllReduce::call,
                                                   &ar, &rows, &stride);
            if (st != FQ_OK) {
                why[(size_t)r] = fq_last_error();
                return;
            }
            const uint8_t *p = (const uint8_t *)rows;
            for (int q = 0; q < world; ++q)
                for (size_t i = 0; i < stride; ++i) {
                    const uint8_t exp = i < lens[(size_t)q] ? payload(q, i) : 0;
                    if (p[(size_t)q * stride + i] != exp) {
                        why[(size_t)r] = "rank " + std::to_string(r) + " row " + std::to_string(q) + " byte " +
                                         std::to_string(i);
                        return;
                    }
                }
        });
    for (auto &t : ts) t.join();
    for (auto &w : why)
        if (!w.empty()) return "FAIL " + w;
    return "OK";
}

// fq_engine_execute_exchange with one host-only engine per rank thread: every
// partial fails (no device), so every rank ships an error record through the
// sized exchange and every rank must report the same error.
std::string exchange_errors(int world, const std::string &sql) {
    LocalAllReduce ar;
    ar.world = world;
    std::vector<std::string> msg((size_t)world);
    std::vector<std::thread> ts;
    for (int r = 0; r < world; ++r)
        ts.emplace_back([&, r] {
            fq_engine *e = nullptr;
            if (fq_engine_create(-1, &e) != FQ_OK) {
                msg[(size_t)r] = "create";
                return;
            }
            fq_result *out = nullptr;
            const fq_status st = fq_engine_execute_exchange(e, sql.c_str(), r, world, LocalAllReduce::call, &ar, &out);
            msg[(size_t)r] = st == FQ_OK ? std::string("no error") : std::to_string(st) + " " + fq_last_error();
            fq_engine_stats s;
            if (fq_engine_get_stats(e, &s) != FQ_OK || s.exchanges != 1) msg[(size_t)r] += " (no exchange counted)";
            fq_result_free(out);
            fq_engine_destroy(e);
        });
    for (auto &t : ts) t.join();
    for (auto &m : msg)
        if (m != msg[0]) return "FAIL ranks disagree: " + msg[0] + " / " + m;
    return msg[0].rfind(std::to_string(FQ_E_HIP) + " ", 0) == 0 ? "OK" : "FAIL " + msg[0];
}

std::string merge_check() {
    fq_agg_state s[3] = {};
    s[0].sum = 10, s[0].count = 4, s[0].max = 4, s[0].min = 1, s[0].blocks = 1, s[0].dtype = FQ_DT_UINT64;
    s[1].sum = ~0ull - 4, s[1].count = 9, s[1].max = 3, s[1].min = 2, s[1].blocks = 2, s[1].dtype = FQ_DT_UINT64;
    s[2] = s[0];
    fq_agg_state out;
    if (fq_state_merge(s, 3, &out) != FQ_OK) return "FAIL merge status";
    if (out.sum != 15 || out.count != 17 || out.max != 4 || out.min != 1 || out.blocks != 4) return "FAIL merge values";
    int32_t t = 0;
    if (fq_arith_result_type(FQ_OP_ADD, FQ_DT_UINT64, FQ_DT_FLOAT64, &t) != FQ_OK || t != FQ_DT_FLOAT64)
        return "FAIL coercion";
    if (fq_arith_result_type(FQ_OP_ADD, FQ_DT_UTF8, FQ_DT_UTF8, &t) == FQ_OK) return "FAIL coercion error";
    return "OK";
}

// Deterministic planner fuzz: byte/token mutations of the seed statements.
std::string fuzz(fq_engine *e, const std::vector<std::string> &seeds, uint32_t seed, int count) {
    static const char *toks[] = {"(",     ")",     ",",     "+",     "-",    "*",       "/",  "%",  "<",
                                 ">",     "=",     "<=",    ">=",    "AND",  "OR",      "NOT", "sum(", "max(",
                                 "count(", "min(", "number", "1",     "-1",   "1.5",     "'a'", " ",  "LIMIT ",
                                 "WHERE ", "GROUP BY ", "AS x", "18446744073709551615", "99999999999999999999999",
                                 "system.numbers_mt(", "SELECT ", "FROM ", "\"", "''", "HAVING ", "EXPLAIN "};
    std::mt19937 rng(seed);
    int ok = 0, err = 0;
    for (int i = 0; i < count && !seeds.empty(); ++i) {
        std::string s = seeds[rng() % seeds.size()];
        const int edits = 1 + (int)(rng() % 4);
        for (int k = 0; k < edits; ++k) {
            const size_t pos = s.empty() ? 0 : rng() % (s.size() + 1);
            switch (rng() % 4) {
                case 0: s.insert(pos, toks[rng() % (sizeof toks / sizeof *toks)]); break;
                case 1: if (pos < s.size()) s.erase(pos, 1 + rng() % 8); break;
                case 2: if (pos < s.size()) s[pos] = (char)(32 + rng() % 95); break;
                default: s = s.substr(0, pos); break;
            }
        }
        fq_status st = FQ_OK;
        explain(e, s, &st);
        (st == FQ_OK ? ok : err)++;
    }
    return "OK " + std::to_string(ok) + " " + std::to_string(err);
}

}  // namespace

int main() {
    fq_engine *e = nullptr;
    if (fq_engine_create(-1, &e) != FQ_OK) {
        printf("FATAL %s\n", fq_last_error());
        return 2;
    }
    std::vector<std::string> seeds;
    std::string line;
    while (std::getline(std::cin, line)) {
        std::istringstream in(line);
        std::string cmd;
        in >> cmd;
        std::string out;
        if (cmd == "EXPLAIN") {
            std::string sql = line.substr(8);
            seeds.push_back(sql);
            out = explain(e, sql);
        } else if (cmd == "FINAL") {
            int world = 0;
            in >> world;
            std::vector<std::vector<uint8_t>> states;
            for (int r = 0; r < world; ++r) {
                std::string h;
                in >> h;
                states.push_back(unhex(h));
            }
            std::string sql;
            std::getline(in, sql);
            out = final_merge(e, sql.substr(1), states);
        } else if (cmd == "EXCHANGE") {
            std::vector<size_t> lens;
            size_t l;
            while (in >> l) lens.push_back(l);
            out = run_exchange(lens);
        } else if (cmd == "XSIZED") {  // XSIZED <cap> <len0> <len1> ...
            long cap = 0;
            in >> cap;
            std::vector<size_t> lens;
            size_t l;
            while (in >> l) lens.push_back(l);
            out = run_exchange(lens, cap);
        } else if (cmd == "XERRORS") {  // XERRORS <world> <sql>
            int world = 0;
            in >> world;
            std::string sql;
            std::getline(in, sql);
            out = exchange_errors(world, sql.substr(1));
        } else if (cmd == "FUZZ") {
            uint32_t seed = 0;
            int count = 0;
            in >> seed >> count;
            out = fuzz(e, seeds, seed, count);
        } else if (cmd == "MERGE") {
            out = merge_check();
        } else {
            out = "FAIL unknown command";
        }
        printf("%s\n", out.c_str());
        fflush(stdout);
    }
    fq_engine_destroy(e);
    return 0;
}
