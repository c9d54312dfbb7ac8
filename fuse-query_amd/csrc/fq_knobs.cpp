// Launch-shape knobs (include/fq_gpu.h "Launch-shape knobs"): compiled-in
// defaults, the measured best on MI355X, overridable only through the C ABI
// (the sweep tools) -- the library reads no environment for them.
#include <string.h>

#include <atomic>
#include <mutex>
#include <string>

#include "fq_common.h"

namespace {

struct KnobDef {
    int64_t def, lo, hi;
    int64_t step;    // value must be lo + k * step (1: any in range)
    bool pow2;       // value must be a power of two (LBW 1/2/4/8, ...)
};

// index = FQ_TUNE_*; the sweeps behind the defaults are in DESIGN.md
constexpr KnobDef kDefs[FQ_TUNE_COUNT] = {
    {2, 1, 16, 1, false},           // SCAN_WG_PER_CU
    {0, 0, 16, 1, false},           // EW_WG_PER_CU
    {8, 4, 16, 1, true},            // BLOCK_U
    {8, 1, 16, 1, false},           // SELECT_WG_PER_CU
    {8, 1, 16, 1, false},           // SELECT_BLOCKS_WG_PER_CU
    {32, 8, 32, 1, true},           // SELECT_BLOCKS_ROWS
    {2, 0, 4, 1, true},             // SELECT_BLOCKS_STAGE
    {1, 0, 1, 1, false},            // BLOCK_CACHE
    {0, 0, 100000, 1, false},       // POOL_SPIN_US
    {1024, 256, 1024, 256, false},  // GROUP_THREADS
    {128, 8, 160, 1, false},        // GROUP_LDS_KB
    {1, 1, 8, 1, false},            // GROUP_WG_PER_CU
    {160, 0, 512, 1, false},        // GROUP_CLUSTER
    {1, 0, 1, 1, false},            // GROUP_CHUNKED
    {1, 0, 1, 1, false},            // GROUP_RANGE_BINS
    {1, 0, 1, 1, false},            // GROUP_NARROW
    {2, 1, 4, 1, false},            // GPART_WG_PER_CU
    {2, 1, 4, 1, false},            // GBINS_WG_PER_CU
};

std::atomic<int64_t> g_val[FQ_TUNE_COUNT] = {};
std::once_flag g_init;

void init() {
    std::call_once(g_init, [] {
        for (int i = 0; i < FQ_TUNE_COUNT; ++i) g_val[i].store(kDefs[i].def);
    });
}

bool valid(int k, int64_t v) {
    const KnobDef &d = kDefs[k];
    if (v < d.lo || v > d.hi) return false;
    if ((v - d.lo) % d.step) return false;
    if (d.pow2 && (v & (v - 1))) return false;
    return true;
}

std::mutex g_dump_mu;
std::string g_dump_dir;

}  // namespace

namespace fqc {

int64_t knob(int k) {
    init();
    return g_val[k].load(std::memory_order_relaxed);
}

std::string jit_dump_dir() {
    std::lock_guard<std::mutex> lk(g_dump_mu);
    return g_dump_dir;
}

}  // namespace fqc

extern "C" {

fq_status fq_tune_set(int32_t knob, int64_t value) {
    if (knob < 0 || knob >= FQ_TUNE_COUNT) return fqc::fail(FQ_E_INVALID, "fq_tune_set: unknown knob");
    if (!valid(knob, value))
        return fqc::fail(FQ_E_INVALID, "fq_tune_set: value " + std::to_string(value) + " outside knob " +
                                           std::to_string(knob) + "'s set");
    init();
    g_val[knob].store(value);
    return FQ_OK;
}

int64_t fq_tune_get(int32_t knob) {
    if (knob < 0 || knob >= FQ_TUNE_COUNT) return -1;
    return fqc::knob(knob);
}

fq_status fq_tune_reset(void) {
    init();
    for (int i = 0; i < FQ_TUNE_COUNT; ++i) g_val[i].store(kDefs[i].def);
    return FQ_OK;
}

fq_status fq_tune_jit_dump_dir(const char *dir) {
    std::lock_guard<std::mutex> lk(g_dump_mu);
    g_dump_dir = dir ? dir : "";
    return FQ_OK;
}

}  // extern "C"
