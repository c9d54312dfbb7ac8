// hipRTC specialisation of the fused AggregatePartial scan.
//
// The precompiled scan kernels (fq_aggregate.hip) interpret the lowered
// expression program step by step: every step is a wave-uniform switch, which
// is cheap per step but leaves the compiler a kernel of thousands of
// instructions with copies at every join, 160+ VGPRs and three waves per SIMD.
// For a filtered/computed scan (BASELINE C4, `max(number+1) WHERE
// (number%8)<3`) that is compute-bound at ~60 % of HBM bandwidth.
//
// Here the same program is emitted as straight-line HIP source -- one inline
// function for the predicate, one for the argument expression -- around the
// same tile-contiguous streaming loop, compiled once per expression SHAPE
// (step ops, operand kinds, dtypes, libdivide "add" marker, aggregate mask)
// with hipRTC for the device's own gfx target, and cached for the process.
// Constants (literals, divide magics, shifts) stay kernel arguments, so
// `WHERE number % 8 < 3` and `WHERE number % 8 < 5` share one kernel.
//
// Semantics are the interpreter's, element for element (flag raising for
// live rows only, the same per-lane accumulation order, the same partial
// layout), so a specialised scan and an interpreted one return identical
// fq_agg_state bits for the same grid; tests/test_kernels_gpu.py checks both
// against the oracle.
#include <dlfcn.h>
#include <pthread.h>
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "fq_common.h"
#include "fq_device.h"
#include "fq_scan.h"

namespace fqk {
namespace {

// ---------------------------------------------------------------------------
// hipRTC, loaded on first use (libfq_amd.so does not link it, so the library
// still loads where hipRTC is absent).
//
// Which compiler: a process that imported torch already holds torch's
// bundled libhiprtc + libamd_comgr (an older LLVM), and dlopen by SONAME
// returns those.  That compiler allocated 288 VGPRs for the select kernel
// that ROCm 7.2's compiles to 61 (one workgroup per CU instead of 7: the
// Filter+Projection scan ran 3x slower).  So the system ROCm's hipRTC is
// loaded into a link-map namespace of its own (dlmopen), where it resolves
// its own comgr; only the code object bytes cross back.  FQ_JIT_RTC=process
// takes the process's hipRTC instead (A/B).
// ---------------------------------------------------------------------------
struct Rtc {
    decltype(&hiprtcCreateProgram) create = nullptr;
    decltype(&hiprtcCompileProgram) compile = nullptr;
    decltype(&hiprtcGetProgramLogSize) log_size = nullptr;
    decltype(&hiprtcGetProgramLog) log = nullptr;
    decltype(&hiprtcGetCodeSize) code_size = nullptr;
    decltype(&hiprtcGetCode) code = nullptr;
    decltype(&hiprtcDestroyProgram) destroy = nullptr;
    bool ok = false;
    bool isolated = false;  // the system ROCm's hipRTC in its own link-map namespace
};

// Every hipRTC call runs on one thread of its own (64 MB stack), the one
// that loaded it: the namespace's own libc copy then serves a single thread.
// Sources with inline asm (round 3's since-removed LDS-DMA path in the
// partition kernel) compiled from several threads -- the engine's workers --
// crashed the process inside hipRTC (SIGSEGV); on one thread, or with the
// process's hipRTC, they compile (tests/test_jit_cpu.py::
// test_compiles_from_many_threads compiles 16 shapes from fresh threads).
class RtcThread {
  public:
    static RtcThread &get() {
        static RtcThread *t = new RtcThread;  // never destroyed: the thread outlives static teardown
        return *t;
    }
    void run(const std::function<void()> &f) {
        std::lock_guard<std::mutex> one(call_mu_);  // one job at a time
        if (!ok_) {
            f();
            return;
        }
        std::unique_lock<std::mutex> lk(mu_);
        job_ = &f;
        done_ = false;
        cv_.notify_all();
        cv_.wait(lk, [this] { return done_; });
    }

  private:
    RtcThread() {
        pthread_attr_t a;
        pthread_attr_init(&a);
        pthread_attr_setstacksize(&a, (size_t)64 << 20);
        pthread_t t;
        ok_ = pthread_create(&t, &a, &RtcThread::main, this) == 0;
        pthread_attr_destroy(&a);
        if (ok_) pthread_detach(t);
    }
    static void *main(void *self) {
        RtcThread &t = *(RtcThread *)self;
        std::unique_lock<std::mutex> lk(t.mu_);
        for (;;) {
            t.cv_.wait(lk, [&t] { return t.job_ != nullptr; });
            (*t.job_)();
            t.job_ = nullptr;
            t.done_ = true;
            t.cv_.notify_all();
        }
        return nullptr;
    }
    std::mutex call_mu_, mu_;
    std::condition_variable cv_;
    const std::function<void()> *job_ = nullptr;
    bool done_ = false, ok_ = false;
};

const Rtc &rtc() {
    static const Rtc r = [] {
        Rtc x;
        RtcThread::get().run([&x] {
            void *h = nullptr;
            {  // its own link namespace: hipRTC's LLVM never meets another copy in the process
                const char *root = getenv("ROCM_PATH");
                const std::string path = std::string(root && *root ? root : "/opt/rocm") + "/lib/libhiprtc.so.7";
                h = dlmopen(LM_ID_NEWLM, path.c_str(), RTLD_NOW | RTLD_LOCAL);
                x.isolated = h != nullptr;
            }
            if (!h) h = dlopen("libhiprtc.so.7", RTLD_NOW | RTLD_GLOBAL);
            if (!h) h = dlopen("libhiprtc.so", RTLD_NOW | RTLD_GLOBAL);
            if (!h) return;
            x.create = (decltype(x.create))dlsym(h, "hiprtcCreateProgram");
            x.compile = (decltype(x.compile))dlsym(h, "hiprtcCompileProgram");
            x.log_size = (decltype(x.log_size))dlsym(h, "hiprtcGetProgramLogSize");
            x.log = (decltype(x.log))dlsym(h, "hiprtcGetProgramLog");
            x.code_size = (decltype(x.code_size))dlsym(h, "hiprtcGetCodeSize");
            x.code = (decltype(x.code))dlsym(h, "hiprtcGetCode");
            x.destroy = (decltype(x.destroy))dlsym(h, "hiprtcDestroyProgram");
            x.ok = x.create && x.compile && x.log_size && x.log && x.code_size && x.code && x.destroy;
        });
        return x;
    }();
    return r;
}

// ---------------------------------------------------------------------------
// policy + statistics
// ---------------------------------------------------------------------------
std::atomic<int32_t> g_mode{-1};
std::atomic<int64_t> g_min_rows{-1};
std::atomic<int64_t> g_compiled{0}, g_jit_launches{0}, g_interp_launches{0};
std::atomic<int64_t> g_compile_us{0};
std::atomic<int32_t> g_available{-1};

int32_t jit_mode() {
    int32_t m = g_mode.load(std::memory_order_relaxed);
    if (m < 0) {
        const char *e = getenv("FQ_JIT");
        m = e ? atoi(e) : FQ_JIT_AUTO;
        if (m < FQ_JIT_OFF || m > FQ_JIT_ALWAYS) m = FQ_JIT_AUTO;
        int32_t expect = -1;
        g_mode.compare_exchange_strong(expect, m);
        m = g_mode.load();
    }
    return m;
}

int64_t jit_min_rows() {
    int64_t r = g_min_rows.load(std::memory_order_relaxed);
    if (r < 0) {
        const char *e = getenv("FQ_JIT_MIN_ROWS");
        r = e ? atoll(e) : (int64_t)1 << 22;
        if (r < 0) r = (int64_t)1 << 22;
        int64_t expect = -1;
        g_min_rows.compare_exchange_strong(expect, r);
        r = g_min_rows.load();
    }
    return r;
}

// ---------------------------------------------------------------------------
// source generation
// ---------------------------------------------------------------------------
const char *ctype(int32_t dt) {
    switch (dt) {
        case FQ_DT_INT64: return "long long";
        case FQ_DT_UINT64: return "unsigned long long";
        case FQ_DT_FLOAT64: return "double";
        default: return nullptr;
    }
}

// column element x (type tin) -> 64-bit value encoding
std::string x_bits(int32_t tin) {
    if (tin == FQ_DT_FLOAT64) return "__builtin_bit_cast(u64, x)";
    return "(u64)x";
}

// Constants of step i of the predicate ("p") or argument ("v") program are
// kernel arguments c.p[i] / c.v[i] (fields c, m = magic, s = shift), packed
// straight from the lowered KProg (pack_consts); the predicate's constant
// right-hand side is c.rhs.
constexpr int kSteps = (int)(sizeof(KProg{}.s) / sizeof(KStep));
struct HostStep {
    uint64_t c, m, s;
};
struct HostConsts {
    uint64_t rhs;
    HostStep p[kSteps], v[kSteps];
    uint64_t rl[FQ_MAX_PRED_LEAVES];  // FQ_PRED_TREE leaves
    HostStep pl[FQ_MAX_PRED_LEAVES][kSteps];
};

template <typename HC>
void pack_tree_consts(const KPred &pr, HC &hc) {
    for (int l = 0; l < FQ_MAX_PRED_LEAVES; ++l) {
        hc.rl[l] = pr.leaves[l].rhs;
        for (int i = 0; i < kSteps; ++i)
            hc.pl[l][i] = HostStep{pr.leaves[l].lhs.s[i].c, pr.leaves[l].lhs.s[i].magic, pr.leaves[l].lhs.s[i].shift};
    }
}

struct Gen {
    const char *prefix = "v";
    int step = 0;
    int uid = 0;                    // names of pushed tree values (s0, s1, ...)
    std::vector<std::string> stk;  // the value stack of FQ_OP_PUSH / FQ_OPERAND_STACK
    std::string K(const char *field) const {
        return std::string("c.") + prefix + "[" + std::to_string(step) + "]." + field;
    }
};

void pack_consts(const Launch &L, HostConsts &hc) {
    hc.rhs = L.pred.rhs;
    for (int i = 0; i < kSteps; ++i) {
        hc.p[i] = HostStep{L.pred.lhs.s[i].c, L.pred.lhs.s[i].magic, L.pred.lhs.s[i].shift};
        hc.v[i] = HostStep{L.val.s[i].c, L.val.s[i].magic, L.val.s[i].shift};
    }
    pack_tree_consts(L.pred, hc);
}

// the predicate's part of a shape key
void put_pred_key(const KPred &pr, std::string &k) {
    auto put = [&k](int32_t v) { k.append(reinterpret_cast<const char *>(&v), sizeof v); };
    auto prog = [&put](const KProg &p) {
        put(p.n);
        for (int i = 0; i < p.n; ++i) {
            put(p.s[i].code);
            put(p.s[i].operand);
            put(p.s[i].reversed);
            put(p.s[i].dtype);
            put((int32_t)p.s[i].add);
            put(p.s[i].sdtype);
        }
    };
    put(pr.kind);
    if (pr.kind == FQ_PRED_EXPR) {
        put(pr.cmp);
        put(pr.cmp_dtype);
        put(pr.rhs_operand);
        prog(pr.lhs);
    } else if (pr.kind == FQ_PRED_TREE) {
        put(pr.n_leaves);
        put(pr.n_prog);
        for (int i = 0; i < pr.n_prog; ++i) put(pr.prog[i]);
        for (int l = 0; l < pr.n_leaves; ++l) {
            put(pr.leaves[l].cmp);
            put(pr.leaves[l].cmp_dtype);
            put(pr.leaves[l].rhs_operand);
            prog(pr.leaves[l].lhs);
        }
    }
}

// 16-byte vectors per lane in flight in the block-mode scan (FQ_TUNE_BLOCK_U:
// 4, 8 or 16)
int block_mode_vectors() { return (int)fqc::knob(FQ_TUNE_BLOCK_U); }

// Binary shape key: everything the generated source depends on.
std::string shape_key(const Launch &L, int32_t tin, bool chain, int dev) {
    std::string k;
    k.reserve(256);
    auto put = [&k](int32_t v) { k.append(reinterpret_cast<const char *>(&v), sizeof v); };
    put(dev);
    put(block_mode_vectors());
    put(tin);
    put(L.vdtype);
    put((int32_t)L.mask);
    put_pred_key(L.pred, k);
    put(L.block_mode ? 1 : 0);
    put(chain ? 1 : 0);
    auto prog = [&put](const KProg &p) {
        put(p.n);
        for (int i = 0; i < p.n; ++i) {
            put(p.s[i].code);
            put(p.s[i].operand);
            put(p.s[i].reversed);
            put(p.s[i].dtype);
            put((int32_t)p.s[i].add);
            put(p.s[i].sdtype);
        }
    };
    if (chain) prog(L.val);
    return k;
}

// col_as(dtype, x, live): the column as the operand of a step in `dt`
std::string col_as(Gen &g, std::string &body, int32_t tin, int32_t dt) {
    if (dt == FQ_DT_FLOAT64) return "__builtin_bit_cast(u64, (double)x)";
    if (tin == FQ_DT_UINT64 && dt == FQ_DT_INT64)
        body += "    flags |= (u32)((x >> 63) & (u64)live) * " + std::to_string(FQ_STATE_CAST_NULL) + "u;\n";
    (void)g;
    return x_bits(tin);
}

// Straight-line code for one lowered program acting on `a`.
void emit_prog(Gen &g, std::string &body, const KProg &p, int32_t tin, const char *prefix) {
    g.prefix = prefix;
    for (int i = 0; i < p.n; ++i) {
        const KStep &st = p.s[i];
        g.step = i;
        const std::string DZ = std::to_string(FQ_STATE_DIV_ZERO) + "u";
        switch (st.code) {
            case K_NOP: continue;
            case K_CAST_U2I:
                body += "    flags |= (u32)((a >> 63) & (u64)live) * " + std::to_string(FQ_STATE_CAST_NULL) + "u;\n";
                continue;
            case K_CAST_U2F: body += "    a = __builtin_bit_cast(u64, (double)a);\n"; continue;
            case K_CAST_I2F: body += "    a = __builtin_bit_cast(u64, (double)(long long)a);\n"; continue;
            case K_PUSH: {  // expression tree: keep acc, restart from the column
                const std::string v = "s" + std::to_string(g.uid++);
                body += "    const u64 " + v + " = a;\n    a = " + x_bits(tin) + ";\n";
                g.stk.push_back(v);
                continue;
            }
            case K_SHR_U: body += "    a = a >> (u32)" + g.K("s") + ";\n"; continue;
            case K_AND_U: body += "    a = a & " + g.K("m") + ";\n"; continue;
            case K_MODM32_U: {
                const std::string M = g.K("m"), S = g.K("s"), C = g.K("c");
                const char *q = st.add ? "(((n - q) >> 1) + q) >> sh" : "q >> sh";
                body += "    { const u32 m = (u32)" + M + ", c2 = (u32)(" + M + " >> 32), sh = (u32)" + S +
                        ", d = (u32)" + C + ";\n";
                body += std::string("      auto md = [&](u32 n) -> u32 { u32 q = __umulhi(n, m); q = ") + q +
                        "; return n - q * d; };\n";
                body += "      a = (u64)md(md((u32)(a >> 32)) * c2 + md((u32)a)); }\n";
                continue;
            }
            case K_DIVM32_U: {
                const std::string M = g.K("m"), S = g.K("s"), C = g.K("c");
                const char *q = st.add ? "(((n - q) >> 1) + q) >> sh" : "q >> sh";
                body += "    { const u32 m = (u32)" + M + ", sh = (u32)" + S + ", d = (u32)" + C + ";\n";
                body += std::string("      auto dv = [&](u32 n) -> u32 { u32 q = __umulhi(n, m); return ") + q + "; };\n";
                body += "      const u32 hi = (u32)(a >> 32), lo = (u32)a;\n"
                        "      const u32 qh = dv(hi), t1 = ((hi - qh * d) << 16) | (lo >> 16);\n"
                        "      const u32 q1 = dv(t1), q0 = dv(((t1 - q1 * d) << 16) | (lo & 0xffffu));\n"
                        "      a = ((u64)qh << 32) | (u64)((q1 << 16) + q0); }\n";
                continue;
            }
            case K_DIVM_U:
            case K_MODM_U: {
                const std::string M = g.K("m"), S = g.K("s");
                body += "    { u64 q = __umul64hi(a, " + M + ");\n";
                if (st.add) body += "      q = (((a - q) >> 1) + q) >> (u32)" + S + ";\n";
                else body += "      q = q >> (u32)" + S + ";\n";
                if (st.code == K_DIVM_U) body += "      a = q; }\n";
                else body += "      a = a - q * " + g.K("c") + "; }\n";
                continue;
            }
            default: break;
        }
        // binary step with an operand b
        std::string b;
        if (st.operand == FQ_OPERAND_COLUMN) {
            b = col_as(g, body, tin, st.dtype);
        } else if (st.operand == FQ_OPERAND_STACK) {  // the left subtree's value, cast like acc
            const std::string v = g.stk.empty() ? std::string("0ull") : g.stk.back();
            if (!g.stk.empty()) g.stk.pop_back();
            if (st.sdtype == st.dtype) b = v;
            else if (st.sdtype == FQ_DT_UINT64 && st.dtype == FQ_DT_INT64) {
                body += "    flags |= (u32)((" + v + " >> 63) & (u64)live) * " + std::to_string(FQ_STATE_CAST_NULL) + "u;\n";
                b = v;
            } else if (st.sdtype == FQ_DT_UINT64) b = "__builtin_bit_cast(u64, (double)" + v + ")";
            else b = "__builtin_bit_cast(u64, (double)(long long)" + v + ")";
        } else {
            b = g.K("c");
        }
        body += "    { const u64 b = " + b + ";\n";
        body += st.reversed ? "      const u64 L = b, R = a;\n" : "      const u64 L = a, R = b;\n";
        switch (st.code) {
            case K_ADD_I: body += "      a = L + R; }\n"; break;
            case K_SUB_I: body += "      a = L - R; }\n"; break;
            case K_MUL_I: body += "      a = L * R; }\n"; break;
            case K_DIV_U:
                body += "      flags |= (R == 0 && live) ? " + DZ + " : 0u;\n      a = R ? L / R : 0; }\n";
                break;
            case K_MOD_U:
                body += "      flags |= (R == 0 && live) ? " + DZ + " : 0u;\n      a = R ? L % R : 0; }\n";
                break;
            case K_DIV_S:
            case K_MOD_S: {
                const bool div = st.code == K_DIV_S;
                body += "      flags |= (R == 0 && live) ? " + DZ + " : 0u;\n";
                body += "      const long long sl = (long long)L, sr = (long long)R;\n";
                body += std::string("      a = sr == 0 ? 0 : (sr == -1 ? ") + (div ? "(u64)0 - L" : "(u64)0") +
                        " : (u64)(sl " + (div ? "/" : "%") + " sr)); }\n";
                break;
            }
            case K_ADD_F:
            case K_SUB_F:
            case K_MUL_F:
            case K_DIV_F:
            case K_MOD_F: {
                body += "      const double fl = __builtin_bit_cast(double, L), fr = __builtin_bit_cast(double, R);\n";
                const char *e = st.code == K_ADD_F   ? "fl + fr"
                                : st.code == K_SUB_F ? "fl - fr"
                                : st.code == K_MUL_F ? "fl * fr"
                                : st.code == K_DIV_F ? "fl / fr"
                                                     : "fmod(fl, fr)";
                if (st.code == K_DIV_F || st.code == K_MOD_F)
                    body += "      flags |= (fr == 0.0 && live) ? " + DZ + " : 0u;\n";
                body += std::string("      a = __builtin_bit_cast(u64, ") + e + "); }\n";
                break;
            }
            default: body += "      (void)L; (void)R; }\n"; break;
        }
    }
}

const char *cmp_op(int32_t cmp) {
    switch (cmp) {
        case FQ_CMP_EQ: return "==";
        case FQ_CMP_LT: return "<";
        case FQ_CMP_LTEQ: return "<=";
        case FQ_CMP_GT: return ">";
        case FQ_CMP_GTEQ: return ">=";
        default: return nullptr;
    }
}

const char *kCommon = R"(
typedef unsigned long long u64;
typedef unsigned int u32;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
struct Partial { u64 sum, max, min, count, blocks; u32 flags; int dtype; };
template <typename T> __device__ __forceinline__ T shfl64(T v, int m) {
    const u64 b = __builtin_bit_cast(u64, v);
    const u32 lo = __shfl_xor((u32)(b & 0xffffffffu), m, 64);
    const u32 hi = __shfl_xor((u32)(b >> 32), m, 64);
    return __builtin_bit_cast(T, ((u64)hi << 32) | lo);
}
template <typename T> __device__ __forceinline__ T vmax(T a, T b) { return b > a ? b : a; }
template <typename T> __device__ __forceinline__ T vmin(T a, T b) { return b < a ? b : a; }
)";

// Body of `bool fq_pred(TIn x, ...)`: the lowered predicate program on x,
// then the comparison in cmp_dtype.
bool emit_leaf(Gen &g, int32_t cmp, int32_t cmp_dtype, int32_t rhs_operand, const KProg &lhs, const std::string &rhs,
               const char *prefix, int32_t tin, std::string &body, const std::string &result) {
    const char *op = cmp_op(cmp);
    if (!op) return false;
    body += "    {\n    u64 a = " + x_bits(tin) + ";\n";
    emit_prog(g, body, lhs, tin, prefix);
    std::string r;
    if (rhs_operand == FQ_OPERAND_COLUMN) r = col_as(g, body, tin, cmp_dtype);
    else r = rhs;
    body += "    const u64 r = " + r + ";\n";
    if (cmp_dtype == FQ_DT_UINT64) body += "    " + result + " = a " + op + " r;\n";
    else if (cmp_dtype == FQ_DT_INT64) body += "    " + result + " = (long long)a " + op + " (long long)r;\n";
    else if (cmp_dtype == FQ_DT_FLOAT64)
        body += "    " + result + " = __builtin_bit_cast(double, a) " + op + " __builtin_bit_cast(double, r);\n";
    else
        return false;
    body += "    }\n";
    return true;
}

bool emit_pred_body(Gen &g, const KPred &pr, int32_t tin, std::string &body) {
    if (pr.kind == FQ_PRED_TREE) {
        // every leaf evaluated (no short circuit: arrow and/or evaluate both
        // sides, so either side's errors raise), then the postfix program
        std::vector<std::string> names;
        for (int l = 0; l < pr.n_leaves; ++l) {
            const std::string b = "b" + std::to_string(l);
            body += "    bool " + b + ";\n";
            const std::string prefix = "pl[" + std::to_string(l) + "]";
            if (!emit_leaf(g, pr.leaves[l].cmp, pr.leaves[l].cmp_dtype, pr.leaves[l].rhs_operand, pr.leaves[l].lhs,
                           "c.rl[" + std::to_string(l) + "]", prefix.c_str(), tin, body, b))
                return false;
        }
        std::vector<std::string> st;
        for (int i = 0; i < pr.n_prog; ++i) {
            const int32_t t = pr.prog[i];
            if (t >= 0 && t < pr.n_leaves) {
                st.push_back("b" + std::to_string(t));
            } else {
                if (st.size() < 2) return false;
                const std::string r = st.back();
                st.pop_back();
                const std::string l = st.back();
                st.pop_back();
                st.push_back("(" + l + (t == FQ_PRED_AND ? " & " : " | ") + r + ")");
            }
        }
        if (st.size() != 1) return false;
        body += "    return " + st[0] + ";\n";
        return true;
    }
    const char *op = cmp_op(pr.cmp);
    if (!op) return false;
    body += "    u64 a = " + x_bits(tin) + ";\n";
    emit_prog(g, body, pr.lhs, tin, "p");
    std::string r;
    if (pr.rhs_operand == FQ_OPERAND_COLUMN) r = col_as(g, body, tin, pr.cmp_dtype);
    else r = "c.rhs";
    body += "    const u64 r = " + r + ";\n";
    if (pr.cmp_dtype == FQ_DT_UINT64) body += std::string("    return a ") + op + " r;\n";
    else if (pr.cmp_dtype == FQ_DT_INT64) body += std::string("    return (long long)a ") + op + " (long long)r;\n";
    else if (pr.cmp_dtype == FQ_DT_FLOAT64)
        body += std::string("    return __builtin_bit_cast(double, a) ") + op + " __builtin_bit_cast(double, r);\n";
    else
        return false;
    return true;
}

// Body of `V fq_val(TIn x, ...)`: the lowered argument program (identity
// when prog is null) returning a value of type `vname` (dtype vdt).
void emit_value_body(Gen &g, const KProg *prog, int32_t tin, int32_t vdt, const char *prefix, const char *vname,
                     std::string &body) {
    if (!prog) {
        body += std::string("    return (") + vname + ")x;\n";
        return;
    }
    body += "    u64 a = " + x_bits(tin) + ";\n";
    emit_prog(g, body, *prog, tin, prefix);
    if (vdt == FQ_DT_FLOAT64) body += "    return __builtin_bit_cast(double, a);\n";
    else body += std::string("    return (") + vname + ")a;\n";
}

// Full kernel source for one shape.  Returns false if the shape is outside
// what the generator handles (the caller then interprets).
bool gen_source(const Launch &L, int32_t tin, bool chain, Gen &g, std::string &src) {
    const char *TIn = ctype(tin);
    const char *V = ctype(L.vdtype);
    if (!TIn || !V) return false;
    const int32_t pk = L.pred.kind;

    std::string pred_body, val_body;
    const bool expr_pred = pk == FQ_PRED_EXPR || pk == FQ_PRED_TREE;
    if (expr_pred && !emit_pred_body(g, L.pred, tin, pred_body)) return false;
    emit_value_body(g, chain ? &L.val : nullptr, tin, L.vdtype, "v", "V", val_body);

    src = kCommon;
    src += "typedef " + std::string(TIn) + " TIn;\ntypedef " + V + " V;\n";
    src += "struct Step { u64 c, m, s; };\nstruct Consts { u64 rhs; Step p[" + std::to_string(kSteps) +
           "], v[" + std::to_string(kSteps) + "]; u64 rl[" + std::to_string(FQ_MAX_PRED_LEAVES) + "]; Step pl[" +
           std::to_string(FQ_MAX_PRED_LEAVES) + "][" + std::to_string(kSteps) + "]; };\n";
    src += "__device__ __forceinline__ bool fq_pred(TIn x, const Consts &c, u32 &flags, u32 live) {\n";
    src += expr_pred ? pred_body : "    return true;\n";
    src += "}\n";
    src += "__device__ __forceinline__ V fq_val(TIn x, const Consts &c, u32 &flags, u32 live) {\n" + val_body + "}\n";
    const uint32_t m = L.mask;
    src += "#define BM_U " + std::to_string(block_mode_vectors()) + "\n";
    src += "struct Acc { V sum, mx, mn; u64 cnt; u32 flags; };\n";
    src += "__device__ __forceinline__ u32 fq_acc(Acc &acc, TIn x, long long idx, u32 live, const Consts &c,\n"
           "                                      const u64 *__restrict__ bitmap) {\n"
           "    u32 pass = live;\n";
    if (expr_pred) src += "    pass &= fq_pred(x, c, acc.flags, live) ? 1u : 0u;\n";
    else if (pk == FQ_PRED_BITMAP)
        src += "    if (live) pass &= (u32)((bitmap[idx >> 6] >> (idx & 63)) & 1ull);\n";
    src += "    (void)idx; (void)bitmap;\n    const V v = fq_val(x, c, acc.flags, pass);\n";
    if (m & FQ_AGG_SUM) src += "    acc.sum = acc.sum + (pass ? v : V(0));\n";
    if (m & FQ_AGG_MAX) src += "    acc.mx = pass ? vmax(acc.mx, v) : acc.mx;\n";
    if (m & FQ_AGG_MIN) src += "    acc.mn = pass ? vmin(acc.mn, v) : acc.mn;\n";
    src += "    acc.cnt += pass;\n    return pass;\n}\n";

    // limits of V for the accumulator init (Lim<V> in fq_device.h)
    std::string lo, hi;
    if (L.vdtype == FQ_DT_UINT64) lo = "0ull", hi = "~0ull";
    else if (L.vdtype == FQ_DT_INT64) lo = "(-9223372036854775807ll - 1)", hi = "9223372036854775807ll";
    else lo = "-__builtin_huge_val()", hi = "__builtin_huge_val()";

    // reduce_and_store (fq_aggregate.hip): wave butterfly, LDS across the 4
    // waves; thread 0 returns the workgroup's Partial
    src += R"(
__device__ __forceinline__ Partial wg_reduce(Acc acc) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        acc.sum = acc.sum + shfl64(acc.sum, off);
        acc.mx = vmax(acc.mx, shfl64(acc.mx, off));
        acc.mn = vmin(acc.mn, shfl64(acc.mn, off));
        acc.cnt += shfl64(acc.cnt, off);
        acc.flags |= (u32)__shfl_xor((int)acc.flags, off, 64);
    }
    __shared__ V s_sum[4], s_mx[4], s_mn[4];
    __shared__ u64 s_cnt[4];
    __shared__ u32 s_flags[4];
    const int wave = threadIdx.x / 64;
    if ((threadIdx.x & 63) == 0) {
        s_sum[wave] = acc.sum; s_mx[wave] = acc.mx; s_mn[wave] = acc.mn;
        s_cnt[wave] = acc.cnt; s_flags[wave] = acc.flags;
    }
    __syncthreads();
    Partial p;
    if (threadIdx.x == 0) {
        V sum = s_sum[0], mx = s_mx[0], mn = s_mn[0];
        u64 cnt = s_cnt[0];
        u32 flags = s_flags[0];
#pragma unroll
        for (int w = 1; w < 4; ++w) {
            sum = sum + s_sum[w]; mx = vmax(mx, s_mx[w]); mn = vmin(mn, s_mn[w]);
            cnt += s_cnt[w]; flags |= s_flags[w];
        }
        p.sum = __builtin_bit_cast(u64, sum); p.max = __builtin_bit_cast(u64, mx); p.min = __builtin_bit_cast(u64, mn);
        p.count = cnt; p.blocks = 0; p.flags = flags; p.dtype = )" + std::to_string(L.vdtype) + R"(;
    }
    return p;
}
)";
    src += "extern \"C\" __global__ void __launch_bounds__(256)\n"
           "fq_jit_scan(const TIn *__restrict__ col, long long n, long long head, long long R,\n"
           "            const u64 *__restrict__ bitmap, Consts c, Partial *parts) {\n"
           "    Acc acc;\n    acc.sum = V(0); acc.mx = " + lo + "; acc.mn = " + hi + "; acc.cnt = 0; acc.flags = 0;\n";
    if (!L.block_mode) {
        // flat tile-contiguous streaming (agg_flat_kernel, U = 4 16-byte vectors per lane)
        src += R"(
    (void)R;
    const long long T = (long long)gridDim.x * 256;
    const long long g = (long long)blockIdx.x * 256 + threadIdx.x;
    const long long nvec = (n - head) / 2;
    const u32x4 *__restrict__ vp = (const u32x4 *)(col + head);
    const long long TV = 4 * 256;
    const long long ntiles = nvec / TV;
    // next tile's loads in flight while this tile is evaluated
    u32x4 nxt[4];
    if ((long long)blockIdx.x < ntiles) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            nxt[k] = __builtin_nontemporal_load(vp + (long long)blockIdx.x * TV + threadIdx.x + (long long)k * 256);
    }
    for (long long t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const long long base = t * TV + threadIdx.x;
        u32x4 raw[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) raw[k] = nxt[k];
        const long long tn = t + gridDim.x;
        if (tn < ntiles) {
#pragma unroll
            for (int k = 0; k < 4; ++k) nxt[k] = __builtin_nontemporal_load(vp + tn * TV + threadIdx.x + (long long)k * 256);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            TIn x[2];
            __builtin_memcpy(&x[0], &raw[k], 16);
            const long long i0 = head + (base + (long long)k * 256) * 2;
            fq_acc(acc, x[0], i0, 1u, c, bitmap);
            fq_acc(acc, x[1], i0 + 1, 1u, c, bitmap);
        }
    }
    for (long long v = ntiles * TV + g; v < nvec; v += T) {
        const u32x4 raw = __builtin_nontemporal_load(vp + v);
        TIn x[2];
        __builtin_memcpy(&x[0], &raw, 16);
        fq_acc(acc, x[0], head + v * 2, 1u, c, bitmap);
        fq_acc(acc, x[1], head + v * 2 + 1, 1u, c, bitmap);
    }
    const long long tail0 = head + nvec * 2;
    const long long nedge = head + (n - tail0);
    for (long long t = g; t < nedge; t += T) {
        const long long i = t < head ? t : tail0 + (t - head);
        fq_acc(acc, col[i], i, 1u, c, bitmap);
    }
)";
    } else {
        // block mode (agg_block_kernel): one wave per reference block; with a
        // 16-byte-aligned column and an even block size every block starts
        // on a 16-byte boundary and is read with 16-byte loads (4 per lane in
        // flight), else with 8-byte loads (8 per lane)
        src += R"(
    (void)head;
    const int lane = threadIdx.x & 63;
    const long long w = ((long long)blockIdx.x * 256 + threadIdx.x) / 64;
    const long long W = ((long long)gridDim.x * 256) / 64;
    const long long nb = (n + R - 1) / R;
    const bool vec = ((((unsigned long long)col) & 15ull) == 0ull) && ((R & 1) == 0);
    for (long long b = w; b < nb; b += W) {
        const long long s = b * R;
        const long long e = (s + R < n) ? s + R : n;
        u32 any = 0;
        if (vec) {
            const long long nv = (e - s) >> 1;
            const u32x4 *__restrict__ bp = (const u32x4 *)(col + s);
            for (long long v = lane; v < nv; v += 64 * BM_U) {
                u32x4 raw[BM_U];
#pragma unroll
                for (int k = 0; k < BM_U; ++k) {
                    const long long vk = v + (long long)k * 64;
                    if (vk < nv) raw[k] = __builtin_nontemporal_load(bp + vk);
                    else raw[k] = u32x4{0u, 0u, 0u, 0u};
                }
#pragma unroll
                for (int k = 0; k < BM_U; ++k) {
                    const long long vk = v + (long long)k * 64;
                    const u32 li = vk < nv ? 1u : 0u;
                    TIn x[2];
                    __builtin_memcpy(&x[0], &raw[k], 16);
                    any |= fq_acc(acc, x[0], s + 2 * vk, li, c, bitmap);
                    any |= fq_acc(acc, x[1], s + 2 * vk + 1, li, c, bitmap);
                }
            }
            if (((e - s) & 1) && lane == 0) any |= fq_acc(acc, col[e - 1], e - 1, 1u, c, bitmap);
            if (__ballot(any != 0) == 0ull) acc.flags |= )" + std::to_string(FQ_STATE_ANY_EMPTY) + R"(u;
            continue;
        }
        for (long long i = s + lane; i < e; i += 64 * 8) {
            TIn x[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const long long ik = i + (long long)k * 64;
                x[k] = ik < e ? __builtin_nontemporal_load(col + ik) : TIn(0);
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const long long ik = i + (long long)k * 64;
                any |= fq_acc(acc, x[k], ik, ik < e ? 1u : 0u, c, bitmap);
            }
        }
        if (__ballot(any != 0) == 0ull) acc.flags |= )" + std::to_string(FQ_STATE_ANY_EMPTY) + R"(u;
    }
)";
    }
    // this workgroup's partial (agg_finalize_kernel folds them, fq_aggregate.hip)
    src += R"JIT(
    const Partial p = wg_reduce(acc);
    if (threadIdx.x == 0) parts[blockIdx.x] = p;
}
)JIT";
    return true;
}


// ---------------------------------------------------------------------------
// GROUP BY (fq_group_aggregate).  Same streaming loop as the scan; each
// passing row computes its key and arguments, updates a workgroup-private
// LDS hash table (ds_cmpst_b64 to claim a slot, LDS atomics for the states)
// and, when its key finds no LDS slot within kLdsProbe probes, the HBM table
// directly.  At the end each workgroup flushes its LDS groups into the HBM
// table (one global insert + one atomic per state per group).  HBM keys go
// EMPTY -> key once, so a relaxed (possibly stale) read followed by a CAS is
// enough to find or claim a slot across XCDs.
// ---------------------------------------------------------------------------

// Fixed by round-1/2 sweeps (their knobs were removed in round 6):
// LDS slot hash keeps consecutive keys in consecutive slots (1; 0 = Fibonacci
// hash of the whole key, profiles/r01_groupby_sweep_hash.txt); the HBM key
// probe reads plain before any CAS (1; r01_groupby_sweep_keyprobe.txt);
// wave-uniform key runs merged across the wave (1; r02_group_shapes.txt)
constexpr int group_lds_local() { return 1; }
constexpr int group_key_plain() { return 1; }
constexpr int group_wave_runs() { return 1; }

// clustered-key row layout of the GROUP BY kernel (mode 1 in fq_jit_groupby):
// chosen per workgroup from its first tile when a wave's 512 rows change key
// at most this often (default 160: runs of ~4+ rows), 0 = never
// (FQ_TUNE_GROUP_CLUSTER; tools/group_shapes_probe.py)
int group_cluster() { return (int)fqc::knob(FQ_TUNE_GROUP_CLUSTER); }

// GROUP BY tile order: 1 (default) = one contiguous run of tiles per
// workgroup, 0 = grid stride over tiles (FQ_TUNE_GROUP_CHUNKED; tools/
// group_shapes_probe.py: % 1000 keys 1.569 -> 1.531 ms per 10 GB, % 4093
// 1.656 -> 1.605)
int group_chunked() { return (int)fqc::knob(FQ_TUNE_GROUP_CHUNKED); }

int lds_slots(int n_aggs, int budget) {
    int s = 16384;
    while (s > 64 && (int64_t)s * 8 * (1 + n_aggs) > budget) s >>= 1;
    return s;
}

// Dense keys: a UInt64 key whose last step is `% d` by a constant d <= S
// lies in [0, d), so its LDS slot IS the key -- no hash, no probe, no claim
// (1 for the shape; d goes with the launch, so d > S takes the hashed shape)
}  // namespace

int64_t group_key_range(const KProg &key, int32_t key_dtype) {
    if (key_dtype != FQ_DT_UINT64 || key.n < 1) return 0;
    const KStep &st = key.s[key.n - 1];
    if (st.operand != FQ_OPERAND_CONST || st.reversed || st.dtype != FQ_DT_UINT64) return 0;
    uint64_t d = 0;
    if (st.code == K_AND_U) d = st.magic + 1;
    else if (st.code == K_MODM32_U || st.code == K_MODM_U) d = st.c;
    else return 0;
    return d >= 1 && d <= (uint64_t)INT64_MAX ? (int64_t)d : 0;
}

int group_lds_slots(int n_aggs, int lds_bytes) { return lds_slots(n_aggs, lds_bytes); }

int64_t group_dense_bound(const KProg &key, int32_t key_dtype, int n_aggs, int lds_bytes) {
    const int64_t d = group_key_range(key, key_dtype);
    return (d >= 1 && d <= (int64_t)lds_slots(n_aggs, lds_bytes)) ? d : 0;
}

namespace {
int dense_of(const GroupLaunch &G) {
    return group_dense_bound(G.key, G.key_dtype, G.n_aggs, G.lds_bytes) > 0 ? 1 : 0;
}

struct HostGroupConsts {
    uint64_t rhs;
    HostStep p[kSteps], k[kSteps], v[FQ_MAX_GROUP_AGGS][kSteps];
    uint64_t rl[FQ_MAX_PRED_LEAVES];
    HostStep pl[FQ_MAX_PRED_LEAVES][kSteps];
};

void pack_group_consts(const GroupLaunch &G, HostGroupConsts &hc) {
    hc.rhs = G.pred.rhs;
    for (int i = 0; i < kSteps; ++i) {
        hc.p[i] = HostStep{G.pred.lhs.s[i].c, G.pred.lhs.s[i].magic, G.pred.lhs.s[i].shift};
        hc.k[i] = HostStep{G.key.s[i].c, G.key.s[i].magic, G.key.s[i].shift};
        for (int a = 0; a < FQ_MAX_GROUP_AGGS; ++a)
            hc.v[a][i] = HostStep{G.vals[a].s[i].c, G.vals[a].s[i].magic, G.vals[a].s[i].shift};
    }
    pack_tree_consts(G.pred, hc);
}

// Range bins over 4-byte rows store each row straight from its registers, which
// coalesces when a wave's consecutive rows share a bin: keys that advance by at
// most 16 per row (adds, subtractions and divisions by constants, small
// multipliers, then the `% d` or `& m`).  Other key programs stage the tile in
// LDS sorted by bin.  Resident numbers_mt(1e10) through the engine
// (profiles/r04_o_group_key_shapes*.jsonl): `(number * 7919) % 100000` 84.7 ms
// per query with direct stores, 62.8 staged; `(number / 3) % 100000` 58.4
// direct, 62.8 staged.
bool group_stage_narrow(const GroupLaunch &G) {
    if (!G.narrow || !G.range_bins) return false;
    for (int i = 0; i + 1 < G.key.n; ++i) {
        const KStep &st = G.key.s[i];
        if (st.operand != FQ_OPERAND_CONST || st.reversed) return true;
        switch (st.code) {
            case K_ADD_I: case K_SUB_I: case K_DIV_U: case K_SHR_U: case K_DIVM_U: case K_DIVM32_U: break;
            case K_MUL_I: if (st.c > 16) return true; break;
            default: return true;
        }
    }
    return false;
}

std::string group_shape_key(const GroupLaunch &G, int32_t tin, int dev) {
    std::string k = "G" + std::to_string(group_lds_local()) + std::to_string(group_key_plain()) +
                    std::to_string(group_chunked()) + std::to_string(group_wave_runs()) +
                    std::to_string(group_cluster()) + "s" + std::to_string(group_stage_narrow(G) ? 1 : 0);
    auto put = [&k](int32_t v) { k.append(reinterpret_cast<const char *>(&v), sizeof v); };
    auto prog = [&put](const KProg &p) {
        put(p.n);
        for (int i = 0; i < p.n; ++i) {
            put(p.s[i].code);
            put(p.s[i].operand);
            put(p.s[i].reversed);
            put(p.s[i].dtype);
            put((int32_t)p.s[i].add);
            put(p.s[i].sdtype);
        }
    };
    put(dev);
    put(tin);
    put(G.key_dtype);
    put_pred_key(G.pred, k);
    prog(G.key);
    put(G.lds_bytes);
    put(dense_of(G));
    put(G.threads);
    put(G.rowmap);
    put(G.range_bins);
    put(G.narrow);
    put(G.n_aggs);
    for (int a = 0; a < G.n_aggs; ++a) {
        put(G.kinds[a]);
        put(G.dtypes[a]);
        put(G.chain[a] ? 1 : 0);
        if (G.chain[a]) prog(G.vals[a]);
    }
    return k;
}

// state update snippets: `P` = pointer expression, `v` = value of type Vi
std::string state_update(int32_t kind, int32_t dt, const std::string &P, const std::string &v) {
    const char *T = dt == FQ_DT_INT64 ? "long long" : (dt == FQ_DT_FLOAT64 ? "double" : "unsigned long long");
    switch (kind) {
        case FQ_AGG_COUNT:  // v = the rows to count ("" = one)
            return "atomicAdd((unsigned long long *)(" + P + "), " + (v.empty() ? std::string("1ull") : "(unsigned long long)(" + v + ")") + ");";
        case FQ_AGG_SUM:
            if (dt == FQ_DT_FLOAT64) return "atomicAdd((double *)(" + P + "), " + v + ");";
            return "atomicAdd((unsigned long long *)(" + P + "), (unsigned long long)(" + v + "));";
        case FQ_AGG_MAX:
            if (dt == FQ_DT_FLOAT64) return "amax_f64((u64 *)(" + P + "), " + v + ");";
            return std::string("atomicMax((") + T + " *)(" + P + "), (" + T + ")(" + v + "));";
        default:
            if (dt == FQ_DT_FLOAT64) return "amin_f64((u64 *)(" + P + "), " + v + ");";
            return std::string("atomicMin((") + T + " *)(" + P + "), (" + T + ")(" + v + "));";
    }
}

// High-cardinality GROUP BY (fq_group_aggregate_partitioned): more groups
// than an LDS table holds make every row an HBM atomic (100,000 groups x 3
// aggregates: 149 ms per 10 GB).  Instead the passing rows are radix-
// partitioned by key (range or hash) into P = 2^log2p bins, then aggregated
// bin by bin, so every workgroup's LDS table only sees the groups of one bin:
//   fq_jit_gpart   read the column once, LDS counting sort of each 8,192-row
//                  tile by bin; each (workgroup, bin) appends its run to a
//                  chain of GP_BLK-row blocks taken from the workgroup's own
//                  region of the workspace (an LDS counter: no histogram
//                  pass, no global atomic per tile -- one shared counter put
//                  ~2 us of cross-XCD atomic latency on every tile);
//   (blocks)       the blocks grouped by bin, fq_groupby.hip (a P-bin scan
//                  and a scatter of ~rows/256 block numbers);
//   fq_jit_groupby_bins  the blocks split evenly over the workgroups, cut at
//                  bin boundaries: LDS table per bin slice, flushed to the HBM
//                  table (whose home slot is the mixer's top bits, so a bin's
//                  groups share 1/P of the table).
// HBM bytes per passing row: 8 (read) + 8 (blocks written) + 8 (blocks read)
// = 24 B (8 B for a filtered-out one), against 8 B + 3 random atomics; the
// histogram pass this replaces read the column once more (32 B per row).
// With GP_NARROW (FQ_GROUP_NARROW_ROWS: the caller vouches that every value
// lies within 2^31 of col[0], as a numbers_mt block's do) the blocks hold
// 4-byte offsets from col[0] - 2^31: 8 + 4 + 4 = 16 B per passing row; a
// value outside the range sets flag 1024 and the launch reports it.
const char *kGroupPartitionKernels = R"GP(
#ifndef GP_ROWS
#define GP_ROWS 8
#endif
#if GP_NARROW
typedef u32 PRow;  // a kept row in the blocks: its offset from col[0] - 2^31
__device__ __forceinline__ u64 gp_vbase(const TIn *__restrict__ col) { return (u64)col[0] - 0x80000000ull; }
__device__ __forceinline__ PRow gp_pack(TIn x, u64 vbase, u32 &flags) {
    const u64 d = (u64)x - vbase;
    if (d >> 32) flags |= 1024u;
    return (PRow)d;
}
__device__ __forceinline__ TIn gp_unpack(PRow v, u64 vbase) { return (TIn)(vbase + (u64)v); }
// 4-byte rows: plain accesses (GP_NT_NARROW 1: non-temporal, as the 8-byte rows)
#ifndef GP_NT_NARROW
#define GP_NT_NARROW 0
#endif
__device__ __forceinline__ void gp_store(PRow *p, PRow v) {
#if GP_NT_NARROW
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}
__device__ __forceinline__ PRow gp_fetch(const PRow *p) {
#if GP_NT_NARROW
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}
#else
typedef TIn PRow;
__device__ __forceinline__ u64 gp_vbase(const TIn *__restrict__) { return 0; }
__device__ __forceinline__ PRow gp_pack(TIn x, u64, u32 &) { return x; }
__device__ __forceinline__ TIn gp_unpack(PRow v, u64) { return v; }
__device__ __forceinline__ void gp_store(PRow *p, PRow v) { __builtin_nontemporal_store(v, p); }
__device__ __forceinline__ PRow gp_fetch(const PRow *p) { return __builtin_nontemporal_load(p); }
#endif
#define GP_TILE (BT * GP_ROWS)
// Staging a tile's rows in LDS sorted by bin makes every store of a run
// coalesced whatever the key order; range bins over 4-byte rows (numbers_mt
// blocks: consecutive values, so a wave's rows share a bin and gp_rank hands
// out consecutive places) store straight from the registers instead.  8-byte
// rows are any column: random keys put a wave's 64 rows in ~64 bins, and the
// direct stores ran gpart at 15.5 ms per 4.2e8 random rows (r04_d_g2_random)
#ifndef GP_STAGE
#if RANGE_BINS && GP_NARROW
#define GP_STAGE 0
#else
#define GP_STAGE 1
#endif
#endif
#define GP_TBLK (GP_TILE / GP_BLK)
// rows per thread of the partition pass's tiles
#ifndef GPR_ROWS
#define GPR_ROWS GP_ROWS
#endif
#define GPR_TILE (BT * GPR_ROWS)
#define GP_NOBIN 0xffffu
// The kernels' log2p argument carries the bin shift of range bins in bits
// 8..15: keys in [0, d), d <= P << shift, 2^shift <= S: bin b holds the keys
// [b << shift, (b + 1) << shift), so its LDS table is indexed by the key's
// low bits (no hash, probe or claim)
#if RANGE_BINS
__device__ __forceinline__ u32 gbin(u64 k, int lpa) { return (u32)(k >> (lpa >> 8)); }
#else
__device__ __forceinline__ u32 gbin(u64 k, int lpa) { return (u32)(mix(k) >> (64 - (lpa & 255))); }
#endif
__device__ __forceinline__ u32 wave_or32(u32 f) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) f |= (u32)__shfl_xor((int)f, off, 64);
    return f;
}

// Bin ranks: with range bins consecutive keys share a bin, so a wave's
// passing lanes usually all hit one counter -- one LDS atomic for the wave
// (ranks = its base + the lane's place among them) instead of 64 serialised
// ones
__device__ __forceinline__ u32 gp_rank(u32 *cnt, u32 b, bool p) {
#if RANGE_BINS
    const u64 act = __ballot(p);
    if (!act) return 0u;
    const int lane = (int)(threadIdx.x & 63), l0 = __builtin_ctzll(act);
    const u32 b0 = (u32)__builtin_amdgcn_readlane((int)b, l0);
    if (__ballot(p && b == b0) == act) {
        u32 base = 0;
        if (lane == l0) base = atomicAdd(&cnt[b0], (u32)__popcll(act));
        base = (u32)__builtin_amdgcn_readlane((int)base, l0);
        return base + (u32)__popcll(act & ((1ull << lane) - 1ull));
    }
#endif
    return p ? atomicAdd(&cnt[b], 1u) : 0u;
}

#if GP_MOD32
// key = x % d for a 4-byte row: x = mbase + a with a < 2^32 (mbase = the
// narrow rows' base, or 0 when that base would wrap: the values then lie
// below 2^32), so x % d = (mbase % d + a % d) mod d, a % d by Lemire's direct
// remainder (M = floor((2^64 - 1) / d) + 1, exact for 32-bit a and d)
struct GMod { u64 mbase, M; u32 d, cb; };
__device__ __forceinline__ GMod gp_mod_init(u64 c0, const Consts &c) {
    GMod m;
    m.mbase = c0 >= 0x80000000ull ? c0 - 0x80000000ull : 0ull;
    m.d = (u32)c.k[0].c;
    m.M = 0xffffffffffffffffull / (u64)m.d + 1ull;
    m.cb = (u32)(m.mbase % (u64)m.d);
    return m;
}
__device__ __forceinline__ u32 gp_key32(TIn x, const GMod &m) {
    const u64 low = m.M * (u64)(u32)((u64)x - m.mbase);
    const u64 t = ((u64)(u32)low * m.d) >> 32;
    const u32 r = (u32)(((low >> 32) * m.d + t) >> 32);
    const u32 k = m.cb + r;  // cb, r < d: a sum >= d, or one that wrapped 32 bits, loses one d
    return k >= m.d || k < m.cb ? k - m.d : k;
}
#endif
__device__ __forceinline__ long long gp_row(long long tt, int k) {
    return tt * GPR_TILE + (long long)k * BT + threadIdx.x;
}
__device__ __forceinline__ void gp_load(const TIn *__restrict__ col, long long n, long long tt, TIn (&x)[GPR_ROWS]) {
    if ((tt + 1) * GPR_TILE <= n) {  // a whole tile: no per-row bound
        const TIn *p = col + gp_row(tt, 0);
#pragma unroll
        for (int k = 0; k < GPR_ROWS; ++k) x[k] = __builtin_nontemporal_load(p + k * BT);
        return;
    }
#pragma unroll
    for (int k = 0; k < GPR_ROWS; ++k) {
        const long long row = gp_row(tt, k);
        x[k] = row < n ? __builtin_nontemporal_load(col + row) : TIn(0);
    }
}

// Workgroup w owns blocks [w * q, (w + 1) * q): used[w] of them taken;
// bin_blocks[b]: blocks of bin b; blk_bin / blk_fill: each block's bin and
// rows (GP_BLK but for the last block of a chain)
// two 1,024-thread workgroups per CU = 8 waves per SIMD, which needs <= 80
// SGPRs (84 admit 7 waves: one workgroup, and the pass ran 1.1 -> 1.5 ms).
// Loading the next tile's rows into registers while this one is ranked and
// stored ran it 1.09 -> 1.81 ms per 4.2e8 narrow rows (64 VGPRs: spills);
// loading them into LDS by LDS-DMA instead measured within 1 % of the plain
// loads (round 3, profiles/r03_s3_g2_prefetch_ab.txt) and was removed.
#ifndef GPR_WAVES
#define GPR_WAVES (BT >= 1024 ? 8 : 1)
#endif
extern "C" __global__ void __launch_bounds__(BT) __attribute__((amdgpu_waves_per_eu(GPR_WAVES)))
fq_jit_gpart(const TIn *__restrict__ col, long long n, const u64 *__restrict__ bitmap, Consts c,
             u32 *__restrict__ used, u32 *__restrict__ bin_blocks, u32 *__restrict__ blk_bin,
             u32 *__restrict__ blk_fill, unsigned q, PRow *__restrict__ out, int log2p,
             u32 *__restrict__ hdr) {
    const u64 vbase = n > 0 ? gp_vbase(col) : 0ull;
#if GP_MOD32
    const GMod gm = gp_mod_init(n > 0 ? (u64)col[0] : 0ull, c);
#endif
#if GP_STAGE
    // a tile's passing rows sorted by bin in LDS, written out run by run
    __shared__ PRow s_stage[GPR_TILE];
    __shared__ unsigned char s_bin[GPR_TILE];
    __shared__ u32 s_start[256], s_tot;
#endif
    // per bin: this tile's rows, the chain's current block and its rows, the
    // first of the blocks taken for this tile, blocks taken in all.  GP_DBUF:
    // the counts and the chain state are double-buffered by tile parity --
    // the claims of tile t write the state tile t + 1 starts from and zero its
    // counts, so a tile takes two barriers instead of four (staged: three
    // instead of five)
#if GP_DBUF
    __shared__ u32 s_cnt2[2][256], s_blk2[2][256], s_fill2[2][256];
    int par = 0;
#define s_cnt (s_cnt2[par])
#define s_blk (s_blk2[par])
#define s_fill (s_fill2[par])
#else
    __shared__ u32 s_cnt[256], s_blk[256], s_fill[256];
#endif
    __shared__ u32 s_nb[256], s_nblk[256], s_next;
    // first block of the first failed claim (workspace overflow): claims are
    // handed out in increasing order, so every block below it was written and
    // none above it was; used[] stops there.  (An LDS atomic on every claim
    // instead cost 1.11 -> 1.77 ms per chunk: only the failure path pays.)
    __shared__ u32 s_fail;
    const int P = 1 << (log2p & 255);
    for (int i = threadIdx.x; i < P; i += BT) {
        s_blk[i] = 0xffffffffu;
        s_fill[i] = GP_BLK;  // full: the first row takes a block
        s_nblk[i] = 0;
#if GP_DBUF
        s_cnt2[0][i] = 0;
#endif
    }
    if (threadIdx.x == 0) {
        s_next = 0;
        s_fail = 0xffffffffu;
    }
    const u32 region = blockIdx.x * q;
    u32 flags = 0;
    const long long ntiles = (n + GPR_TILE - 1) / GPR_TILE;
#if GP_DBUF
    __syncthreads();
#endif
    for (long long tt = blockIdx.x; tt < ntiles; tt += gridDim.x) {
#if !GP_DBUF
        for (int i = threadIdx.x; i < P; i += BT) s_cnt[i] = 0;
        __syncthreads();
#endif
        TIn x[GPR_ROWS];
        gp_load(col, n, tt, x);
        // per row: bin | rank << 8 (P <= 256 bins, rank < GPR_TILE), one register instead of two
        u32 br[GPR_ROWS], pass = 0;
#if RANGE_BINS && GP_RANK_BATCH
        // bins of all rows first, then every row's rank atomic issued before
        // any return is read (one LDS round trip per tile, not one per row)
        // a row that does not pass holds bin GP_NOBIN, which no bin equals:
        // the wave's tests below are then one compare each
        const bool full = (tt + 1) * GPR_TILE <= n;  // no row past the end (the uniform common case)
#pragma unroll
        for (int k = 0; k < GPR_ROWS; ++k) {
            const long long row = gp_row(tt, k);
            u32 bk = GP_NOBIN;
            if (full || row < n) {
                Row r;
                fq_prep(x[k], row, c, bitmap, flags, r);
                if (r.pass) {
#if GP_MOD32
                    bk = gp_key32(x[k], gm) >> (u32)(log2p >> 8);
#else
                    bk = gbin(r.k, log2p);
#endif
                    pass |= 1u << k;
                }
            }
            br[k] = bk;
        }
        // per row k: when the wave's passing lanes share one bin (act = their
        // mask, b0 the bin), its first lane takes all their places with one
        // LDS atomic; every atomic is issued before any return is read
        u32 rv[GPR_ROWS], uni = 0;
#pragma unroll
        for (int k = 0; k < GPR_ROWS; ++k) {
            const u64 act = __builtin_amdgcn_ballot_w64(br[k] != GP_NOBIN);
            rv[k] = 0u;
            if (!act) continue;
            const int l0 = __builtin_ctzll(act);
            const u32 b0 = (u32)__builtin_amdgcn_readlane((int)br[k], l0);
            if (__builtin_amdgcn_ballot_w64(br[k] == b0) == act) {
                uni |= 1u << k;
                if ((int)(threadIdx.x & 63) == l0) rv[k] = atomicAdd(&s_cnt[b0], (u32)__popcll(act));
            } else if (br[k] != GP_NOBIN) {
                rv[k] = atomicAdd(&s_cnt[br[k]], 1u);
            }
        }
#pragma unroll
        for (int k = 0; k < GPR_ROWS; ++k) {
            u32 r = rv[k];
            if ((uni >> k) & 1u) {
                const u64 act = __builtin_amdgcn_ballot_w64(br[k] != GP_NOBIN);
                r = (u32)__builtin_amdgcn_readlane((int)r, __builtin_ctzll(act)) +
                    __builtin_amdgcn_mbcnt_hi((u32)(act >> 32), __builtin_amdgcn_mbcnt_lo((u32)act, 0u));
            }
            br[k] = (br[k] & 255u) | r << 8;
        }
#else
#pragma unroll
        for (int k = 0; k < GPR_ROWS; ++k) {
            const long long row = gp_row(tt, k);
            bool p = false;
            u32 bk = 0;
            if (row < n) {
                Row r;
                fq_prep(x[k], row, c, bitmap, flags, r);
                p = r.pass != 0;
                if (p) bk = gbin(r.k, log2p);
            }
            br[k] = bk | gp_rank(s_cnt, bk, p) << 8;
            if (p) pass |= 1u << k;
        }
#endif
        // the rows as the blocks hold them (4 bytes for numbers_mt blocks): the
        // 8-byte values are dead from here on
        PRow px[GPR_ROWS];
#pragma unroll
        for (int k = 0; k < GPR_ROWS; ++k) px[k] = ((pass >> k) & 1u) ? gp_pack(x[k], vbase, flags) : (PRow)0;
        __syncthreads();
#if GP_STAGE
        const int t0 = 64;  // these 64 threads scan the bin counts meanwhile
        if (threadIdx.x < 64) {  // exclusive scan of the P <= 256 bin counts: 4 per lane
            const int l = threadIdx.x;
            u32 v[4], t = 0;
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) {
                const int i = l * 4 + qq;
                v[qq] = i < P ? s_cnt[i] : 0u;
                t += v[qq];
            }
            u32 incl = t;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const u32 y = (u32)__shfl_up((int)incl, o, 64);
                if (l >= o) incl += y;
            }
            u32 run = incl - t;
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) {
                const int i = l * 4 + qq;
                if (i < P) s_start[i] = run;
                run += v[qq];
            }
            if (l == 63) s_tot = incl;
        }
#else
        const int t0 = 0;  // every thread takes blocks (no tile scan)
#endif
        // the blocks this tile's run of bin b spills into, consecutive numbers
        // from the workgroup's region; bin b's chain is kept by thread t0 + b
        // (mod BT - t0) throughout
        if ((int)threadIdx.x >= t0) {
            for (int b = (int)threadIdx.x - t0; b < P; b += BT - t0) {
                const u32 cnt = s_cnt[b], f = s_fill[b];
#if GP_DBUF
                s_cnt2[par ^ 1][b] = 0;
                if (!cnt || f + cnt <= GP_BLK) {
                    s_fill2[par ^ 1][b] = f + cnt;
                    s_blk2[par ^ 1][b] = s_blk[b];
                    continue;
                }
#else
                if (!cnt || f + cnt <= GP_BLK) continue;
#endif
                const u32 need = (f + cnt - 1) / GP_BLK;
                u32 base = atomicAdd(&s_next, need);
                if (base + need > q) {  // cannot happen within the region bound; never write past it
                    flags |= 512u;
                    atomicMin(&s_fail, base);
                    base = 0xffffffffu;
                } else {
                    base += region;
                    for (u32 j = 0; j < need; ++j) {
                        blk_bin[base + j] = (u32)b;
                        blk_fill[base + j] = GP_BLK;
                    }
                    s_nblk[b] += need;
                }
                s_nb[b] = base;
#if GP_DBUF
                s_blk2[par ^ 1][b] = base == 0xffffffffu ? 0xffffffffu : base + need - 1u;
                s_fill2[par ^ 1][b] = f + cnt - need * GP_BLK;
#endif
            }
        }
        __syncthreads();
#if !GP_STAGE
        {
            // range bins over running keys: straight from the registers -- a
            // wave's passing lanes mostly hold consecutive ranks of one bin
            // (gp_rank), so the stores coalesce without the staging (one
            // barrier and a per-row LDS round trip less)
            // every row's two LDS reads are issued before any is waited on (a
            // row that does not pass reads bin 255's entries, unused)
            u32 o[GPR_ROWS], blk[GPR_ROWS];
#pragma unroll
            for (int k = 0; k < GPR_ROWS; ++k) o[k] = s_fill[br[k] & 255u] + (br[k] >> 8);
#pragma unroll
            for (int k = 0; k < GPR_ROWS; ++k) {
                const u32 b = br[k] & 255u;
                blk[k] = *(o[k] < GP_BLK ? &s_blk[b] : &s_nb[b]);
            }
#pragma unroll
            for (int k = 0; k < GPR_ROWS; ++k) {
                if (!((pass >> k) & 1u) || blk[k] == 0xffffffffu) continue;  // (0xffffffff: workspace overflow, reported)
                const u32 bb = o[k] < GP_BLK ? blk[k] : blk[k] + o[k] / GP_BLK - 1u;
                gp_store(out + (long long)bb * GP_BLK + (o[k] & (GP_BLK - 1)), px[k]);
            }
        }
#else
        {
            // rows sorted by bin in LDS, then written run by run: consecutive
            // threads store consecutive rows of one bin's chain
#pragma unroll
            for (int k = 0; k < GPR_ROWS; ++k) {
                if (!((pass >> k) & 1u)) continue;
                const u32 pos = s_start[br[k] & 255u] + (br[k] >> 8);
                s_stage[pos] = px[k];
                s_bin[pos] = (unsigned char)(br[k] & 255u);
            }
            __syncthreads();
            const u32 kept = s_tot;
            for (u32 i = threadIdx.x; i < kept; i += BT) {
                const u32 b = s_bin[i];
                const u32 o = s_fill[b] + (i - s_start[b]);  // place in the chain from its current block
                u32 blk = o < GP_BLK ? s_blk[b] : s_nb[b];
                if (blk == 0xffffffffu) continue;  // (workspace overflow, reported)
                if (o >= GP_BLK) blk += o / GP_BLK - 1u;
                gp_store(out + (long long)blk * GP_BLK + (o & (GP_BLK - 1)), s_stage[i]);
            }
        }
#endif
#if GP_DBUF
        par ^= 1;  // the claims above wrote the next tile's state
#else
        __syncthreads();
        for (int b = threadIdx.x; b < P; b += BT) {
            const u32 cnt = s_cnt[b], t = s_fill[b] + cnt;
            if (!cnt) continue;
            if (t > GP_BLK) {
                const u32 need = (t - 1) / GP_BLK;
                s_blk[b] = s_nb[b] == 0xffffffffu ? 0xffffffffu : s_nb[b] + need - 1u;
                s_fill[b] = t - need * GP_BLK;
            } else {
                s_fill[b] = t;
            }
        }
#endif
    }
    __syncthreads();
    for (int b = (int)threadIdx.x; b < P; b += BT) {
        if (s_blk[b] != 0xffffffffu) blk_fill[s_blk[b]] = s_fill[b];
        if (s_nblk[b]) atomicAdd(&bin_blocks[b], s_nblk[b]);
    }
    if (threadIdx.x == 0) used[blockIdx.x] = min(min(s_next, q), s_fail);
    flags = wave_or32(flags);
    if ((threadIdx.x & 63) == 0 && flags) atomicOr(&hdr[0], flags);
#if GP_DBUF
#undef s_cnt
#undef s_blk
#undef s_fill
#endif
}

// rows of tile ti of a bin slice: row j of the tile is row j % GP_BLK of the
// slice's block ti * GP_TBLK + j / GP_BLK (a wave's 64 rows lie in one block:
// 512 contiguous bytes), whose order entry (block | rows << 32) is staged in
// LDS with those of the next GP_ORD_TILES - 1 tiles: the row loads wait on
// LDS, not on a dependent HBM load
#define GP_ORD 1024
#define GP_ORD_TILES (GP_ORD / GP_TBLK)
#ifndef GB_PREFETCH
#define GB_PREFETCH 1
#endif
__device__ __forceinline__ u32 gb_load(const PRow *__restrict__ vals, u64 vbase, const u64 *s_ord, long long ti,
                                       TIn (&x)[GP_ROWS]) {
    u32 live = 0;
    const int t0 = (int)(ti % GP_ORD_TILES) * GP_TBLK;
#if GP_NARROW
    // four adjacent 4-byte rows per lane and load: 16-byte accesses (one
    // 4-byte row per lane per load ran the pass 0.60 -> 1.04 ms per 4.2e8
    // rows, two per 8-byte load 0.71 ms; swapping rows across the wave so
    // consecutive lanes hold consecutive rows cost more than it saved).
    // Slot q of lane L takes the lane's row (q + L / 4) % 4: consecutive keys
    // 4 apart across lanes would put a 16-lane group's 8-byte LDS updates on
    // 4 bank pairs (4-way conflicts); rotated they cover all 16.
    const u32 rot = (threadIdx.x >> 2) & 3u;
#pragma unroll
    for (int k = 0; k < GP_ROWS / 4; ++k) {
        const int j = 4 * (k * BT + (int)threadIdx.x);  // this lane's first row
        const int off = j & (GP_BLK - 1);
        const u64 ent = s_ord[t0 + j / GP_BLK];
        const u32 fill = (u32)(ent >> 32);
        u32x4 four = {0u, 0u, 0u, 0u};
        if ((u32)off < fill) four = __builtin_nontemporal_load((const u32x4 *)(vals + (long long)(u32)ent * GP_BLK + off));
        const u32x4 r1 = (rot & 1u) ? u32x4{four[1], four[2], four[3], four[0]} : four;
        const u32x4 r2 = (rot & 2u) ? u32x4{r1[2], r1[3], r1[0], r1[1]} : r1;
        const u32 nl = (u32)off < fill ? fill - (u32)off : 0u;  // live rows from off (>= 4: all)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const bool lv = ((q + rot) & 3u) < nl;
            x[4 * k + q] = lv ? gp_unpack(r2[q], vbase) : TIn(0);
            live |= (lv ? 1u : 0u) << (4 * k + q);
        }
    }
#else
#pragma unroll
    for (int k = 0; k < GP_ROWS; ++k) {
        const int j = k * BT + (int)threadIdx.x;
        const int off = j & (GP_BLK - 1);
        const u64 ent = s_ord[t0 + j / GP_BLK];
        x[k] = TIn(0);
        if ((u32)off < (u32)(ent >> 32)) {
            x[k] = gp_unpack(gp_fetch(vals + (long long)(u32)ent * GP_BLK + off), vbase);
            live |= 1u << k;
        }
    }
#endif
    return live;
}
__device__ __forceinline__ void gb_stage(u64 *s_ord, const u64 *__restrict__ order, long long lo, long long e,
                                         long long ti) {
    const long long b0 = lo + ti * GP_TBLK;
    for (int i = threadIdx.x; i < GP_ORD; i += BT) s_ord[i] = b0 + i < e ? order[b0 + i] : 0ull;
}

extern "C" __global__ void __launch_bounds__(BT)
fq_jit_groupby_bins(const PRow *__restrict__ vals, const u64 *__restrict__ order, const u32 *__restrict__ bstart,
                    int log2p, Consts c, Tab t, const TIn *__restrict__ col) {
    const u64 vbase = gp_vbase(col);  // the launch has rows, so col[0] exists
#if GP_MOD32
    const GMod gm = gp_mod_init((u64)col[0], c);
#endif
    __shared__ u64 s_keys[S];
    __shared__ u64 s_st[NA][S];
    __shared__ int s_bypass[2];
    __shared__ u64 s_ord[GP_ORD];
    Tab tr = t;
    const long long roff = (long long)(blockIdx.x & t.rmask) * (t.mask + 2);
    for (int a = 0; a < NA; ++a) tr.st[a] += roff;
    const int P = 1 << (log2p & 255);
    const long long total = (long long)bstart[P];
    // this workgroup's even share of the blocks, cut at bin boundaries
    const long long per = (total + gridDim.x - 1) / gridDim.x;
    long long lo = (long long)blockIdx.x * per;
    const long long hi = lo + per < total ? lo + per : total;
    int p = 0;
    while (p < P && (long long)bstart[p + 1] <= lo) ++p;
    u32 flags = 0;
    while (lo < hi && p < P) {
        const long long e = (long long)bstart[p + 1] < hi ? (long long)bstart[p + 1] : hi;
        if (e > lo) {
            fq_lds_reset(s_keys, s_st, s_bypass);
            gb_stage(s_ord, order, lo, e, 0);
            __syncthreads();
            // blocks [lo, e) as tiles of GP_TBLK blocks; the next tile's
            // loads are in flight while this one goes through the LDS table
            const long long nt = (e - lo + GP_TBLK - 1) / GP_TBLK;
#if GB_PREFETCH
            TIn nxt[GP_ROWS];
            u32 nlive = gb_load(vals, vbase, s_ord, 0, nxt);
#endif
            for (long long ti = 0; ti < nt; ++ti) {
                TIn x[GP_ROWS];
#if GB_PREFETCH
#pragma unroll
                for (int k = 0; k < GP_ROWS; ++k) x[k] = nxt[k];
                const u32 live = nlive;
                if (ti + 1 < nt) {
                    if ((ti + 1) % GP_ORD_TILES == 0) {  // (uniform) the next GP_ORD entries
                        __syncthreads();
                        gb_stage(s_ord, order, lo, e, ti + 1);
                        __syncthreads();
                    }
                    nlive = gb_load(vals, vbase, s_ord, ti + 1, nxt);
                }
#else
                // (two workgroups per CU hide each other's loads)
                if (ti > 0 && ti % GP_ORD_TILES == 0) {  // (uniform) the next GP_ORD entries
                    __syncthreads();
                    gb_stage(s_ord, order, lo, e, ti);
                    __syncthreads();
                }
                const u32 live = gb_load(vals, vbase, s_ord, ti, x);
#endif
                Row r[GP_ROWS];
#pragma unroll
                for (int k = 0; k < GP_ROWS; ++k) {
                    fq_prep_all(x[k], (live >> k) & 1u, c, flags, r[k]);
#if GP_MOD32
                    r[k].k = gp_key32(x[k], gm);  // (the 64-bit key fq_prep_all computed is dead)
#endif
                }
                u32 cnt[GP_ROWS];
                fq_runs(r, cnt);
#if RANGE_BINS
#pragma unroll
                for (int j = 0; j < GP_ROWS; ++j) fq_commit_range(r[j], s_keys, s_st, (u64)cnt[j]);
#else
                u64 cur[GP_ROWS];
#pragma unroll
                for (int j = 0; j < GP_ROWS; ++j) cur[j] = fq_first(r[j], s_keys);
#pragma unroll
                for (int j = 0; j < GP_ROWS; ++j) fq_commit_lane(r[j], cur[j], tr, s_keys, s_st, s_bypass, (u64)cnt[j]);
#endif
            }
            __syncthreads();
            fq_flush(tr, s_keys, s_st, (u64)p << (log2p >> 8), (1ull << (log2p >> 8)) - 1ull);
            __syncthreads();
            lo = e;
        }
        ++p;
    }
    if (flags) atomicOr(&t.hdr[0], flags);
}
)GP";

bool gen_groupby_source(const GroupLaunch &G, int32_t tin, Gen &g, std::string &src, bool cluster = true) {
    const char *TIn = ctype(tin);
    if (!TIn || (G.key_dtype != FQ_DT_UINT64 && G.key_dtype != FQ_DT_INT64)) return false;
    if (G.n_aggs < 1 || G.n_aggs > FQ_MAX_GROUP_AGGS) return false;
    const int NA = G.n_aggs;
    const int S = lds_slots(NA, G.lds_bytes);
    src = kCommon;
    src += "typedef " + std::string(TIn) + " TIn;\n";
    src += "struct Step { u64 c, m, s; };\nstruct Consts { u64 rhs; Step p[" + std::to_string(kSteps) + "], k[" +
           std::to_string(kSteps) + "], v[" + std::to_string(FQ_MAX_GROUP_AGGS) + "][" + std::to_string(kSteps) +
           "]; u64 rl[" + std::to_string(FQ_MAX_PRED_LEAVES) + "]; Step pl[" + std::to_string(FQ_MAX_PRED_LEAVES) +
           "][" + std::to_string(kSteps) + "]; };\n";
    src += "struct Tab { u64 *keys; u64 *st[" + std::to_string(FQ_MAX_GROUP_AGGS) +
           "]; u32 *hdr; long long mask; int rmask; };\n";
    src += "#define BT " + std::to_string(G.threads) + "\n#define ROWMAP " + std::to_string(G.rowmap) + "\n";
    src += "#define LDS_LOCAL " + std::to_string(group_lds_local()) + "\n";
    src += "#define GKEY_PLAIN " + std::to_string(group_key_plain()) + "\n";
    src += "#define GCHUNK " + std::to_string(group_chunked()) + "\n";
    src += "#define GWAVE " + std::to_string(group_wave_runs()) + "\n";
    src += "#define RANGE_BINS " + std::to_string(G.range_bins ? 1 : 0) + "\n";
    src += "#define GP_NARROW " + std::to_string(G.narrow ? 1 : 0) + "\n";
    {
        // partition pass, range bins over 4-byte rows: a `% d` key (d < 2^32)
        // from the row's 32-bit offset, and the rows' rank atomics issued
        // together.  Per 4.2e8-row chunk of g2 on one box: 1.137 ms with
        // neither, 1.132 with the batched ranks alone, 1.136 with the 32-bit
        // key alone, 1.044 with both; the bins pass's key the same way: 0.566
        // -> 0.483 ms (profiles/r03_s4_gpart_ab.txt)
        const KStep &ks = G.key.s[0];
        const bool mod32 = G.narrow && G.range_bins && tin == FQ_DT_UINT64 && G.key.n == 1 &&
                           (ks.code == K_MODM_U || ks.code == K_MODM32_U) && ks.operand == FQ_OPERAND_CONST &&
                           !ks.reversed && ks.c >= 1 && ks.c <= 0xffffffffull;
        src += "#define GP_MOD32 " + std::to_string(mod32 ? 1 : 0) + "\n#define GP_RANK_BATCH 1\n";
        if (group_stage_narrow(G)) src += "#define GP_STAGE 1\n";
    }
    // Rows per thread per tile (round-4 sweeps, profiles/r04_m_gpart_rows4_ab/, r04_o_gbins_ab/): 8-byte rows
    // 8 in both passes (their 64 KB staging leaves no LDS for the double buffers); 4-byte rows 8 in the
    // partition pass (double-buffered tile state, two barriers per tile) and 4 in the bins pass, without the
    // next tile's loads in registers (54 VGPRs: room for a second workgroup per CU)
    if (G.narrow) src += "#define GP_ROWS 4\n#define GB_PREFETCH 0\n#define GPR_ROWS 8\n";
    src += std::string("#define GP_DBUF ") + (G.narrow ? "1" : "0") + "\n";
    // (range bins only: the hash bins' 72 KB staging leaves no LDS for it)
    // blocks are 2 KB either way: 256 8-byte rows, or 512 narrow ones (1 KB
    // blocks measured 1.11 -> 1.53 ms per 4.2e8-row partition pass)
    src += "#define GP_BLK " + std::to_string(kPartBlockRows * (G.narrow ? 2 : 1)) + "\n";
    src += "#define GCLUSTER " + std::to_string(cluster && group_cluster() > 0 && fqc::dtype_size(tin) == 8 &&
                                                          G.lds_bytes + G.threads * 16 <= 160 * 1024 ? 1 : 0) + "\n";
    src += "#define GCLUSTER_CHANGES " + std::to_string(group_cluster() > 0 ? group_cluster() : 160) + "\n";
    // dense keys (see dense_of): a COUNT state doubles as the slot's
    // occupancy, else the key is stored (a plain write, every writer writes
    // the same value)
    int dense_cnt = -1;
    for (int a = 0; a < NA && dense_cnt < 0; ++a)
        if (G.kinds[a] == FQ_AGG_COUNT) dense_cnt = a;
    src += "#define DENSE " + std::to_string(dense_of(G)) + "\n#define DENSE_CNT " + std::to_string(dense_cnt) + "\n";
    src += "#define PMAX 16\n#define EMPTY 0xffffffffffffffffull\n#define NA " + std::to_string(NA) + "\n#define S " +
           std::to_string(S) + "\n#define LOG2S " + std::to_string(__builtin_ctz((unsigned)S)) + "\n";
    src += R"(
template <int V> struct IC { static constexpr int value = V; };
__device__ __forceinline__ u64 mix(u64 z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
// LDS slot hash: one 32-bit multiply (Fibonacci hashing of the folded key),
// top bits kept; the HBM table keeps the full 64-bit mixer.  (An XOR-fold
// that keeps consecutive keys in consecutive slots measured no faster: a
// lane holds rows 2l and 2l+1, so a wave's keys are strided anyway.)
// key partition (independent of the LDS slot bits)
__device__ __forceinline__ u32 part_of(u64 k, u32 P) {
    return ((((u32)k ^ (u32)(k >> 32)) * 0x2545F491u) >> 26) & (P - 1);
}
__device__ __forceinline__ u32 lds_hash(u64 k) {
#if LDS_LOCAL
    // low LOG2S bits kept, the rest Fibonacci-hashed onto them: a wave's 64
    // consecutive keys land in 64 consecutive slots (no LDS bank conflicts),
    // keys that differ only above the table size still spread
    const u32 f = (u32)k ^ (u32)(k >> 32);
    return f + (((f >> LOG2S) * 0x9E3779B1u) >> (32 - LOG2S));
#else
    return (((u32)k ^ (u32)(k >> 32)) * 0x9E3779B1u) >> (32 - LOG2S);
#endif
}
__device__ __forceinline__ void amax_f64(u64 *p, double v) {
    u64 old = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (v > __builtin_bit_cast(double, old)) {
        const u64 prev = atomicCAS((unsigned long long *)p, old, __builtin_bit_cast(u64, v));
        if (prev == old) return;
        old = prev;
    }
}
__device__ __forceinline__ void amin_f64(u64 *p, double v) {
    u64 old = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (v < __builtin_bit_cast(double, old)) {
        const u64 prev = atomicCAS((unsigned long long *)p, old, __builtin_bit_cast(u64, v));
        if (prev == old) return;
        old = prev;
    }
}
// slot of key k in the HBM table (claiming an empty one), -1 if full
__device__ long long ginsert(const Tab &t, u64 k) {
    if (k == EMPTY) {
        atomicOr(&t.hdr[1], 1u);
        return t.mask + 1;
    }
    // home slot = the top log2(capacity) bits of the mixer, so the keys of
    // partition bin b (its top log2(P) bits, fq_jit_gpart) live in one
    // contiguous 1/P of the table
    long long h = (long long)(mix(k) >> __clzll(t.mask));
    for (long long p = 0; p <= t.mask; ++p) {
#if GKEY_PLAIN
        // a plain (L2-cached) read: a slot's key is written once (EMPTY ->
        // key), so a stale value can only be EMPTY, which the CAS below
        // resolves; a hit never needs the memory-side round trip
        const u64 cur = t.keys[h];
#else
        const u64 cur = __hip_atomic_load(&t.keys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
        if (cur == k) return h;
        if (cur == EMPTY) {
            const u64 old = atomicCAS((unsigned long long *)&t.keys[h], EMPTY, k);
            if (old == EMPTY) atomicAdd(&t.hdr[4], 1u);  // groups claimed (sizes later launches' partitions)
            if (old == EMPTY || old == k) return h;
        }
        h = (h + 1) & t.mask;
    }
    atomicOr(&t.hdr[0], 256u);
    return -1;
}
)";
    // predicate, key and value functions
    std::string body;
    if (G.pred.kind == FQ_PRED_EXPR || G.pred.kind == FQ_PRED_TREE) {
        if (!emit_pred_body(g, G.pred, tin, body)) return false;
    } else {
        body = "    return true;\n";
    }
    src += "__device__ __forceinline__ bool fq_pred(TIn x, const Consts &c, u32 &flags, u32 live) {\n" + body + "}\n";
    body.clear();
    emit_value_body(g, G.key.n ? &G.key : nullptr, tin, G.key_dtype, "k", "u64", body);
    src += "__device__ __forceinline__ u64 fq_key(TIn x, const Consts &c, u32 &flags, u32 live) {\n" + body + "}\n";
    for (int a = 0; a < NA; ++a) {
        if (G.kinds[a] == FQ_AGG_COUNT) continue;
        const char *V = ctype(G.dtypes[a]);
        if (!V) return false;
        body.clear();
        emit_value_body(g, G.chain[a] ? &G.vals[a] : nullptr, tin, G.dtypes[a],
                        ("v[" + std::to_string(a) + "]").c_str(), V, body);
        src += std::string("__device__ __forceinline__ ") + V + " fq_val" + std::to_string(a) +
               "(TIn x, const Consts &c, u32 &flags, u32 live) {\n" + body + "}\n";
    }
    // identity of each state (fq_groupby.hip initialises the HBM table the same way)
    auto identity = [](int32_t kind, int32_t dt) -> std::string {
        if (kind == FQ_AGG_COUNT || kind == FQ_AGG_SUM) return "0ull";
        if (dt == FQ_DT_UINT64) return kind == FQ_AGG_MAX ? "0ull" : "0xffffffffffffffffull";
        if (dt == FQ_DT_INT64) return kind == FQ_AGG_MAX ? "0x8000000000000000ull" : "0x7fffffffffffffffull";
        return kind == FQ_AGG_MAX ? "0xfff0000000000000ull" : "0x7ff0000000000000ull";  // -inf / +inf
    };
    // per-row work in two halves so a tile's 8 rows issue their first LDS
    // probe reads together (independent loads, one latency): fq_prep
    // evaluates predicate, key and arguments; fq_commit finds/claims the
    // slot and applies the states.
    std::string row = "struct Row { u64 k; int h; u32 pass;";
    for (int a = 0; a < NA; ++a)
        if (G.kinds[a] != FQ_AGG_COUNT) row += std::string(" ") + ctype(G.dtypes[a]) + " v" + std::to_string(a) + ";";
    row += " };\n";
    row += "__device__ __forceinline__ void fq_prep(TIn x, long long idx, const Consts &c,\n"
           "    const u64 *__restrict__ bitmap, u32 &flags, Row &r) {\n    r.pass = 1u;\n";
    if (G.pred.kind == FQ_PRED_EXPR || G.pred.kind == FQ_PRED_TREE)
        row += "    r.pass = fq_pred(x, c, flags, 1u) ? 1u : 0u;\n";
    else if (G.pred.kind == FQ_PRED_BITMAP) row += "    r.pass = (u32)((bitmap[idx >> 6] >> (idx & 63)) & 1ull);\n";
    row += "    (void)idx; (void)bitmap;\n    r.k = fq_key(x, c, flags, r.pass);\n";
    for (int a = 0; a < NA; ++a)
        if (G.kinds[a] != FQ_AGG_COUNT)
            row += "    r.v" + std::to_string(a) + " = fq_val" + std::to_string(a) + "(x, c, flags, r.pass);\n";
    row += "#if DENSE\n    r.h = (int)r.k;\n#else\n    r.h = (int)(lds_hash(r.k) & (u32)(S - 1));\n#endif\n}\n";
    // rows of the partitioned buffer already passed the predicate
    row += "__device__ __forceinline__ void fq_prep_all(TIn x, u32 live, const Consts &c, u32 &flags, Row &r) {\n"
           "    r.pass = live;\n    r.k = fq_key(x, c, flags, live);\n";
    for (int a = 0; a < NA; ++a)
        if (G.kinds[a] != FQ_AGG_COUNT)
            row += "    r.v" + std::to_string(a) + " = fq_val" + std::to_string(a) + "(x, c, flags, live);\n";
    row += "#if DENSE\n    r.h = (int)r.k;\n#else\n    r.h = (int)(lds_hash(r.k) & (u32)(S - 1));\n#endif\n}\n";
    row += "__device__ __forceinline__ u64 fq_first(const Row &r, const u64 *s_keys) {\n"
           "#if DENSE\n    (void)r; (void)s_keys;\n    return EMPTY;\n#else\n"
           "    return (r.pass && r.k != EMPTY) ? s_keys[r.h] : EMPTY;\n#endif\n}\n";
    row += "__device__ __forceinline__ void fq_commit_lane(const Row &r, u64 cur0, const Tab &t, u64 *s_keys,\n"
           "    u64 (*s_st)[S], int *s_bypass, u64 cnt) {\n    if (!r.pass) return;\n";
    row += "#if DENSE\n    (void)cur0; (void)t; (void)s_bypass;\n    const int slot = r.h;\n#if DENSE_CNT < 0\n"
           "    s_keys[slot] = r.k;\n#endif\n";
    for (int a = 0; a < NA; ++a)
        row += "    " + state_update(G.kinds[a], G.dtypes[a], "&s_st[" + std::to_string(a) + "][slot]",
                                     G.kinds[a] == FQ_AGG_COUNT ? "cnt" : "r.v" + std::to_string(a)) + "\n";
    row += "#else\n    const u64 k = r.k;\n";
    row += R"(    int slot = -1;
    if (k != EMPTY) {
        // Once the LDS table is 3/4 full (more groups than it holds) it stops
        // taking new keys: resident keys still aggregate in LDS, the others
        // go to HBM after a short probe (an empty slot proves absence: there
        // are no deletions).
        const bool full = *s_bypass != 0;
        const int maxp = full ? 4 : 16;
        int h = r.h;
#pragma unroll 1
        for (int p = 0; p < maxp; ++p) {
            const u64 cur = p == 0 ? cur0 : s_keys[h];
            if (cur == k) { slot = h; break; }
            if (cur == EMPTY) {
                if (full) break;
                const u64 old = atomicCAS((unsigned long long *)&s_keys[h], EMPTY, k);
                if (old == EMPTY) {
                    if (atomicAdd(s_bypass + 1, 1) + 1 >= S * 3 / 4) *s_bypass = 1;
                    slot = h;
                    break;
                }
                if (old == k) { slot = h; break; }
            }
            h = (h + 1) & (S - 1);
        }
    }
    if (slot >= 0) {
)";
    for (int a = 0; a < NA; ++a)
        row += "        " + state_update(G.kinds[a], G.dtypes[a], "&s_st[" + std::to_string(a) + "][slot]",
                                         G.kinds[a] == FQ_AGG_COUNT ? "cnt" : "r.v" + std::to_string(a)) + "\n";
    row += "    } else {\n        const long long gs = ginsert(t, k);\n        if (gs >= 0) {\n";
    for (int a = 0; a < NA; ++a)
        row += "            " + state_update(G.kinds[a], G.dtypes[a], "&t.st[" + std::to_string(a) + "][gs]",
                                             G.kinds[a] == FQ_AGG_COUNT ? "cnt" : "r.v" + std::to_string(a)) + "\n";
    row += "        }\n    }\n#endif\n}\n";
    // range bins (fq_jit_groupby_bins): the slot is the key's low LOG2S bits;
    // the key is stored for the flush (a plain write: every writer of a slot
    // writes the same key) -- unless a COUNT state marks the occupied slots,
    // when the flush rebuilds the key from the bin and the slot (one LDS
    // write per row less)
    row += "__device__ __forceinline__ void fq_commit_range(const Row &r, u64 *s_keys, u64 (*s_st)[S], u64 cnt) {\n"
           "    if (!r.pass) return;\n    const int slot = (int)(r.k & (u64)(S - 1));\n"
           "#if DENSE_CNT < 0\n    s_keys[slot] = r.k;\n#endif\n";
    for (int a = 0; a < NA; ++a)
        row += "    " + state_update(G.kinds[a], G.dtypes[a], "&s_st[" + std::to_string(a) + "][slot]",
                                     G.kinds[a] == FQ_AGG_COUNT ? "cnt" : "r.v" + std::to_string(a)) + "\n";
    row += "}\n";
    row += "__device__ __forceinline__ void fq_commit(const Row &r, u64 cur0, const Tab &t, u64 *s_keys,\n"
           "    u64 (*s_st)[S], int *s_bypass) {\n"
           "    fq_commit_lane(r, cur0, t, s_keys, s_st, s_bypass, 1ull);\n}\n";
    // Runs of equal keys among a lane's rows of one tile (clustered keys such
    // as number / 1000000: a lane's rows are 1,024 apart, so all of them
    // share a key) are merged in registers first and committed once: 64
    // lanes' LDS atomics on one address serialise otherwise (12 ms against
    // 1.6 ms per 10 GB, tools/group_shapes_probe.py).  cnt[j] = rows merged
    // into row j (0 for a row merged away or not passing).
    // (Only when some lane's first two rows share a key -- one compare and a
    // ballot per tile, so scattered keys skip the chain: `% 1000` keys 1.587
    // -> 1.556 ms per 10 GB.)
    row += "template <int N> __device__ __forceinline__ bool fq_runs(Row (&r)[N], u32 (&cnt)[N]) {\n"
           "#pragma unroll\n    for (int j = 0; j < N; ++j) cnt[j] = r[j].pass;\n"
           "    if (!__ballot(r[0].pass && r[1].pass && r[0].k == r[1].k)) return false;\n"
           "#pragma unroll\n    for (int j = N - 1; j > 0; --j) {\n"
           "        if (r[j].pass && r[j - 1].pass && r[j].k == r[j - 1].k) {\n";
    for (int a = 0; a < NA; ++a) {
        if (G.kinds[a] == FQ_AGG_COUNT) continue;
        const std::string A = std::to_string(a);
        row += "            r[j - 1].v" + A + " = " +
               (G.kinds[a] == FQ_AGG_SUM ? "r[j - 1].v" + A + " + r[j].v" + A
                                         : std::string(G.kinds[a] == FQ_AGG_MAX ? "vmax" : "vmin") + "(r[j - 1].v" + A +
                                               ", r[j].v" + A + ")") + ";\n";
    }
    row += "            cnt[j - 1] += cnt[j];\n            cnt[j] = 0;\n            r[j].pass = 0;\n        }\n    }\n    return true;\n}\n";
    // Runs of equal keys across a wave: a slot whose passing lanes (64
    // consecutive rows) all hold one key -- runs of 64+ rows, e.g.
    // (number / 1000) % 1000 -- is reduced across the wave in registers (DPP
    // within each 16-lane row, readlane across the four) and committed by one
    // lane; 64 lanes' LDS atomics on one slot serialise otherwise (12.2 ms
    // against 1.5 ms per 10 GB).  Gate per tile: lanes 0 and 63 of the first
    // or last slot share a key.
    row += R"(template <int C> __device__ __forceinline__ u32 dpp32(u32 v) {
    return (u32)__builtin_amdgcn_mov_dpp((int)v, C, 0xf, 0xf, false);
}
template <typename T, int C> __device__ __forceinline__ T dppT(T v) {
    if constexpr (sizeof(T) == 4) {
        return __builtin_bit_cast(T, dpp32<C>(__builtin_bit_cast(u32, v)));
    } else {
        const u64 b = __builtin_bit_cast(u64, v);
        return __builtin_bit_cast(T, ((u64)dpp32<C>((u32)(b >> 32)) << 32) | dpp32<C>((u32)b));
    }
}
template <typename T> __device__ __forceinline__ T rlane(T v, int l) {
    if constexpr (sizeof(T) == 4) {
        return __builtin_bit_cast(T, (u32)__builtin_amdgcn_readlane((int)__builtin_bit_cast(u32, v), l));
    } else {
        const u64 b = __builtin_bit_cast(u64, v);
        const u32 lo = (u32)__builtin_amdgcn_readlane((int)(u32)b, l), hi = (u32)__builtin_amdgcn_readlane((int)(u32)(b >> 32), l);
        return __builtin_bit_cast(T, ((u64)hi << 32) | lo);
    }
}
struct WSum { template <typename T> __device__ __forceinline__ T operator()(T a, T b) const { return a + b; } };
// NaN never wins, as with the HBM / LDS f64 max/min atomics (v > old)
struct WMax { template <typename T> __device__ __forceinline__ T operator()(T a, T b) const { return (b > a || a != a) ? b : a; } };
struct WMin { template <typename T> __device__ __forceinline__ T operator()(T a, T b) const { return (b < a || a != a) ? b : a; } };
// every lane's v combined; quad_perm xor 1, xor 2, row_ror 4, 8 -> each
// 16-lane row's total in every lane of it, then the four rows by readlane
template <typename T, typename OP> __device__ __forceinline__ T wave_all(T v, OP op) {
    v = op(v, dppT<T, 0xb1>(v));
    v = op(v, dppT<T, 0x4e>(v));
    v = op(v, dppT<T, 0x124>(v));
    v = op(v, dppT<T, 0x128>(v));
    return op(op(rlane(v, 0), rlane(v, 16)), op(rlane(v, 32), rlane(v, 48)));
}
// Up to GWAVE keys per slot (2: a run boundary inside the 64 rows) are
// merged; a key held by fewer than 8 passing lanes commits lane by lane.
template <int N> __device__ __forceinline__ void fq_wave_runs(Row (&r)[N], u32 (&cnt)[N]) {
    if (rlane(r[0].k, 0) != rlane(r[0].k, 63) && rlane(r[N - 1].k, 0) != rlane(r[N - 1].k, 63)) return;
    const int lane = (int)(threadIdx.x & 63);
#pragma unroll
    for (int j = 0; j < N; ++j) {
        u64 act = __ballot(r[j].pass != 0);
#pragma unroll
        for (int it = 0; it < GWAVE; ++it) {
        if (__popcll(act) < 8) break;
        const int l0 = __builtin_ctzll(act);
        const u64 kk = rlane(r[j].k, l0);
        const u64 same = __ballot(r[j].pass != 0 && r[j].k == kk);
        if (__popcll(same) < 8) break;
        act &= ~same;
        const bool in = (same >> lane) & 1ull;
        const u32 tot = wave_all(in ? cnt[j] : 0u, WSum());
)";
    for (int a = 0; a < NA; ++a) {
        if (G.kinds[a] == FQ_AGG_COUNT) continue;
        const std::string A = std::to_string(a), V = ctype(G.dtypes[a]);
        const char *op = G.kinds[a] == FQ_AGG_SUM ? "WSum()" : (G.kinds[a] == FQ_AGG_MAX ? "WMax()" : "WMin()");
        row += "        { const " + V + " w = wave_all(in ? r[j].v" + A + " : __builtin_bit_cast(" + V + ", (u64)" +
               identity(G.kinds[a], G.dtypes[a]) + "), " + op + ");\n          if (lane == l0) r[j].v" + A + " = w; }\n";
    }
    row += "        if (lane == l0) {\n            cnt[j] = tot;\n        } else if (in) {\n            cnt[j] = 0;\n"
           "            r[j].pass = 0;\n        }\n        }\n    }\n}\n";
    row += "__device__ __forceinline__ void fq_row(TIn x, long long idx, const Consts &c, const Tab &t,\n"
           "    const u64 *__restrict__ bitmap, u64 *s_keys, u64 (*s_st)[S], u32 &flags, int *s_bypass, u32 P,\n"
           "    u32 part) {\n"
           "    Row r;\n    fq_prep(x, idx, c, bitmap, flags, r);\n"
           "    if (P > 1 && part_of(r.k, P) != part) r.pass = 0;\n"
           "    fq_commit(r, fq_first(r, s_keys), t, s_keys, s_st, s_bypass);\n}\n";
    src += row;

    // LDS table reset and flush (every kernel that aggregates through LDS)
    src += "__device__ __forceinline__ void fq_lds_reset(u64 *s_keys, u64 (*s_st)[S], int *s_bypass) {\n"
           "    if (threadIdx.x < 2) s_bypass[threadIdx.x] = 0;\n"
           "    for (int i = threadIdx.x; i < S; i += BT) {\n        s_keys[i] = EMPTY;\n";
    for (int a = 0; a < NA; ++a)
        src += "        s_st[" + std::to_string(a) + "][i] = " + identity(G.kinds[a], G.dtypes[a]) + ";\n";
    src += "    }\n}\n";
    src += R"(// this workgroup's groups into the HBM table
// (range bins: the slice's keys are kbin | (slot & kmask))
__device__ __forceinline__ void fq_flush(const Tab &tr, const u64 *s_keys, u64 (*s_st)[S], u64 kbin = 0,
                                         u64 kmask = 0) {
    for (int i = threadIdx.x; i < S; i += BT) {
#if DENSE && DENSE_CNT >= 0
        if (s_st[DENSE_CNT][i] == 0) continue;
        const u64 k = (u64)i;
#elif RANGE_BINS && DENSE_CNT >= 0
        if (s_st[DENSE_CNT][i] == 0) continue;
        const u64 k = kbin | ((u64)i & kmask);
#else
        const u64 k = s_keys[i];
        if (k == EMPTY) continue;
#endif
        const long long gs = ginsert(tr, k);
        if (gs < 0) continue;
)";
    for (int a = 0; a < NA; ++a) {
        const std::string sa = "s_st[" + std::to_string(a) + "][i]";
        std::string v;
        if (G.kinds[a] == FQ_AGG_COUNT) {
            src += "        atomicAdd((unsigned long long *)&tr.st[" + std::to_string(a) + "][gs], (unsigned long long)" + sa +
                   ");\n";
            continue;
        }
        if (G.dtypes[a] == FQ_DT_FLOAT64) v = "__builtin_bit_cast(double, " + sa + ")";
        else v = "(" + std::string(ctype(G.dtypes[a])) + ")" + sa;
        src += "        " + state_update(G.kinds[a], G.dtypes[a], "&tr.st[" + std::to_string(a) + "][gs]", v) + "\n";
    }
    src += "    }\n}\n";

    // kernel
    src += R"(
extern "C" __global__ void __launch_bounds__(BT)
fq_jit_groupby(const TIn *__restrict__ col, long long n, long long head, const u64 *__restrict__ bitmap,
               Consts c, Tab t) {
    __shared__ u64 s_keys[S];
    __shared__ u64 s_st[NA][S];
    __shared__ int s_bypass[2];  // [0] bypass flag, [1] slots claimed
    fq_lds_reset(s_keys, s_st, s_bypass);
    __syncthreads();
    // this workgroup's replica of the HBM states
    Tab tr = t;
    const long long roff = (long long)(blockIdx.x & t.rmask) * (t.mask + 2);
    for (int a = 0; a < NA; ++a) tr.st[a] += roff;
    // Key partitions: when the HBM table already holds more groups (from
    // earlier launches into it) than half an LDS table, workgroup b only
    // aggregates the keys of partition b % P and walks the rows with the
    // other (grid / P) - 1 workgroups of its partition: every row is read P
    // times, but every group stays in LDS.
    const u32 seen = __hip_atomic_load(&t.hdr[4], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // (only past the LDS saturation point, 3/4 of S; beyond PMAX partitions
    // the rows are cheaper to send to the HBM table than to re-read)
    // and only once a launch saw an LDS table saturate (hdr[5]): keys that
    // differ from block to block (clustered, number / 1000000) fill the HBM
    // table without crowding any one launch's LDS
    const u32 saturated = __hip_atomic_load(&t.hdr[5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    u32 P = 1;
    if (!DENSE && saturated && seen > (u32)(S * 3 / 4))  // (dense keys never outgrow the table)
        while (P <= PMAX && P * (u32)(S / 2) < seen) P <<= 1;
    if (P > PMAX || gridDim.x % P) P = 1;
    const u32 part = blockIdx.x & (P - 1);
    const long long RG = gridDim.x / P, rb = blockIdx.x / P;
    u32 flags = 0;
    const long long T = RG * BT;
    const long long g = rb * BT + threadIdx.x;
    const long long nvec = (n - head) / 2;
    const u32x4 *__restrict__ vp = (const u32x4 *)(col + head);
#if ROWMAP == 1
    // lane-consecutive rows (8-byte loads): the 64 keys of one LDS access are
    // 64 consecutive rows, so small sequential keys hit distinct banks
    const TIn *__restrict__ cp = col + head;
    const long long TV = 4 * BT;  // vectors (pairs) per tile, as below
    const long long ntiles = nvec / TV;
#if GCHUNK
    // one contiguous run of tiles per workgroup: clustered keys then meet a
    // workgroup's LDS table a few at a time, so its flush stays small
    const long long per = (ntiles + RG - 1) / RG, t_lo = rb * per, t_hi = t_lo + per < ntiles ? t_lo + per : ntiles;
    const long long t_step = 1;
#else
    const long long t_lo = rb, t_hi = ntiles, t_step = RG;
#endif
    // Row layout per tile: mode 0 = lane-consecutive rows (row k * BT + tid:
    // a wave's 64 keys of one LDS access are 64 consecutive rows); mode 1 =
    // eight consecutive rows per lane (row 8 * tid + j), so runs of equal keys
    // merge in the lane's registers (fq_runs) and then across the wave
    // (fq_wave_runs) instead of 64 lanes serialising on one LDS slot.  Mode 1
    // loads each wave's 512 rows coalesced (slot k = rows 64k + lane of the
    // wave's chunk) and transposes them through 1 KB of LDS per wave in four
    // rounds of 128 rows (per-lane 64-B loads ran at 2.6 ms per 10 GB).  The
    // workgroup picks the mode once, from its first tile: mode 1 when most
    // waves see at most GCLUSTER_CHANGES key changes over their 512 rows and
    // their lanes' rows BT apart differ (scattered keys stay in mode 0, where
    // mode 1 would put a lane's eight neighbouring keys on eight slots per
    // lane; runs longer than BT rows already merge in mode 0).  Each mode has
    // its own loop, so mode 0 is the plain kernel.
    TIn nxt[8];
    const long long tile_rows = TV * 2;
    auto gload = [&](long long tile, auto M) {
        if constexpr (decltype(M)::value == 1) {
            const TIn *__restrict__ q = cp + tile * tile_rows + (long long)(threadIdx.x >> 6) * 512 + (threadIdx.x & 63);
#pragma unroll
            for (int k = 0; k < 8; ++k) nxt[k] = __builtin_nontemporal_load(q + 64 * k);
        } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) nxt[k] = __builtin_nontemporal_load(cp + tile * tile_rows + threadIdx.x + (long long)k * BT);
        }
    };
#if GCLUSTER
    __shared__ u64 s_tr[BT / 64][128];
#endif
    // mode 1: nxt (the wave's rows 64k + lane) -> raw (rows 8 * lane + i)
    // through 1 KB of LDS per wave; nxt is free again for the next tile's
    // loads, so raw, nxt and the transpose never hold three tiles of registers
    auto transpose = [&](TIn (&raw)[8]) {
#if GCLUSTER
        const int w = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            s_tr[w][lane] = __builtin_bit_cast(u64, nxt[2 * p]);
            s_tr[w][64 + lane] = __builtin_bit_cast(u64, nxt[2 * p + 1]);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if ((lane >> 4) == p) {
#pragma unroll
                for (int i = 0; i < 8; ++i) raw[i] = __builtin_bit_cast(TIn, s_tr[w][8 * (lane & 15) + i]);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
#else
        (void)raw;
#endif
    };
    // one tile's rows through the LDS table
    auto work = [&](auto M, long long tt, TIn (&raw)[8]) {
        constexpr int mode = decltype(M)::value;
        Row r[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const long long row = mode ? (long long)threadIdx.x * 8 + k : threadIdx.x + (long long)k * BT;
            fq_prep(raw[k], head + tt * tile_rows + row, c, bitmap, flags, r[k]);
            if (P > 1 && part_of(r[k].k, P) != part) r[k].pass = 0;
        }
        u32 cnt[8];
        fq_runs(r, cnt);
#if GWAVE
        if constexpr (mode == 1) fq_wave_runs(r, cnt);
#endif
        u64 cur[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) cur[j] = fq_first(r[j], s_keys);
#pragma unroll
        for (int j = 0; j < 8; ++j) fq_commit_lane(r[j], cur[j], tr, s_keys, s_st, s_bypass, (u64)cnt[j]);
    };
    auto loop = [&](auto M, long long from) {
        for (long long tt = from; tt < t_hi; tt += t_step) {
            TIn raw[8];
            if constexpr (decltype(M)::value == 1) {
                transpose(raw);
            } else {
#pragma unroll
                for (int k = 0; k < 8; ++k) raw[k] = nxt[k];
            }
            const long long tn = tt + t_step;
            if (tn < t_hi) gload(tn, M);
            work(M, tt, raw);
        }
    };
    if (t_lo < t_hi) {
        // the first tile in mode 0 decides the layout of the rest
        gload(t_lo, IC<0>());
        TIn raw[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) raw[k] = nxt[k];
        int nmode = 0;
#if GCLUSTER
        {
            __shared__ int s_vote;
            const int lane = (int)(threadIdx.x & 63);
            u32 vf = 0, changes = 0;
            u64 k0 = 0, k1 = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const u64 kk = fq_key(raw[k], c, vf, 1u);
                const u64 prev = ((u64)(u32)__shfl_up((int)(u32)(kk >> 32), 1, 64) << 32) | (u32)__shfl_up((int)(u32)kk, 1, 64);
                changes += (u32)__popcll(__ballot(lane > 0 && kk != prev));
                if (k == 0) k0 = kk;
                if (k == 1) k1 = kk;
            }
            // runs longer than BT rows already merge in mode 0 (a lane's rows
            // are BT apart): keep it
            const u32 far = (u32)__popcll(__ballot(k0 == k1));
            if (threadIdx.x == 0) s_vote = 0;
            __syncthreads();
            if (lane == 0 && changes <= GCLUSTER_CHANGES && far < 32) atomicAdd(&s_vote, 1);
            __syncthreads();
            nmode = s_vote * 2 > BT / 64 ? 1 : 0;
        }
#endif
        if (t_lo + t_step < t_hi) {
            if (nmode) gload(t_lo + t_step, IC<1>());
            else gload(t_lo + t_step, IC<0>());
        }
        work(IC<0>(), t_lo, raw);
#if GCLUSTER
        if (nmode) loop(IC<1>(), t_lo + t_step);
        else
#endif
        loop(IC<0>(), t_lo + t_step);
    }
#else
    const long long TV = 4 * BT;
    const long long ntiles = nvec / TV;
    // software pipelined: the next tile's loads are in flight while this
    // tile's rows go through the LDS table (2 waves per SIMD cannot hide the
    // HBM latency otherwise)
    u32x4 nxt[4];
    if (rb < ntiles) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            nxt[k] = __builtin_nontemporal_load(vp + rb * TV + threadIdx.x + (long long)k * BT);
    }
    for (long long tt = rb; tt < ntiles; tt += RG) {
        const long long base = tt * TV + threadIdx.x;
        u32x4 raw[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) raw[k] = nxt[k];
        const long long tn = tt + RG;
        if (tn < ntiles) {
#pragma unroll
            for (int k = 0; k < 4; ++k) nxt[k] = __builtin_nontemporal_load(vp + tn * TV + threadIdx.x + (long long)k * BT);
        }
        Row r[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            TIn x[2];
            __builtin_memcpy(&x[0], &raw[k], 16);
            const long long i0 = head + (base + (long long)k * BT) * 2;
            fq_prep(x[0], i0, c, bitmap, flags, r[2 * k]);
            fq_prep(x[1], i0 + 1, c, bitmap, flags, r[2 * k + 1]);
            if (P > 1 && part_of(r[2 * k].k, P) != part) r[2 * k].pass = 0;
            if (P > 1 && part_of(r[2 * k + 1].k, P) != part) r[2 * k + 1].pass = 0;
        }
        u32 cnt[8];
        const bool lane_runs = fq_runs(r, cnt);
#if GWAVE
        if (!lane_runs) fq_wave_runs(r, cnt);
#else
        (void)lane_runs;
#endif
        u64 cur[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) cur[j] = fq_first(r[j], s_keys);
#pragma unroll
        for (int j = 0; j < 8; ++j) fq_commit_lane(r[j], cur[j], tr, s_keys, s_st, s_bypass, (u64)cnt[j]);
    }
#endif
    for (long long v = ntiles * TV + g; v < nvec; v += T) {
        const u32x4 raw = __builtin_nontemporal_load(vp + v);
        TIn x[2];
        __builtin_memcpy(&x[0], &raw, 16);
        fq_row(x[0], head + v * 2, c, tr, bitmap, s_keys, s_st, flags, s_bypass, P, part);
        fq_row(x[1], head + v * 2 + 1, c, tr, bitmap, s_keys, s_st, flags, s_bypass, P, part);
    }
    const long long tail0 = head + nvec * 2;
    const long long nedge = head + (n - tail0);
    for (long long e = g; e < nedge; e += T) {
        const long long i = e < head ? e : tail0 + (e - head);
        fq_row(col[i], i, c, tr, bitmap, s_keys, s_st, flags, s_bypass, P, part);
    }
    if (flags) atomicOr(&t.hdr[0], flags);
    __syncthreads();
    if (threadIdx.x == 0 && s_bypass[0]) atomicOr(&t.hdr[5], 1u);
    fq_flush(tr, s_keys, s_st);
}
)";
    src += kGroupPartitionKernels;
    return true;
}

// ---------------------------------------------------------------------------
// FilterTransform -> ProjectionTransform over one column (fq_filter_project,
// fq_predicate_bitmap).  One module per shape holds three kernels:
//   fq_jit_pbits    predicate -> bitmap: each wave evaluates 8 consecutive
//                   64-row words per step (lane l = row l of each word, 8-byte
//                   loads, 8 in flight per lane), one ballot per word, lanes
//                   0..7 store the 8 words;
//   fq_jit_pselect  one pass: predicate, decoupled look-back over tiles for
//                   the output offsets, the projection evaluated on the kept
//                   rows only, one store per output;
//   fq_jit_pmap     no predicate: every row's outputs, 16-byte loads/stores.
// ---------------------------------------------------------------------------
struct HostProjConsts {
    uint64_t rhs;
    HostStep p[kSteps], v[FQ_MAX_PROJECT][kSteps];
    uint64_t rl[FQ_MAX_PRED_LEAVES];
    HostStep pl[FQ_MAX_PRED_LEAVES][kSteps];
};

void pack_proj_consts(const ProjLaunch &P, HostProjConsts &hc) {
    hc.rhs = P.pred.rhs;
    for (int i = 0; i < kSteps; ++i) {
        hc.p[i] = HostStep{P.pred.lhs.s[i].c, P.pred.lhs.s[i].magic, P.pred.lhs.s[i].shift};
        for (int j = 0; j < FQ_MAX_PROJECT; ++j) hc.v[j][i] = HostStep{P.vals[j].s[i].c, P.vals[j].s[i].magic, P.vals[j].s[i].shift};
    }
    pack_tree_consts(P.pred, hc);
}

std::string proj_shape_key(const ProjLaunch &P, int32_t tin, int dev) {
    // the tunable part of the shape: the block kernel's rows per thread and stage
    std::string k = "PROJb" + std::to_string(fqc::knob(FQ_TUNE_SELECT_BLOCKS_ROWS)) + "S" +
                    std::to_string(fqc::knob(FQ_TUNE_SELECT_BLOCKS_STAGE));
    auto put = [&k](int32_t v) { k.append(reinterpret_cast<const char *>(&v), sizeof v); };
    put(dev);
    put(tin);
    put_pred_key(P.pred, k);
    put(P.n_out);
    for (int j = 0; j < P.n_out; ++j) {
        put(P.dtypes[j]);
        put(P.chain[j] ? 1 : 0);
        if (!P.chain[j]) continue;
        put(P.vals[j].n);
        for (int i = 0; i < P.vals[j].n; ++i) {
            const KStep &st = P.vals[j].s[i];
            put(st.code);
            put(st.operand);
            put(st.reversed);
            put(st.dtype);
            put((int32_t)st.add);
            put(st.sdtype);
        }
    }
    return k;
}

// fq_jit_pblocks (fq_filter_project_blocks): Filter ->
// Projection over a stream of DataBlocks of B rows, the way the reference runs
// both transforms (ExpressionStream applies FilterTransform::expression_executor
// to each numbers block, transform_filter.rs:38-55, numbers_stream.rs:29, then
// transform_projection.rs:45-56): block b's kept rows go, in order, to output
// rows [b * B, b * B + count[b]) -- an output block starts where its input
// block does, so no block's offsets depend on another block's count and no
// workgroup waits on another (no look-back: fq_jit_pselect's contiguous output
// needs one).  Workgroups draw whole blocks from a counter, so the blocks in
// flight are adjacent (one static range per workgroup, or blocks dealt
// round-robin, measured 7-10 % slower: profiles/r03_s3_blocks_sweeps.txt),
// and walk a block in tiles of PB_THREADS x PB_ROWS rows that ignore block
// edges; B >= the tile, so a tile holds at most one block edge: rows before it
// go to the open block at its running count (carry), rows after it start the
// next block.  Kept rows before the edge are exactly those of in-tile rank <
// re, the edge's rank, read from the tile's ballots and exclusive group
// offsets in LDS (double-buffered by tile parity: two barriers per tile).
// Outputs are written with nontemporal stores (3.42 -> 3.12 ms per 10 GB, no
// change for the look-back kernel).  PB_STAGE (round 5): the tile's
// kept rows go to LDS by in-tile rank first, then consecutive threads write
// them out as 16-byte row pairs (pb_copy), so every store instruction covers
// one contiguous span instead of the ~24 kept lanes of a 64-row ballot.  The
// stage holds 1/PB_STAGE of a tile (a tile keeping more takes several passes).
// In one process, 4 rounds x 8 queries of p1 each, ms per 3.125e8-row block
// (profiles/r05_e_p1_stage_ab.json, r05_g_p1_stage_ab.json): 32 rows per
// thread with a half-tile stage (32 KB, 4 workgroups per CU, p1's 3/8 kept in
// one pass) 0.725; a whole-tile stage at 16 rows 0.730-0.734, at 32 rows (2
// workgroups per CU) 0.945; a quarter-tile stage at 32 rows (two passes)
// 0.733; the round-4 kernel (32 rows, stores from registers) 0.760-0.769.
// Row pairs (round 6): each lane loads two adjacent rows with one 16-byte
// non-temporal load and a 128-row group takes two ballots (first and second
// rows); in-tile ranks count both.  Round 4 measured pairs slower (4.52 vs
// 3.10 ms) while lanes stored their own kept rows -- a wave's stores then
// interleave; behind the LDS stage the stores no longer depend on the lane
// mapping and pairs win: 0.7045 -> 0.6768 ms per 3.125e8-row block, 22.66 ->
// 21.75 ms per p1 query, one process, 4 rounds (profiles/r06_i_p1_pairs_ab.json).
// A tile that is ragged or not 16-byte aligned loads its pairs 8 bytes at a time.
std::string gen_project_blocks_kernel(bool bitmap_pred) {
    std::string s = "#define PB_ROWS " + std::to_string(fqc::knob(FQ_TUNE_SELECT_BLOCKS_ROWS)) + "\n#define PB_STAGE " +
                    std::to_string(fqc::knob(FQ_TUNE_SELECT_BLOCKS_STAGE)) + "\n";
    s += R"(
#define PB_THREADS 256
#define PB_WAVES (PB_THREADS / 64)
#define PB_TILE (PB_THREADS * PB_ROWS)
#define PB_NP (PB_ROWS / 2)        // 16-byte row pairs per thread per tile
#define PB_NE (PB_NP * PB_WAVES)   // 128-row groups per tile
#define PB_PUT fq_put_nt
// group i = k * PB_WAVES + wave holds tile rows [128 i, 128 i + 128): lane l's
// pair is rows 128 i + 2 l (its b0 bit) and 128 i + 2 l + 1 (its b1 bit)
struct PbShared {
    u64 b0[2][PB_NE], b1[2][PB_NE];
    u32 off[2][PB_NE + 1];  // exclusive in-tile offset of each group; [PB_NE]: the tile's kept rows
};
// exclusive scan of the ng group counts in off[] by wave 0; off[PB_NE] = total
__device__ __forceinline__ void pb_scan(u32 *__restrict__ off, int ng, int lane) {
    constexpr int PER = (PB_NE + 63) / 64;
    u32 cv[PER], tot = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        cv[q] = lane * PER + q < ng ? off[lane * PER + q] : 0u;
        tot += cv[q];
    }
    u32 incl = tot;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const u32 v = (u32)__shfl_up((int)incl, d, 64);
        if (lane >= d) incl += v;
    }
    u32 run = incl - tot;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        if (lane * PER + q < ng) off[lane * PER + q] = run;
        run += cv[q];
    }
    if (lane == 63) off[ng] = incl;
}
#if PB_STAGE
// PB_STAGE: the tile's kept rows staged in LDS by in-tile rank, then written
// out by consecutive threads: ranks [lo, hi) go to output rows d + rank, rank
// r in st[r - base].  al: every output is 16-byte aligned -- row pairs as one
// 16-byte store each, the odd row at either end alone; else one row per thread.
// The stage holds PB_CAP = PB_TILE / PB_STAGE rows: a tile keeping more takes
// several passes.
#define PB_CAP (PB_TILE / PB_STAGE)
__device__ __forceinline__ void pb_copy(const TIn *__restrict__ st, u32 base, u32 lo, u32 hi, long long d, int al,
                                        int tid, const Consts &c, u32 &vflags, const Outs &o) {
    if (lo >= hi) return;
    if (!al) {
        for (u32 r = lo + tid; r < hi; r += PB_THREADS) PB_PUT(st[r - base], c, vflags, 1u, o, d + (long long)r);
        return;
    }
    const long long p0 = d + lo, p1 = d + hi, sb = d + base;
    if ((p0 & 1) && tid == 0) PB_PUT(st[lo - base], c, vflags, 1u, o, p0);
    if ((p1 & 1) && tid == 64) PB_PUT(st[hi - 1 - base], c, vflags, 1u, o, p1 - 1);
    for (long long q = ((p0 + 1) >> 1) + tid; q < (p1 >> 1); q += PB_THREADS)
        fq_put2(st[2 * q - sb], st[2 * q + 1 - sb], c, vflags, o, q);
}
#endif
)";
    s += R"(extern "C" __global__ void __launch_bounds__(PB_THREADS)
fq_jit_pblocks(const TIn *__restrict__ col, long long n, long long B, Consts c,
    const u64 *__restrict__ bm, Outs o, long long *__restrict__ counts, u32 *__restrict__ fl,
    unsigned long long *__restrict__ total, u32 *__restrict__ ticket, int al) {
    __shared__ PbShared sh;
#if PB_STAGE
    __shared__ TIn stage[PB_CAP];
#else
    (void)al;
#endif
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const long long nb = (n + B - 1) / B;
    u64 kept = 0;  // the workgroup's kept rows
    u32 pflags = 0, vflags = 0;
    const u64 lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    int par = 0;
    // one block per draw from the counter: the blocks in flight stay adjacent
    __shared__ long long s_run;
    for (;;) {
        if (tid == 0) s_run = (long long)atomicAdd(ticket, 1u);
        __syncthreads();
        const long long run = s_run;
        if (run >= nb) break;
        const long long b_lo = run, b_hi = run + 1;
    const long long end = b_hi * B < n ? b_hi * B : n;
    long long cur = b_lo;  // the open block
    u64 carry = 0;         // its kept rows so far
    for (long long r0 = b_lo * B; r0 < end; r0 += PB_TILE, par ^= 1) {
)";
    const std::string predp =
        bitmap_pred ? "            const bool p0 = live0 && ((bm[row >> 6] >> (row & 63)) & 1ull);\n"
                      "            const bool p1 = live1 && ((bm[(row + 1) >> 6] >> ((row + 1) & 63)) & 1ull);\n"
                      "            (void)c;\n"
                    : "            const bool p0 = fq_pred(x0[k], c, pflags, live0) && live0;\n"
                      "            const bool p1 = fq_pred(x1[k], c, pflags, live1) && live1;\n";
    s += R"(
        u64 *__restrict__ b0s = sh.b0[par];
        u64 *__restrict__ b1s = sh.b1[par];
        u32 *__restrict__ off = sh.off[par];
        // 16-byte row-pair loads when the tile is whole and 16-byte aligned
        TIn x0[PB_NP], x1[PB_NP];
        if (r0 + PB_TILE <= end && ((((unsigned long long)(col + r0)) & 15ull) == 0ull)) {
            const u32x4 *__restrict__ vp = (const u32x4 *)(col + r0);
#pragma unroll
            for (int k = 0; k < PB_NP; ++k) {
                const u32x4 raw = __builtin_nontemporal_load(vp + tid + k * PB_THREADS);
                __builtin_memcpy(&x0[k], &raw, 8);
                __builtin_memcpy(&x1[k], ((const char *)&raw) + 8, 8);
            }
        } else {
#pragma unroll
            for (int k = 0; k < PB_NP; ++k) {
                const long long row = r0 + 2 * (long long)(tid + k * PB_THREADS);
                x0[k] = row < end ? __builtin_nontemporal_load(col + row) : TIn(0);
                x1[k] = row + 1 < end ? __builtin_nontemporal_load(col + row + 1) : TIn(0);
            }
        }
#pragma unroll
        for (int k = 0; k < PB_NP; ++k) {
            const long long row = r0 + 2 * (long long)(tid + k * PB_THREADS);
            const u32 live0 = row < end ? 1u : 0u, live1 = row + 1 < end ? 1u : 0u;
)" + predp + R"(
            const u64 c0 = __ballot(p0), c1 = __ballot(p1);
            if (lane == 0) {
                b0s[k * PB_WAVES + wave] = c0;
                b1s[k * PB_WAVES + wave] = c1;
                off[k * PB_WAVES + wave] = (u32)(__popcll(c0) + __popcll(c1));
            }
        }
        __syncthreads();
        if (wave == 0) pb_scan(off, PB_NE, lane);
        __syncthreads();
        const u32 tot = off[PB_NE];
        const long long bnd = (cur + 1) * B < n ? (cur + 1) * B : n;
        const long long e = bnd - r0;
        u32 re = tot;  // kept rows of the tile before the open block's edge
        if (e < PB_TILE) {
            const int g = (int)(e >> 7), pos = (int)(e & 127), h = pos >> 1;
            const u64 m = (1ull << h) - 1ull;
            re = off[g] + (u32)__popcll(b0s[g] & m) + (u32)__popcll(b1s[g] & m) +
                 ((pos & 1) ? (u32)((b0s[g] >> h) & 1ull) : 0u);
        }
        const long long before = cur * B + (long long)carry;
        const long long after = (cur + 1) * B - (long long)re;
#if PB_STAGE
        for (u32 base = 0; base < tot; base += PB_CAP) {
            if (base) __syncthreads();
#pragma unroll
            for (int k = 0; k < PB_NP; ++k) {
                const u64 c0 = b0s[k * PB_WAVES + wave], c1 = b1s[k * PB_WAVES + wave];
                const u32 k0 = (u32)((c0 >> lane) & 1ull), k1 = (u32)((c1 >> lane) & 1ull);
                // rank - base, wrapping for ranks below base (then >= PB_CAP)
                const u32 r = off[k * PB_WAVES + wave] + (u32)__popcll(c0 & lt) + (u32)__popcll(c1 & lt) - base;
                if (k0 && r < PB_CAP) stage[r] = x0[k];
                if (k1 && r + k0 < PB_CAP) stage[r + k0] = x1[k];
            }
            __syncthreads();
            const u32 hi = tot - base < PB_CAP ? tot : base + PB_CAP;
            pb_copy(stage, base, base, re < hi ? re : hi, before, al, tid, c, vflags, o);
            pb_copy(stage, base, re > base ? re : base, hi, after, al, tid, c, vflags, o);
        }
#else
#pragma unroll
        for (int k = 0; k < PB_NP; ++k) {
            const u64 c0 = b0s[k * PB_WAVES + wave], c1 = b1s[k * PB_WAVES + wave];
            const u32 k0 = (u32)((c0 >> lane) & 1ull), k1 = (u32)((c1 >> lane) & 1ull);
            const u32 rank = off[k * PB_WAVES + wave] + (u32)__popcll(c0 & lt) + (u32)__popcll(c1 & lt);
            if (k0) PB_PUT(x0[k], c, vflags, 1u, o, (rank < re ? before : after) + (long long)rank);
            if (k1) PB_PUT(x1[k], c, vflags, 1u, o, (rank + k0 < re ? before : after) + (long long)(rank + k0));
        }
#endif
)";
    s += R"PB(
        kept += tot;
        if (e <= PB_TILE) {
            if (tid == 0) counts[cur] = (long long)(carry + re);
            carry = tot - re;
            ++cur;
        } else {
            carry += tot;
        }
    }
    }
    pflags = wave_or(pflags);
    vflags = wave_or(vflags);
    if (lane == 0 && pflags) atomicOr(fl, pflags);
    if (lane == 0 && vflags) atomicOr(fl + 1, vflags);
    if (tid == 0 && kept) atomicAdd(total, (unsigned long long)kept);
}
)PB";
    return s;
}

bool gen_project_source(const ProjLaunch &P, int32_t tin, int dev, Gen &g, std::string &src) {
    const char *TIn = ctype(tin);
    if (!TIn || P.n_out < 1 || P.n_out > FQ_MAX_PROJECT) return false;
    const int32_t pk = P.pred.kind;
    std::string pred_body;
    const bool expr_pred = pk == FQ_PRED_EXPR || pk == FQ_PRED_TREE;
    if (expr_pred && !emit_pred_body(g, P.pred, tin, pred_body)) return false;
    src = kCommon;
    src += "typedef " + std::string(TIn) + " TIn;\n";
    src += "struct Step { u64 c, m, s; };\nstruct Consts { u64 rhs; Step p[" + std::to_string(kSteps) + "], v[" +
           std::to_string(FQ_MAX_PROJECT) + "][" + std::to_string(kSteps) + "]; u64 rl[" +
           std::to_string(FQ_MAX_PRED_LEAVES) + "]; Step pl[" + std::to_string(FQ_MAX_PRED_LEAVES) + "][" +
           std::to_string(kSteps) + "]; };\n";
    src += "struct Outs { void *p[" + std::to_string(FQ_MAX_PROJECT) + "]; };\n";
    src += "#define PS_ROWS " + std::to_string(select_rows_per_thread()) + "\n#define PS_THREADS " +
           std::to_string(select_threads()) + "\n#define PS_SLEEP " + std::to_string(select_sleep()) +
           "\n";
    src += "typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));\n";
    src += "__device__ __forceinline__ bool fq_pred(TIn x, const Consts &c, u32 &flags, u32 live) {\n";
    src += expr_pred ? pred_body : "    (void)x; (void)c; (void)flags; (void)live;\n    return true;\n";
    src += "}\n";
    // every output: its value function and its 64-bit store
    std::string put_all = "__device__ __forceinline__ void fq_put(TIn x, const Consts &c, u32 &flags, u32 live, const Outs &o,\n"
                          "                                       long long pos) {\n";
    std::string put_nt = "__device__ __forceinline__ void fq_put_nt(TIn x, const Consts &c, u32 &flags, u32 live, const Outs &o,\n"
                         "                                          long long pos) {\n";
    std::string vals_pair = "__device__ __forceinline__ void fq_put2(TIn x0, TIn x1, const Consts &c, u32 &flags, const Outs &o,\n"
                            "                                        long long pair) {\n";
    for (int j = 0; j < P.n_out; ++j) {
        const char *V = ctype(P.dtypes[j]);
        if (!V) return false;
        std::string body;
        const std::string prefix = "v[" + std::to_string(j) + "]";
        emit_value_body(g, P.chain[j] ? &P.vals[j] : nullptr, tin, P.dtypes[j], prefix.c_str(), V, body);
        const std::string J = std::to_string(j);
        src += std::string("__device__ __forceinline__ ") + V + " fq_val" + J + "(TIn x, const Consts &c, u32 &flags, u32 live) {\n" +
               "    (void)live;\n" + body + "}\n";
        put_all += std::string("    ((") + V + " *)o.p[" + J + "])[pos] = fq_val" + J + "(x, c, flags, live);\n";
        put_nt += std::string("    __builtin_nontemporal_store(fq_val") + J + "(x, c, flags, live), ((" + V + " *)o.p[" + J + "]) + pos);\n";
        vals_pair += std::string("    { const ") + V + " a = fq_val" + J + "(x0, c, flags, 1u), b = fq_val" + J +
                     "(x1, c, flags, 1u);\n      __builtin_nontemporal_store(u64x2{__builtin_bit_cast(u64, a), "
                     "__builtin_bit_cast(u64, b)}, ((u64x2 *)o.p[" + J + "]) + pair); }\n";
    }
    src += put_all + "}\n" + put_nt + "}\n" + vals_pair + "}\n";
    src += R"(
__device__ __forceinline__ u32 wave_or(u32 f) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) f |= (u32)__shfl_xor((int)f, off, 64);
    return f;
}

extern "C" __global__ void __launch_bounds__(256)
fq_jit_pbits(const TIn *__restrict__ col, long long n, Consts c, u64 *__restrict__ bm, u32 *__restrict__ fl) {
    const int lane = threadIdx.x & 63;
    const long long wave = ((long long)blockIdx.x * 256 + threadIdx.x) >> 6;
    const long long W = ((long long)gridDim.x * 256) >> 6;
    const long long nwords = (n + 63) >> 6;
    u32 flags = 0;
    for (long long w0 = wave * 8; w0 < nwords; w0 += W * 8) {
        TIn x[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const long long r = (w0 + k) * 64 + lane;
            x[k] = r < n ? __builtin_nontemporal_load(col + r) : TIn(0);
        }
        u64 mine = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const long long r = (w0 + k) * 64 + lane;
            const u32 live = r < n ? 1u : 0u;
            const bool pass = fq_pred(x[k], c, flags, live) && live;
            const u64 word = __ballot(pass);
            if (lane == k) mine = word;
        }
        if (lane < 8 && w0 + lane < nwords) bm[w0 + lane] = mine;
    }
    flags = wave_or(flags);
    if (lane == 0 && flags) atomicOr(fl, flags);
}

// Single pass over the column (decoupled look-back).  A workgroup draws a
// tile of PS_TILE rows (lane-consecutive 8-byte rows, PS_ROWS per lane in
// flight), evaluates the predicate (one ballot per 64 rows, kept in LDS),
// publishes the tile's kept count as flag A; wave 0 walks back over the
// predecessors' status words, 64 * PS_LBW per round trip, until it meets an
// inclusive prefix (flag P), publishes its own P; then every wave writes its
// kept rows' outputs at base + rank.  A workgroup only draws a tile when it
// can start it at once: a reserved tile whose A waits behind another tile's
// look-back chains look-backs across workgroups (a prefetching variant that
// drew the next tile before its look-back measured 3-4x slower; one that
// held two tiles and published the second's A while the first waited
// measured no faster -- tools/select_sweep.sh, profiles/r02_select_*).
//
// Tickets: ONE device-scope counter, so tiles are drawn in order and the
// lowest unfinished tile always has every predecessor drawn by a resident
// workgroup -- the look-back progresses whatever else runs on the GPU.  (Round
// 2's per-XCD ticket classes were faster alone on the GPU, but their progress
// argument needed a resident workgroup in every class: beside the engine's
// other LIMIT pipes on private queues a launch could hold fewer, and two such
// launches once waited on each other's CUs until the poll bound -- round 5,
// tests/test_memory_gpu.py.  Removed in round 6; tests/test_project_gpu.py
// runs two look-back launches side by side.)
// Status words are 64-bit agent-scope atomics: flag in the top 2 bits, count
// below.  The look-back is bounded: after ~2^20 polls the kernel flags an
// error (fl[1] bit 31) and moves on, so a wave can never spin forever.
// LDS state is double-buffered by tile parity: two barriers per tile.
#ifndef PS_ROWS
#define PS_ROWS 16
#endif
#ifndef PS_THREADS
#define PS_THREADS 256
#endif
#ifndef PS_SLEEP
#define PS_SLEEP 2
#endif
#ifndef PS_LBW
#define PS_LBW 1
#endif
#define PS_WAVES (PS_THREADS / 64)
#define PS_TILE (PS_THREADS * PS_ROWS)
#define PS_A (1ull << 62)
#define PS_P (2ull << 62)
#define PS_VAL(s) ((s) & ((1ull << 62) - 1ull))
__device__ __forceinline__ u64 wave_sum64(u64 v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const u32 lo = __shfl_xor((u32)(v & 0xffffffffu), off, 64);
        const u32 hi = __shfl_xor((u32)(v >> 32), off, 64);
        v += ((u64)hi << 32) | lo;
    }
    return v;
}
struct PsShared {
    u64 bal[2][PS_ROWS][PS_WAVES];   // ballots of the tile in each slot
    u32 off[2][PS_ROWS * PS_WAVES];  // exclusive in-tile offsets, (row group, wave) k-major
    u64 base[2], agg[2];
    long long tk;  // ticket drawn (broadcast)
};
struct PsCtx {
    const TIn *__restrict__ col;
    long long n, ntiles;
    const u64 *__restrict__ bm;
    u64 *__restrict__ status;
    u32 *__restrict__ ticket;
};
// the next tile for this workgroup (thread 0 only); >= ntiles when none is left
__device__ __forceinline__ long long ps_ticket(const PsCtx &X) { return atomicAdd(X.ticket, 1u); }
__device__ __forceinline__ void ps_load(const PsCtx &X, long long t, TIn (&x)[PS_ROWS]) {
    const long long r0 = t * PS_TILE + threadIdx.x;
    if (t * PS_TILE + PS_TILE <= X.n) {
#pragma unroll
        for (int k = 0; k < PS_ROWS; ++k) x[k] = __builtin_nontemporal_load(X.col + r0 + k * PS_THREADS);
    } else {
#pragma unroll
        for (int k = 0; k < PS_ROWS; ++k) {
            const long long row = r0 + k * PS_THREADS;
            x[k] = row < X.n ? __builtin_nontemporal_load(X.col + row) : TIn(0);
        }
    }
}
// tile t's predicate into slot S: ballots, in-tile offsets, aggregate; wave 0
// publishes A (tile 0: P, base 0).  Contains one barrier.
template <int S>
__device__ __forceinline__ void ps_pred(const PsCtx &X, const Consts &c, PsShared &sh, long long t, const TIn (&x)[PS_ROWS],
                                        u32 &pflags) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const long long r0 = t * PS_TILE;
#pragma unroll
    for (int k = 0; k < PS_ROWS; ++k) {
        const long long row = r0 + k * PS_THREADS + tid;
        const u32 live = row < X.n ? 1u : 0u;
)" + std::string(P.pred.kind == FQ_PRED_BITMAP
                     ? "        const bool p = live && ((X.bm[row >> 6] >> (row & 63)) & 1ull);\n        (void)c;\n        (void)x;\n        (void)pflags;\n"
                     : "        const bool p = fq_pred(x[k], c, pflags, live) && live;\n") + R"(
        const u64 b = __ballot(p);
        if (lane == 0) {
            sh.bal[S][k][wave] = b;
            sh.off[S][k * PS_WAVES + wave] = (u32)__popcll(b);
        }
    }
    __syncthreads();
    if (wave == 0) {
        // exclusive scan of the PS_ROWS * PS_WAVES counts: lane l owns
        // entries [l * PER, l * PER + PER)
        constexpr int NE = PS_ROWS * PS_WAVES, PER = (NE + 63) / 64;
        u32 cv[PER], tot = 0;
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const int i = lane * PER + q;
            cv[q] = i < NE ? sh.off[S][i] : 0u;
            tot += cv[q];
        }
        u32 incl = tot;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const u32 v = (u32)__shfl_up((int)incl, off, 64);
            if (lane >= off) incl += v;
        }
        u32 run = incl - tot;
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const int i = lane * PER + q;
            if (i < NE) sh.off[S][i] = run;
            run += cv[q];
        }
        const u64 agg = (u64)__shfl((int)incl, 63, 64);
        if (lane == 0) {
            sh.agg[S] = agg;
            __hip_atomic_store(X.status + t, (t == 0 ? PS_P : PS_A) | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}
// wave 0: advance the look-back of tile t as far as the published words
// allow; true once the exclusive prefix is in excl (or the poll bound hit).
// Each lane reads PS_LBW consecutive status words per round trip (lane 0 the
// nearest), so one round trip covers 64 * PS_LBW predecessors: with ~1,000
// tiles in flight a look-back walks back over hundreds of A-only tiles
// before it meets a P.
__device__ __forceinline__ bool ps_poll(const PsCtx &X, long long &j, u64 &excl, unsigned &polls, u32 &vflags) {
    const int lane = threadIdx.x & 63;
    for (;;) {
        u64 sw[PS_LBW];
#pragma unroll
        for (int q = 0; q < PS_LBW; ++q) {
            const long long idx = j - (long long)lane * PS_LBW - q;
            sw[q] = idx >= 0 ? __hip_atomic_load(X.status + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : PS_P;
        }
        // this lane's words in order of distance: sum up to (and with) its
        // first P; not-ready words before it
        u64 lsum = 0;
        bool lp = false, lnr = false;
#pragma unroll
        for (int q = 0; q < PS_LBW; ++q) {
            if (!lp) {
                lnr |= (sw[q] >> 62) == 0ull;
                lsum += PS_VAL(sw[q]);
                lp = (sw[q] >> 62) == 2ull;
            }
        }
        const u64 isp = __ballot(lp);
        const u64 notready = __ballot(lnr);
        const int pl = isp ? __ffsll((long long)isp) - 1 : 63;  // nearest lane with a P (or the whole window)
        const u64 upto = pl == 63 ? ~0ull : ((2ull << pl) - 1ull);
        if (notready & upto) {  // a predecessor in range has not published yet
            if (++polls > (1u << 20)) {
                vflags |= 0x80000000u;
                return true;
            }
            return false;
        }
        excl += wave_sum64(((upto >> lane) & 1ull) ? lsum : 0ull);
        if (isp) return true;
        j -= 64 * PS_LBW;
    }
}
// one tile: draw, load, predicate, look back, store; false when none is left
template <int S>
__device__ __forceinline__ bool ps_single(PsCtx &X, const Consts &c, const Outs &o, u64 *__restrict__ total,
                                          PsShared &sh, TIn (&x)[PS_ROWS], u32 &pflags, u32 &vflags) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) sh.tk = ps_ticket(X);
    __syncthreads();
    const long long t = sh.tk;
    if (t >= X.ntiles) return false;
    ps_load(X, t, x);
    ps_pred<S>(X, c, sh, t, x, pflags);
    if (wave == 0) {
        u64 excl = 0;
        if (t != 0) {
            long long j = t - 1;
            unsigned polls = 0;
            while (!ps_poll(X, j, excl, polls, vflags)) {
#if PS_SLEEP > 0
                __builtin_amdgcn_s_sleep(PS_SLEEP);
#endif
            }
        }
        if (lane == 0) {
            sh.base[S] = excl;
            if (t != 0) __hip_atomic_store(X.status + t, PS_P | (excl + sh.agg[S]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();
    const u64 base = sh.base[S];
    const u64 lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
    for (int k = 0; k < PS_ROWS; ++k) {
        const u64 b = sh.bal[S][k][wave];
        if ((b >> lane) & 1ull)
            fq_put(x[k], c, vflags, 1u, o, (long long)(base + sh.off[S][k * PS_WAVES + wave] + (u32)__popcll(b & lt)));
    }
    if (t == X.ntiles - 1 && tid == 0) *total = base + sh.agg[S];
    return true;
}
extern "C" __global__ void __launch_bounds__(PS_THREADS)
fq_jit_pselect(const TIn *__restrict__ col, long long n, Consts c, const u64 *__restrict__ bm, Outs o,
               u64 *__restrict__ status, u32 *__restrict__ ticket, u32 *__restrict__ fl, u64 *__restrict__ total) {
    __shared__ PsShared sh;
    PsCtx X;
    X.col = col;
    X.n = n;
    X.ntiles = (n + PS_TILE - 1) / PS_TILE;
    X.bm = bm;
    X.status = status;
    X.ticket = ticket;
    u32 pflags = 0, vflags = 0;
    {
        TIn x[PS_ROWS];
        while (ps_single<0>(X, c, o, total, sh, x, pflags, vflags) && ps_single<1>(X, c, o, total, sh, x, pflags, vflags)) {
        }
    }
    pflags = wave_or(pflags);
    vflags = wave_or(vflags);
    if ((threadIdx.x & 63) == 0 && pflags) atomicOr(fl, pflags);
    if ((threadIdx.x & 63) == 0 && vflags) atomicOr(fl + 1, vflags);
}

// every row: 16-byte loads and stores of row pairs when the column and every
// output are 16-byte aligned (aligned != 0), else 8-byte rows
extern "C" __global__ void __launch_bounds__(256)
fq_jit_pmap(const TIn *__restrict__ col, long long n, Consts c, Outs o, int aligned, u32 *__restrict__ fl) {
    const long long g = (long long)blockIdx.x * 256 + threadIdx.x;
    const long long T = (long long)gridDim.x * 256;
    u32 flags = 0;
    long long done = 0;
    if (aligned) {
        const long long npair = n >> 1;
        const u64x2 *__restrict__ vp = (const u64x2 *)col;
        for (long long p0 = g; p0 < npair; p0 += 4 * T) {
            u64x2 raw[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const long long p = p0 + (long long)k * T;
                raw[k] = p < npair ? __builtin_nontemporal_load(vp + p) : u64x2{0, 0};
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const long long p = p0 + (long long)k * T;
                if (p < npair)
                    fq_put2(__builtin_bit_cast(TIn, (u64)raw[k].x), __builtin_bit_cast(TIn, (u64)raw[k].y), c, flags, o, p);
            }
        }
        done = npair * 2;
    }
    for (long long i = done + g; i < n; i += T) fq_put(col[i], c, flags, 1u, o, i);
    flags = wave_or(flags);
    if ((threadIdx.x & 63) == 0 && flags) atomicOr(fl, flags);
}
)";
    src += gen_project_blocks_kernel(P.pred.kind == FQ_PRED_BITMAP);
    return true;
}

// ---------------------------------------------------------------------------
// compile + cache
// ---------------------------------------------------------------------------
struct Compiled {
    hipModule_t mod = nullptr;
    hipFunction_t fn = nullptr;
    bool ok = false;  // the generator handles this shape
};

std::mutex g_mu;
std::unordered_map<std::string, Compiled> g_cache;

std::string device_arch(int dev) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return "gfx950";
    return prop.gcnArchName;
}

// dev < 0: no device here -- compile for gfx950 to validate the source only.
fq_status compile(const std::string &src, int dev, Compiled &out, const char *fn_name = "fq_jit_scan") {
    const Rtc &r = rtc();
    const auto t0 = std::chrono::steady_clock::now();
    const std::string dump = fqc::jit_dump_dir();
    const std::string dump_path = dump.empty() ? "" : dump + "/fq_jit_" + std::to_string(g_compiled.load() + 1) + ".hip";
    if (!dump.empty())  // the source before compiling: a compiler that crashes leaves it behind
        if (FILE *f = fopen(dump_path.c_str(), "w")) {
            fwrite(src.data(), 1, src.size(), f);
            fclose(f);
        }
    const std::string arch = "--offload-arch=" + (dev >= 0 ? device_arch(dev) : std::string("gfx950"));
    std::vector<char> code;
    std::string log;
    int stage = 0;  // 1: create failed, 2: compile failed (log), 3: code
    RtcThread::get().run([&] {
        hiprtcProgram prog;
        if (r.create(&prog, src.c_str(), "fq_jit_scan.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
            stage = 1;
            return;
        }
        const char *opts[] = {arch.c_str(), "-O3", "-std=c++17"};
        if (r.compile(prog, 3, opts) != HIPRTC_SUCCESS) {
            size_t n = 0;
            r.log_size(prog, &n);
            log.assign(n + 1, '\0');
            r.log(prog, &log[0]);
            r.destroy(&prog);
            stage = 2;
            return;
        }
        size_t n = 0;
        r.code_size(prog, &n);
        code.resize(n);
        r.code(prog, code.data());
        r.destroy(&prog);
        stage = 3;
    });
    if (stage == 1) return fqc::fail(FQ_E_INTERNAL, "hipRTC: cannot create program");
    if (stage == 2)
        return fqc::fail(FQ_E_INTERNAL, "hipRTC compile of the fused scan failed: " + log + "\n--- source ---\n" + src);
    if (dev >= 0) {
        FQ_HIP_TRY(hipModuleLoadData(&out.mod, code.data()));
        FQ_HIP_TRY(hipModuleGetFunction(&out.fn, out.mod, fn_name));
    }
    const auto t1 = std::chrono::steady_clock::now();
    g_compile_us += (int64_t)std::chrono::duration_cast<std::chrono::microseconds>(t1 - t0).count();
    g_compiled += 1;
    if (!dump.empty())
        if (FILE *f = fopen((dump_path + ".co").c_str(), "wb")) {  // the code object hipRTC produced
            fwrite(code.data(), 1, code.size(), f);
            fclose(f);
        }
    return FQ_OK;
}

}  // namespace

void jit_count_interp() { g_interp_launches += 1; }

namespace {

bool eligible(int32_t col_dtype, bool chain, const Launch &L) {
    if (!chain && L.pred.kind == FQ_PRED_NONE) return false;  // identity scans are already specialised
    return fqc::dtype_size(col_dtype) == 8;                      // expressions are 64-bit; narrow columns interpret
}

bool load_rtc(int32_t mode, fq_status *err) {
    const Rtc &r = rtc();
    g_available.store(r.ok ? 1 : 0);
    *err = FQ_OK;
    if (!r.ok && mode == FQ_JIT_ALWAYS)
        *err = fqc::fail(FQ_E_UNSUPPORTED, "FQ_JIT_ALWAYS: hipRTC (libhiprtc.so.7) could not be loaded");
    return r.ok;
}

// Looks up / compiles the kernel for L's shape.  *fn stays null when there is
// no device (source validated only) or the generator declines the shape
// (*ok = false).  The hit path is one binary key and one hash lookup.
fq_status get_kernel(int32_t col_dtype, bool chain, const Launch &L, hipFunction_t *fn, bool *ok) {
    *fn = nullptr;
    *ok = false;
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess) {
        (void)hipGetLastError();
        dev = -1;
    }
    const std::string key = shape_key(L, col_dtype, chain, dev);
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_cache.find(key);
    if (it == g_cache.end()) {
        Gen g;
        std::string src;
        Compiled c;
        if (gen_source(L, col_dtype, chain, g, src)) {
            fq_status s = compile(src, dev, c);
            if (s != FQ_OK) return s;
            c.ok = true;
        }
        if (dev < 0) {  // nothing loaded; do not cache
            *ok = c.ok;
            return FQ_OK;
        }
        it = g_cache.emplace(key, c).first;
    }
    *fn = it->second.fn;
    *ok = it->second.ok;
    return FQ_OK;
}

}  // namespace

fq_status jit_prepare(int32_t col_dtype, bool chain, const Launch &L, bool *ready) {
    *ready = false;
    const int32_t mode = jit_mode();
    if (mode == FQ_JIT_OFF || !eligible(col_dtype, chain, L)) return FQ_OK;
    fq_status err;
    if (!load_rtc(mode, &err)) return err;
    hipFunction_t fn;
    return get_kernel(col_dtype, chain, L, &fn, ready);
}

fq_status jit_scan(int32_t col_dtype, bool chain, const Launch &L, bool *used, bool force) {
    *used = false;
    const int32_t mode = jit_mode();
    if (mode == FQ_JIT_OFF || !eligible(col_dtype, chain, L)) return FQ_OK;
    if (mode == FQ_JIT_AUTO && L.n < jit_min_rows() && !force) return FQ_OK;
    fq_status err;
    if (!load_rtc(mode, &err)) return err;
    hipFunction_t fn;
    bool ok;
    fq_status s = get_kernel(col_dtype, chain, L, &fn, &ok);
    if (s != FQ_OK) return s;
    if (!fn) return FQ_OK;
    HostConsts hc;
    pack_consts(L, hc);
    const void *col = L.col;
    long long n = L.n, head = L.head, R = L.block_rows;
    const uint64_t *bitmap = L.pred.bitmap;
    Partial *parts = L.parts;
    void *args[] = {&col, &n, &head, &R, &bitmap, &hc, &parts};
    FQ_HIP_TRY(hipModuleLaunchKernel(fn, (unsigned)L.grid, 1, 1, kThreads, 1, 1, 0, L.stream, args, nullptr));
    g_jit_launches += 1;
    *used = true;
    return FQ_OK;
}


namespace {

struct GroupFns {
    hipFunction_t agg = nullptr, part = nullptr, bins = nullptr;
};
std::unordered_map<std::string, GroupFns> g_group_cache;

// the shape's module (compiled once): *out stays empty when only validated
fq_status get_group_fns(int32_t col_dtype, const GroupLaunch &G, GroupFns *out) {
    fq_status err;
    if (!load_rtc(FQ_JIT_ALWAYS, &err)) return err;
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess) {
        (void)hipGetLastError();
        dev = -1;
    }
    const std::string key = group_shape_key(G, col_dtype, dev);
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_group_cache.find(key);
    if (it == g_group_cache.end()) {
        Gen g;
        std::string src;
        Compiled c;
        if (!gen_groupby_source(G, col_dtype, g, src))
            return fqc::fail(FQ_E_UNSUPPORTED, "GROUP BY: key/aggregate types outside the device path");
        fq_status s = compile(src, dev, c, "fq_jit_groupby");
        if (s != FQ_OK) return s;
        int scratch = 0;
        if (dev >= 0 && hipFuncGetAttribute(&scratch, HIP_FUNC_ATTRIBUTE_LOCAL_SIZE_BYTES, c.fn) == hipSuccess &&
            scratch > 0) {
            // The clustered-key layout (mode 1) must not cost the shape
            // register spills: 64-bit magic keys (number / 1e7) left 1,024
            // threads with 52 bytes of scratch and ran 1.8 -> 2.4 ms per
            // 10 GB in mode 0.  Their runs are longer than a lane's rows
            // apart, where mode 0 merges them anyway -- recompile without it.
            (void)hipModuleUnload(c.mod);
            c = Compiled{};
            src.clear();
            Gen g2;
            if (!gen_groupby_source(G, col_dtype, g2, src, false))
                return fqc::fail(FQ_E_UNSUPPORTED, "GROUP BY: key/aggregate types outside the device path");
            s = compile(src, dev, c, "fq_jit_groupby");
            if (s != FQ_OK) return s;
        }
        (void)hipGetLastError();
        if (dev < 0) {  // validated only
            *out = GroupFns{};
            return FQ_OK;
        }
        GroupFns f;
        f.agg = c.fn;
        FQ_HIP_TRY(hipModuleGetFunction(&f.part, c.mod, "fq_jit_gpart"));
        FQ_HIP_TRY(hipModuleGetFunction(&f.bins, c.mod, "fq_jit_groupby_bins"));
        it = g_group_cache.emplace(key, f).first;
    }
    *out = it->second;
    return FQ_OK;
}

struct GroupTab {
    uint64_t *keys;
    uint64_t *st[FQ_MAX_GROUP_AGGS];
    uint32_t *hdr;
    long long mask;
    int rmask;
};

GroupTab group_tab(const GroupLaunch &G) {
    GroupTab tab;
    tab.keys = G.keys;
    for (int a = 0; a < FQ_MAX_GROUP_AGGS; ++a) tab.st[a] = G.states[a];
    tab.hdr = G.hdr;
    tab.mask = (long long)G.capacity - 1;
    tab.rmask = group_replicas(G.capacity) - 1;
    return tab;
}

}  // namespace

fq_status jit_groupby(int32_t col_dtype, const GroupLaunch &G) {
    GroupFns f;
    fq_status s = get_group_fns(col_dtype, G, &f);
    if (s != FQ_OK || !f.agg || !G.col || G.n == 0) return s;
    HostGroupConsts hc;
    pack_group_consts(G, hc);
    GroupTab tab = group_tab(G);
    const void *col = G.col;
    long long n = G.n, head = G.head;
    const uint64_t *bitmap = G.pred.bitmap;
    void *args[] = {&col, &n, &head, &bitmap, &hc, &tab};
    FQ_HIP_TRY(hipModuleLaunchKernel(f.agg, (unsigned)G.grid, 1, 1, (unsigned)G.threads, 1, 1, 0, G.stream, args, nullptr));
    g_jit_launches += 1;
    return FQ_OK;
}

fq_status jit_groupby_partitioned(int32_t col_dtype, const GroupLaunch &G, const GroupPartition &X) {
    GroupFns f;
    fq_status s = get_group_fns(col_dtype, G, &f);
    if (s != FQ_OK || !f.agg || !G.col || G.n == 0) return s;
    HostGroupConsts hc;
    pack_group_consts(G, hc);
    GroupTab tab = group_tab(G);
    const void *col = G.col;
    long long n = G.n;
    const uint64_t *bitmap = G.pred.bitmap;
    int log2p = X.log2p;
    uint32_t *used = X.used, *bin_blocks = X.bin_blocks, *blk_bin = X.blk_bin, *blk_fill = X.blk_fill;
    unsigned q = X.q;
    void *vals = X.vals;
    uint32_t *hdr = G.hdr;
    FQ_HIP_TRY(hipMemsetAsync(X.head, 0, X.head_bytes, G.stream));
    void *a1[] = {&col, &n, &bitmap, &hc, &used, &bin_blocks, &blk_bin, &blk_fill, &q, &vals, &log2p, &hdr};
    FQ_HIP_TRY(hipModuleLaunchKernel(f.part, (unsigned)X.grid, 1, 1, (unsigned)G.threads, 1, 1, 0, G.stream, a1, nullptr));
    if ((s = launch_group_part_blocks(X, G.stream)) != FQ_OK) return s;
    const void *cvals = X.vals;
    const uint64_t *order = X.order;
    const uint32_t *bstart = X.bstart;
    void *a2[] = {&cvals, &order, &bstart, &log2p, &hc, &tab, &col};
    FQ_HIP_TRY(hipModuleLaunchKernel(f.bins, (unsigned)X.bins_grid, 1, 1, (unsigned)G.threads, 1, 1, 0, G.stream, a2,
                                     nullptr));
    g_jit_launches += 2;
    return FQ_OK;
}

namespace {

struct ProjKernels {
    hipFunction_t bits = nullptr, scatter = nullptr, map = nullptr, blocks = nullptr;
    hipModule_t mod = nullptr;
};
std::unordered_map<std::string, ProjKernels> g_proj_cache;

fq_status get_proj_kernels(int32_t col_dtype, const ProjLaunch &P, ProjKernels *out) {
    fq_status err;
    if (!load_rtc(FQ_JIT_ALWAYS, &err)) return err;
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess) {
        (void)hipGetLastError();
        dev = -1;
    }
    const std::string key = proj_shape_key(P, col_dtype, dev);
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_proj_cache.find(key);
    if (it == g_proj_cache.end()) {
        Gen g;
        std::string src;
        Compiled c;
        if (!gen_project_source(P, col_dtype, dev, g, src))
            return fqc::fail(FQ_E_UNSUPPORTED, "fused projection: column/expression types outside the device path");
        fq_status s = compile(src, dev, c, "fq_jit_pselect");
        if (s != FQ_OK) return s;
        ProjKernels k;
        if (dev < 0) {  // validated only
            *out = k;
            return FQ_OK;
        }
        k.scatter = c.fn;
        k.mod = c.mod;
        FQ_HIP_TRY(hipModuleGetFunction(&k.bits, c.mod, "fq_jit_pbits"));
        FQ_HIP_TRY(hipModuleGetFunction(&k.map, c.mod, "fq_jit_pmap"));
        FQ_HIP_TRY(hipModuleGetFunction(&k.blocks, c.mod, "fq_jit_pblocks"));
        it = g_proj_cache.emplace(key, k).first;
    }
    *out = it->second;
    return FQ_OK;
}

int proj_grid(int64_t units, int per_wg) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipGetLastError();
    const int64_t want = (units + per_wg - 1) / per_wg;
    const int64_t cap = (int64_t)cus * 8;
    return (int)std::max<int64_t>(1, std::min<int64_t>(want, cap));
}

}  // namespace

bool jit_project_available() { return jit_mode() != FQ_JIT_OFF && rtc().ok; }

fq_status jit_project_prepare(int32_t col_dtype, const ProjLaunch &P) {
    ProjKernels k;
    return get_proj_kernels(col_dtype, P, &k);
}

fq_status jit_project_bits(int32_t col_dtype, const ProjLaunch &P, uint64_t *d_bitmap, uint32_t *d_flag) {
    ProjKernels k;
    fq_status s = get_proj_kernels(col_dtype, P, &k);
    if (s != FQ_OK || !k.bits || P.n == 0) return s;
    HostProjConsts hc;
    pack_proj_consts(P, hc);
    const void *col = P.col;
    long long n = P.n;
    const int64_t nwords = (P.n + 63) / 64;
    void *args[] = {&col, &n, &hc, &d_bitmap, &d_flag};
    FQ_HIP_TRY(hipModuleLaunchKernel(k.bits, (unsigned)proj_grid(nwords, 4 * 8), 1, 1, kThreads, 1, 1, 0, P.stream,
                                     args, nullptr));
    g_jit_launches += 1;
    return FQ_OK;
}

fq_status jit_project_select(int32_t col_dtype, const ProjLaunch &P, const uint64_t *d_bitmap, uint64_t *status,
                             uint32_t *ticket, uint32_t *d_flags, uint64_t *d_total) {
    ProjKernels k;
    fq_status s = get_proj_kernels(col_dtype, P, &k);
    if (s != FQ_OK || !k.scatter || P.n == 0) return s;
    HostProjConsts hc;
    pack_proj_consts(P, hc);
    struct {
        void *p[FQ_MAX_PROJECT];
    } outs;
    for (int j = 0; j < FQ_MAX_PROJECT; ++j) outs.p[j] = j < P.n_out ? P.out[j] : nullptr;
    const void *col = P.col;
    long long n = P.n;
    const int64_t ntiles = (P.n + select_tile_rows() - 1) / select_tile_rows();
    void *args[] = {&col, &n, &hc, &d_bitmap, &outs, &status, &ticket, &d_flags, &d_total};
    const int wg_per_cu = (int)fqc::knob(FQ_TUNE_SELECT_WG_PER_CU);
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipGetLastError();
    // one resident wave of workgroups: at most the occupancy the compiled kernel
    // allows per CU (more would only queue behind them)
    hipFunction_t fn = k.scatter;
    const int threads = select_threads();
    static std::mutex occ_mu;
    static std::unordered_map<hipFunction_t, int> occ_cache;
    int occ = 0;
    {
        std::lock_guard<std::mutex> lk(occ_mu);
        auto it = occ_cache.find(fn);
        if (it != occ_cache.end()) {
            occ = it->second;
        } else {
            if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, threads, 0) != hipSuccess) occ = 1;
            (void)hipGetLastError();
            occ = std::max(1, occ);
            occ_cache.emplace(fn, occ);
        }
    }
    const int64_t grid = std::max<int64_t>(1, std::min<int64_t>(ntiles, (int64_t)cus * std::min(wg_per_cu, occ)));
    FQ_HIP_TRY(hipModuleLaunchKernel(fn, (unsigned)grid, 1, 1, (unsigned)threads, 1, 1, 0, P.stream,
                                     args, nullptr));
    g_jit_launches += 1;
    return FQ_OK;
}

fq_status jit_project_blocks(int32_t col_dtype, const ProjLaunch &P, int64_t block_rows, const uint64_t *d_bitmap,
                             int64_t *d_counts, uint32_t *d_flags, uint64_t *d_total, uint32_t *d_ticket) {
    ProjKernels k;
    fq_status s = get_proj_kernels(col_dtype, P, &k);
    if (s != FQ_OK || !k.blocks || P.n == 0) return s;
    if (block_rows < kProjectBlockTile) return fqc::fail(FQ_E_INVALID, "jit_project_blocks: block_rows below the tile");
    HostProjConsts hc;
    pack_proj_consts(P, hc);
    struct {
        void *p[FQ_MAX_PROJECT];
    } outs;
    for (int j = 0; j < FQ_MAX_PROJECT; ++j) outs.p[j] = j < P.n_out ? P.out[j] : nullptr;
    const void *col = P.col;
    // a block longer than the column is the whole column (one block; keeps n + B in range)
    long long n = P.n, B = std::min<int64_t>(block_rows, P.n);
    const int64_t nb = (P.n + B - 1) / B;
    int al = 1;  // PB_STAGE row pairs need 16-byte aligned outputs
    for (int j = 0; j < P.n_out; ++j) al &= ((uintptr_t)P.out[j] & 15) == 0;
    void *args[] = {&col, &n, &B, &hc, &d_bitmap, &outs, &d_counts, &d_flags, &d_total, &d_ticket, &al};
    hipFunction_t fn = k.blocks;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipGetLastError();
    // one wave of workgroups (each owns an equal run of whole blocks): a grid
    // above the resident capacity would leave a second, partial wave
    static std::mutex occ_mu;
    static std::unordered_map<hipFunction_t, int> occ_cache;
    int occ = 0;
    {
        std::lock_guard<std::mutex> lk(occ_mu);
        auto it = occ_cache.find(fn);
        if (it != occ_cache.end()) {
            occ = it->second;
        } else {
            if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, kProjectBlockThreads, 0) != hipSuccess)
                occ = 1;
            (void)hipGetLastError();
            occ = std::max(1, occ);
            occ_cache.emplace(fn, occ);
        }
    }
    const int wg_per_cu = (int)fqc::knob(FQ_TUNE_SELECT_BLOCKS_WG_PER_CU);
    const int64_t grid = std::max<int64_t>(1, std::min<int64_t>(nb, (int64_t)cus * std::min(wg_per_cu, occ)));
    FQ_HIP_TRY(hipModuleLaunchKernel(fn, (unsigned)grid, 1, 1, kProjectBlockThreads, 1, 1, 0, P.stream, args,
                                     nullptr));
    g_jit_launches += 1;
    return FQ_OK;
}

fq_status jit_project_map(int32_t col_dtype, const ProjLaunch &P, uint32_t *d_flag) {
    ProjKernels k;
    fq_status s = get_proj_kernels(col_dtype, P, &k);
    if (s != FQ_OK || !k.map || P.n == 0) return s;
    HostProjConsts hc;
    pack_proj_consts(P, hc);
    struct {
        void *p[FQ_MAX_PROJECT];
    } outs;
    int aligned = ((uintptr_t)P.col & 15u) == 0;
    for (int j = 0; j < FQ_MAX_PROJECT; ++j) {
        outs.p[j] = j < P.n_out ? P.out[j] : nullptr;
        if (j < P.n_out && ((uintptr_t)P.out[j] & 15u)) aligned = 0;
    }
    const void *col = P.col;
    long long n = P.n;
    void *args[] = {&col, &n, &hc, &outs, &aligned, &d_flag};
    FQ_HIP_TRY(hipModuleLaunchKernel(k.map, (unsigned)proj_grid(n / 2, kThreads * 4), 1, 1, kThreads, 1, 1, 0, P.stream,
                                     args, nullptr));
    g_jit_launches += 1;
    return FQ_OK;
}

}  // namespace fqk

extern "C" {

fq_status fq_jit_config(int32_t mode, int64_t min_rows) {
    if (mode < FQ_JIT_OFF || mode > FQ_JIT_ALWAYS) return fqc::fail(FQ_E_INVALID, "fq_jit_config: bad mode");
    if (min_rows < 0) return fqc::fail(FQ_E_INVALID, "fq_jit_config: negative min_rows");
    fqk::g_mode.store(mode);
    fqk::g_min_rows.store(min_rows);
    return FQ_OK;
}

fq_status fq_jit_get_stats(fq_jit_stats *out) {
    if (!out) return fqc::fail(FQ_E_INVALID, "fq_jit_get_stats: NULL argument");
    out->kernels_compiled = fqk::g_compiled.load();
    out->jit_launches = fqk::g_jit_launches.load();
    out->interp_launches = fqk::g_interp_launches.load();
    out->compile_ms = fqk::g_compile_us.load() / 1000.0;
    out->available = fqk::g_available.load();
    out->mode = fqk::jit_mode();
    out->min_rows = fqk::jit_min_rows();
    return FQ_OK;
}

}  // extern "C"
