// Host-side helpers shared by the C-ABI translation units: thread-local error
// text (FuseQueryError display strings, src/error.rs:10-22) and HIP checks.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "fq_gpu.h"

namespace fqc {

// Records `msg` verbatim as the thread's last error and returns `st`.
fq_status fail(fq_status st, const std::string &msg);
// FuseQueryError::Internal(msg) -> "Internal Error: msg"
fq_status internal(const std::string &msg);
fq_status hip_fail(hipError_t e, const char *what);
// 8 words of pinned host memory owned by the calling thread (nullptr if the
// allocation failed): the staging buffer for the few device-to-host reads of
// counts and flags per call, which from pageable memory cost ~25 us of host
// time each (profiles/r01_readme_limit_trace.txt)
uint64_t *host_staging();

int device_cu_count();  // CUs of the current device (cached per device)

// Launch-shape knob FQ_TUNE_* (fq_knobs.cpp): the compiled-in default unless a
// tuning tool set it through fq_tune_set; read at every launch.
int64_t knob(int k);
// fq_tune_jit_dump_dir's directory ("" = off)
std::string jit_dump_dir();

const char *dtype_name(int32_t dt);  // arrow DataType Debug name ("UInt64", ...)
int dtype_size(int32_t dt);          // bytes per value; 0 for non-primitive
bool dtype_is_numeric(int32_t dt);
bool dtype_is_signed_int(int32_t dt);
bool dtype_is_unsigned_int(int32_t dt);
bool dtype_is_float(int32_t dt);

// numerical_coercion / equal_coercion (src/datavalues/data_type.rs:27-98).
// On error records "Internal Error: Unsupported (L) op (R)" and returns it.
fq_status numerical_coercion(const char *op, int32_t lhs, int32_t rhs, int32_t *out);
fq_status equal_coercion(const char *op, int32_t lhs, int32_t rhs, int32_t *out);
const char *arith_op_str(int32_t op);  // "+", "-", "*", "/", "%"
const char *cmp_op_str(int32_t cmp);   // "=", "<", "<=", ">", ">="

// arrow cast of one scalar (num-traits NumCast semantics): false = null.
bool cast_scalar(uint64_t bits, int32_t from, int32_t to, uint64_t *out);

}  // namespace fqc

#define FQ_HIP_TRY(expr)                                          \
    do {                                                          \
        hipError_t fq_e_ = (expr);                                \
        if (fq_e_ != hipSuccess) return fqc::hip_fail(fq_e_, #expr); \
    } while (0)

// Internal entry points the engine calls beside the C ABI (fq_filter.hip).
namespace fqk {
// fq_filter_project_blocks without waiting (the engine's ProjectionTransform,
// which keeps one queue busy with several pipes' launches): enqueued on
// `stream`; when the stream reaches it, {kept rows, flag words} land in
// h_result[0..1] (pinned host memory), to be turned into the call's status
// and row count by filter_project_blocks_result after waiting.  ev_start /
// ev_end (optional) bracket the kernel alone.  d_result == nullptr: the
// workspace is zeroed before the kernel and the words copied after it; else
// d_result is the device address of h_result (mapped host memory), the
// workspace is zero already (zeroed once by the caller) and a one-thread
// kernel after the projection hands the words over and re-zeroes it.
fq_status filter_project_blocks_enqueue(const fq_col *col, int64_t block_rows, const fq_pred *pred,
                                        const fq_expr *values, int32_t n_out, void *const *d_out, int64_t *d_counts,
                                        uint64_t *h_result, uint64_t *d_result, void *d_ws, size_t ws_bytes,
                                        void *ev_start, void *ev_end, void *stream);
fq_status filter_project_blocks_result(const uint64_t *h_result, int64_t *out_len);
}  // namespace fqk
