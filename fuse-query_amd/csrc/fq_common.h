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
