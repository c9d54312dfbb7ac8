"""Loads lib/libfq_amd.so (the gfx950 kernels + C ABI) and declares the
prototypes of include/fq_gpu.h and include/fq_engine.h.

There is no fallback: if the shared library is missing the import fails,
and every compute entry point fails loudly without a GPU.
"""
import ctypes as C
import os

from . import abi

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.normpath(os.path.join(_HERE, "..", "lib", "libfq_amd.so"))

# Exported symbols promised by include/fq_gpu.h (checked by the CPU tests)
GPU_SYMBOLS = [
    "fq_abi_version", "fq_last_error", "fq_device_count", "fq_fill_numbers_u64", "fq_fill_value",
    "fq_fill_splitmix64", "fq_aggregate_workspace_bytes", "fq_aggregate",
    "fq_arith_result_type", "fq_arith", "fq_compare", "fq_filter_workspace_bytes",
    "fq_filter_compact", "fq_state_merge", "fq_jit_config", "fq_jit_get_stats", "fq_jit_prepare",
    "fq_group_table_bytes", "fq_group_table_init", "fq_group_aggregate", "fq_group_table_count",
    "fq_group_table_extract", "fq_logic", "fq_filter_project_workspace_bytes", "fq_filter_project",
    "fq_predicate_bitmap", "fq_group_partition_workspace_bytes", "fq_group_aggregate_partitioned",
    "fq_group_dense_keys", "fq_group_table_merge", "fq_tune_set", "fq_tune_get", "fq_tune_reset",
    "fq_tune_jit_dump_dir", "fq_filter_project_blocks_workspace_bytes", "fq_filter_project_blocks",
    "fq_blocks_compact_workspace_bytes", "fq_blocks_compact",
]


class FQError(RuntimeError):
    """A non-OK fq_status; .status is the code, str() is fq_last_error()."""

    def __init__(self, status, msg):
        super().__init__(msg)
        self.status = status


def _load():
    # torch ships its own libamdhip64.so (SONAME libamdhip64.so.7).  Load it
    # first so libfq_amd.so binds to the SAME HIP runtime as the tensors we are
    # handed; loading /opt/rocm's copy first gives the process two runtimes
    # and the second one reports hipErrorNoDevice.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError("fq_amd: %s is missing; run `make -C fuse-query_amd` "
                          "(or __graft_entry__.build())" % LIB_PATH)
    return C.CDLL(LIB_PATH)


lib = _load()

P = C.POINTER
vp = C.c_void_p

_protos = {
    "fq_abi_version": (C.c_int32, []),
    "fq_last_error": (C.c_char_p, []),
    "fq_device_count": (C.c_int32, [P(C.c_int32)]),
    "fq_fill_numbers_u64": (C.c_int32, [vp, C.c_uint64, C.c_uint64, vp]),
    "fq_fill_splitmix64": (C.c_int32, [vp, C.c_uint64, C.c_uint64, C.c_uint64, vp]),
    "fq_aggregate_workspace_bytes": (C.c_size_t, [C.c_int64]),
    "fq_aggregate": (C.c_int32, [P(abi.fq_col), C.c_int64, P(abi.fq_pred), P(abi.fq_expr),
                                 C.c_uint32, vp, vp, C.c_size_t, vp]),
    "fq_arith_result_type": (C.c_int32, [C.c_int32, C.c_int32, C.c_int32, P(C.c_int32)]),
    "fq_arith": (C.c_int32, [C.c_int32, P(abi.fq_col), P(abi.fq_value), P(abi.fq_col),
                             P(abi.fq_value), P(abi.fq_col), vp, vp]),
    "fq_compare": (C.c_int32, [C.c_int32, P(abi.fq_col), P(abi.fq_value), P(abi.fq_col),
                               P(abi.fq_value), vp, C.c_int64, vp, vp]),
    "fq_filter_workspace_bytes": (C.c_size_t, [C.c_int64]),
    "fq_filter_compact": (C.c_int32, [P(abi.fq_col), vp, vp, P(C.c_int64), vp, C.c_size_t, vp]),
    "fq_state_merge": (C.c_int32, [P(abi.fq_agg_state), C.c_int32, P(abi.fq_agg_state)]),
    "fq_jit_config": (C.c_int32, [C.c_int32, C.c_int64]),
    "fq_jit_get_stats": (C.c_int32, [P(abi.fq_jit_stats)]),
    "fq_jit_prepare": (C.c_int32, [P(abi.fq_col), C.c_int64, P(abi.fq_pred), P(abi.fq_expr), C.c_uint32,
                                   P(C.c_int32)]),
    "fq_logic": (C.c_int32, [C.c_int32, vp, vp, vp, C.c_int64, vp]),
    "fq_filter_project_workspace_bytes": (C.c_size_t, [C.c_int64]),
    "fq_filter_project": (C.c_int32, [P(abi.fq_col), P(abi.fq_pred), P(abi.fq_expr), C.c_int32, P(vp),
                                      P(C.c_int64), vp, C.c_size_t, vp]),
    "fq_filter_project_blocks_workspace_bytes": (C.c_size_t, []),
    "fq_filter_project_blocks": (C.c_int32, [P(abi.fq_col), C.c_int64, P(abi.fq_pred), P(abi.fq_expr), C.c_int32,
                                             P(vp), vp, P(C.c_int64), vp, C.c_size_t, vp]),
    "fq_blocks_compact_workspace_bytes": (C.c_size_t, [C.c_int64]),
    "fq_blocks_compact": (C.c_int32, [C.c_int32, P(vp), C.c_int64, C.c_int64, vp, P(vp), P(C.c_int64), vp,
                                      C.c_size_t, vp]),
    "fq_predicate_bitmap": (C.c_int32, [P(abi.fq_col), P(abi.fq_pred), vp, vp, vp]),
    "fq_group_table_bytes": (C.c_size_t, [C.c_int64, C.c_int32]),
    "fq_group_table_init": (C.c_int32, [P(abi.fq_group_table), vp]),
    "fq_group_aggregate": (C.c_int32, [P(abi.fq_group_table), P(abi.fq_col), P(abi.fq_pred), P(abi.fq_expr),
                                       P(abi.fq_expr), vp]),
    "fq_group_partition_workspace_bytes": (C.c_size_t, [C.c_int64, C.c_int32]),
    "fq_group_dense_keys": (C.c_int64, [C.c_int32, P(abi.fq_expr), C.c_int32]),
    "fq_group_aggregate_partitioned": (C.c_int32, [P(abi.fq_group_table), P(abi.fq_col), P(abi.fq_pred),
                                                   P(abi.fq_expr), P(abi.fq_expr), C.c_int32, vp, C.c_size_t, vp]),
    "fq_group_table_count": (C.c_int32, [P(abi.fq_group_table), P(C.c_int64), vp]),
    "fq_group_table_extract": (C.c_int32, [P(abi.fq_group_table), vp, P(C.c_void_p), C.c_int64, P(C.c_int64),
                                           vp]),
    "fq_group_table_merge": (C.c_int32, [P(abi.fq_group_table), vp, P(C.c_void_p), C.c_int64, vp]),
    "fq_tune_set": (C.c_int32, [C.c_int32, C.c_int64]),
    "fq_tune_get": (C.c_int64, [C.c_int32]),
    "fq_tune_reset": (C.c_int32, []),
    "fq_tune_jit_dump_dir": (C.c_int32, [C.c_char_p]),
}
for _name, (_res, _args) in _protos.items():
    _f = getattr(lib, _name)
    _f.restype = _res
    _f.argtypes = _args


def last_error():
    m = lib.fq_last_error()
    return m.decode() if m else ""


def check(status):
    if status != abi.FQ_OK:
        raise FQError(status, last_error())
    return status
