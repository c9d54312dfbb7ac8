"""Multi-GPU AggregateFinal: one process per GPU, numbers_mt partitions
sharded [8r/G, 8(r+1)/G), and the partial states exchanged by the
native protocol of include/fq_comm.h -- ONE all-reduce (two for GROUP BY
states above 4 KB) -- then AggregateFinal in rank order on every rank.

The reference's only "exchange" is the in-process MergeProcessor channel of
JSON states (processor_merge.rs:45-63, transform_aggregate_partial.rs:61-72).
Here every rank writes its serialised states into ITS OWN row of a zeroed
u64 buffer and a wrapping SUM all-reduce turns that into an all-gather (each
word has exactly one non-zero contributor, so the result is bit-exact).

Transports for the collective:
  * RcclComm -- the library's own RCCL communicator (ncclCommInitRank, one
    per GPU, xGMI): fq_engine_execute_rccl runs partial -> exchange -> final
    without leaving C++.  torch.distributed only ships the 128-byte unique id.
  * any torch.distributed group (gloo on CPU for the tests, or nccl) through
    an fq_allreduce_fn callback into the same native protocol.
"""
import ctypes as C

import numpy as np
import torch
import torch.distributed as dist

from . import abi
from ._lib import check, lib
from .engine import Result

P = C.POINTER
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int32, P(C.c_uint64), C.c_int64, C.c_void_p)
COMM_ID_BYTES = 128
STATE_CAP = 4096  # FQ_EXCHANGE_CAP_BYTES

COMM_SYMBOLS = [
    "fq_exchange_fail", "fq_exchange_states", "fq_exchange_states_sized", "fq_engine_execute_exchange",
    "fq_engine_execute_exchange_row",
    "fq_comm_unique_id", "fq_comm_init", "fq_comm_init_timeout", "fq_comm_set_timeout", "fq_comm_info",
    "fq_comm_destroy", "fq_state_allreduce", "fq_comm_allreduce_u64", "fq_engine_execute_rccl",
    "fq_engine_execute_rccl_row",
]
COMM_TIMEOUT_MS = 60000  # FQ_COMM_TIMEOUT_MS
_protos = {
    "fq_exchange_fail": (C.c_int32, [C.c_int32, C.c_char_p]),
    "fq_exchange_states": (C.c_int32, [C.c_void_p, C.c_size_t, C.c_int32, C.c_int32, ALLREDUCE_FN, C.c_void_p,
                                       P(C.c_void_p), P(C.c_size_t)]),
    "fq_exchange_states_sized": (C.c_int32, [C.c_void_p, C.c_size_t, C.c_size_t, C.c_int32, C.c_int32, ALLREDUCE_FN,
                                             C.c_void_p, P(C.c_void_p), P(C.c_size_t)]),
    "fq_engine_execute_exchange": (C.c_int32, [C.c_void_p, C.c_char_p, C.c_int32, C.c_int32, ALLREDUCE_FN,
                                               C.c_void_p, P(C.c_void_p)]),
    "fq_engine_execute_exchange_row": (C.c_int32, [C.c_void_p, C.c_char_p, C.c_int32, C.c_int32, ALLREDUCE_FN,
                                                   C.c_void_p, P(abi.fq_value), C.c_int32, P(C.c_int32)]),
    "fq_comm_init_timeout": (C.c_int32, [C.c_int32, C.c_int32, C.c_int32, C.c_void_p, C.c_int64, P(C.c_void_p)]),
    "fq_comm_set_timeout": (C.c_int32, [C.c_void_p, C.c_int64]),
    "fq_engine_execute_rccl_row": (C.c_int32, [C.c_void_p, C.c_char_p, C.c_void_p, P(abi.fq_value), C.c_int32,
                                               P(C.c_int32)]),
    "fq_comm_unique_id": (C.c_int32, [C.c_void_p]),
    "fq_comm_init": (C.c_int32, [C.c_int32, C.c_int32, C.c_int32, C.c_void_p, P(C.c_void_p)]),
    "fq_comm_info": (C.c_int32, [C.c_void_p, P(C.c_int32), P(C.c_int32)]),
    "fq_comm_destroy": (None, [C.c_void_p]),
    "fq_state_allreduce": (C.c_int32, [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]),
    "fq_comm_allreduce_u64": (C.c_int32, [P(C.c_uint64), C.c_int64, C.c_void_p]),
    "fq_engine_execute_rccl": (C.c_int32, [C.c_void_p, C.c_char_p, C.c_void_p, P(C.c_void_p)]),
}
for _n, (_r, _a) in _protos.items():
    _f = getattr(lib, _n)
    _f.restype = _r
    _f.argtypes = _a


def torch_allreduce_fn(group=None, timeout_s=None):
    """An fq_allreduce_fn over a torch.distributed group (keep the returned
    object alive while the library may call it).  timeout_s: the deadline of
    each all-reduce, as fq_comm's for RCCL -- a peer that never arrives makes
    the exchange fail with FQ_E_RCCL and this rank named, instead of a wait
    without end (the group's own timeout is the fallback)."""
    import datetime
    on_gpu = dist.get_backend(group) == "nccl"
    rank, world = dist.get_rank(group), dist.get_world_size(group)

    def cb(ptr, n, _user):
        import time
        t0 = time.monotonic()
        try:
            words = np.ctypeslib.as_array(ptr, shape=(n,)).view(np.int64)
            t = torch.from_numpy(words)
            d = t.cuda() if on_gpu else t  # gloo: in place on the library's words
            work = dist.all_reduce(d, op=dist.ReduceOp.SUM, group=group, async_op=True)
            if timeout_s is None:
                work.wait()
            elif not work.wait(timeout=datetime.timedelta(seconds=timeout_s)):
                raise TimeoutError
            if on_gpu:
                t.copy_(d.cpu())
            return abi.FQ_OK
        except Exception as e:
            timed_out = timeout_s is not None and (isinstance(e, TimeoutError) or
                                                   time.monotonic() - t0 >= 0.9 * timeout_s)
            why = ("did not complete within %g s: a peer rank failed or never reached it" % timeout_s if timed_out
                   else "failed: %s" % (str(e).splitlines()[0][:200] if str(e) else type(e).__name__))
            return lib.fq_exchange_fail(abi.FQ_E_RCCL,
                                        ("rank %d of %d: the state all-reduce %s" % (rank, world, why)).encode())

    return ALLREDUCE_FN(cb)


class RcclComm:
    """The library's RCCL communicator over all ranks of the default
    torch.distributed group (which only carries the unique id)."""

    def __init__(self, device, group=None, timeout_ms=COMM_TIMEOUT_MS):
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        uid = C.create_string_buffer(COMM_ID_BYTES)
        if self.rank == 0:
            check(lib.fq_comm_unique_id(uid))
        box = [uid.raw if self.rank == 0 else None]
        dist.broadcast_object_list(box, src=0, group=group)
        uid = C.create_string_buffer(box[0], COMM_ID_BYTES)
        h = C.c_void_p()
        check(lib.fq_comm_init_timeout(device, self.world, self.rank, uid, int(timeout_ms), C.byref(h)))
        self.h = h

    @classmethod
    def single(cls, device):
        """A one-rank communicator without torch.distributed (the unique id
        never leaves this process): the RCCL exchange path at world 1."""
        self = cls.__new__(cls)
        self.rank, self.world = 0, 1
        uid = C.create_string_buffer(COMM_ID_BYTES)
        check(lib.fq_comm_unique_id(uid))
        h = C.c_void_p()
        check(lib.fq_comm_init(device, 1, 0, uid, C.byref(h)))
        self.h = h
        return self

    def info(self):
        """(rank, world) as the communicator sees them (fq_comm_info)."""
        r, w = C.c_int32(-1), C.c_int32(-1)
        check(lib.fq_comm_info(self.h, C.byref(r), C.byref(w)))
        return r.value, w.value

    def allreduce_(self, words):
        """In-place wrapping u64 sum of a numpy uint64 array over all ranks."""
        assert words.dtype == np.uint64 and words.flags.c_contiguous
        check(lib.fq_comm_allreduce_u64(words.ctypes.data_as(P(C.c_uint64)), words.size, self.h))
        return words

    def close(self):
        if getattr(self, "h", None):
            lib.fq_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def allgather_states(states, group=None, cap=None, timeout_s=None):
    """bytes of this rank -> [bytes of rank 0, ..., rank world-1] (zero padded
    to a common stride) through the native exchange over `group`; `cap`: the
    first round's payload bytes per rank (fq_exchange_states_sized; the same
    on every rank), default FQ_EXCHANGE_CAP_BYTES; timeout_s: each
    all-reduce's deadline (torch_allreduce_fn)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    fn = torch_allreduce_fn(group, timeout_s)
    rows, stride = C.c_void_p(), C.c_size_t()
    if cap is None:
        check(lib.fq_exchange_states(states, len(states), rank, world, fn, None, C.byref(rows), C.byref(stride)))
    else:
        check(lib.fq_exchange_states_sized(states, len(states), cap, rank, world, fn, None, C.byref(rows),
                                           C.byref(stride)))
    blob = C.string_at(rows, stride.value * world)
    return [blob[r * stride.value:(r + 1) * stride.value] for r in range(world)]


def execute(engine, sql, comm=None, group=None):
    """Run an aggregate query across all ranks: local partial on this rank's
    shard -> exchange -> AggregateFinal merge in rank order.  `comm` is an
    RcclComm (native RCCL) or None (the torch.distributed `group`)."""
    out = C.c_void_p()
    if comm is not None:
        check(lib.fq_engine_execute_rccl(engine.h, sql.encode(), comm.h, C.byref(out)))
    else:
        fn = torch_allreduce_fn(group)
        check(lib.fq_engine_execute_exchange(engine.h, sql.encode(), dist.get_rank(group),
                                             dist.get_world_size(group), fn, None, C.byref(out)))
    return Result(out)


def execute_row(engine, sql, comm=None, group=None, row=None, timeout_s=None):
    """execute() for a one-row statement in ONE library call
    (fq_engine_execute_rccl_row / fq_engine_execute_exchange_row): the row's
    values (None for a None value).  `row`: an (abi.fq_value * k) buffer to
    reuse (timed loops); the values are then row[:ncols]."""
    buf = row if row is not None else (abi.fq_value * 8)()
    ncols = C.c_int32(0)
    if comm is not None:
        check(lib.fq_engine_execute_rccl_row(engine.h, sql.encode(), comm.h, buf, len(buf), C.byref(ncols)))
    else:
        fn = torch_allreduce_fn(group, timeout_s)
        check(lib.fq_engine_execute_exchange_row(engine.h, sql.encode(), dist.get_rank(group),
                                                 dist.get_world_size(group), fn, None, buf, len(buf),
                                                 C.byref(ncols)))
    return [v.bits if v.is_some else None for v in buf[:ncols.value]]
