"""The multi-rank path ON THE GPU: 2 processes share cuda:0 (one box has one
GPU), each runs its numbers_mt shard through fq_engine_execute_partial (the
fused scans / GROUP BY kernels), the states go through the native exchange
(fq_engine_execute_exchange) over gloo -- bench.py runs the same protocol over
the library's RCCL communicator -- and every rank's final merge must equal the
single-process oracle."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SQLS = [
    "SELECT sum(number)/count(number), max(number), min(number) FROM system.numbers_mt(%d)",
    "SELECT max(number+1), count(number) FROM system.numbers_mt(%d) WHERE (number%%8)<3",
    "SELECT number%%10, count(number), sum(number)/count(number), max(number+1) "
    "FROM system.numbers_mt(%d) WHERE (number%%8)<3 GROUP BY number%%10",
]


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


ERROR_SQLS = [
    # division by zero only in rank 0's partitions (row 0) / only in rank 1's (row 3e6)
    "SELECT sum(number) FROM system.numbers_mt(%d) WHERE (1000 %% number) = 1000",
    "SELECT max(number) FROM system.numbers_mt(%d) WHERE (1000 %% (number - 3000000)) = 1000",
]


def worker(rank, world, port, n, out_q, sqls=None):
    for p in (os.path.join(ROOT, "fuse-query_amd"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    from fq_amd import dist as fqd
    from fq_amd.engine import Engine

    from fq_amd import FQError

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        with Engine(device=0) as eng:
            out, rounds = [], []
            for sql in (sqls or SQLS):
                r0 = eng.stats()["exchange_rounds"]
                try:
                    out.append(fqd.execute(eng, sql % n).rows)
                except FQError as e:  # every rank must get the error, none may hang
                    out.append(("error", e.status, str(e)))
                rounds.append(eng.stats()["exchange_rounds"] - r0)
        out_q.put((rank, out, rounds))
    finally:
        dist.destroy_process_group()


def test_an_error_on_one_rank_reaches_every_rank():
    # a rank whose partitions fail still takes part in the exchange (an error
    # record instead of states): no rank waits in the collective, all report it
    world, n = 2, 4_000_000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, n, q, ERROR_SQLS)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from fq_amd import abi
    for rank, out, _ in results:
        for got in out:
            assert got == ("error", abi.FQ_E_DIVIDE_BY_ZERO, "Internal Error: Divide by zero error"), (rank, got)


def test_two_ranks_on_the_gpu_match_the_oracle():
    import fq_ref as R
    world, n = 2, 4_000_000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    num = R.E_field("number")
    c = R.E_const
    exp3 = [tuple(v.value for v in R.aggregate_query(n, [
        R.E_bin("/", R.E_fn("sum", num), R.E_fn("count", num)), R.E_fn("max", num), R.E_fn("min", num)]))]
    where = R.E_bin("<", R.E_bin("%", num, c(8)), c(3))
    exp4 = [tuple(v.value for v in R.aggregate_query(n, [R.E_fn("max", R.E_bin("+", num, c(1))),
                                                         R.E_fn("count", num)], where=where))]
    expg = R.group_by_query(n, R.E_bin("%", num, c(10)),
                            [R.E_fn("count", num), R.E_bin("/", R.E_fn("sum", num), R.E_fn("count", num)),
                             R.E_fn("max", R.E_bin("+", num, c(1)))], where=where)
    for rank, out, rounds in results:
        assert out[0] == exp3, rank
        assert out[1] == exp4, rank
        assert out[2] == expg, rank
        # one all-reduce each: C3 / C4 sized to their states, the 10-group
        # GROUP BY rows within the default cap (no lengths-only first round)
        assert rounds == [1, 1, 1], rank


def rccl_worker(port, n, out_q):
    for p in (os.path.join(ROOT, "fuse-query_amd"),):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import ctypes as C

    import numpy as np
    import torch
    import torch.distributed as dist

    from fq_amd import dist as fqd
    from fq_amd._lib import check, lib
    from fq_amd.engine import Engine

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        comm = fqd.RcclComm(0)
        r, w = C.c_int32(-1), C.c_int32(-1)
        check(lib.fq_comm_info(comm.h, C.byref(r), C.byref(w)))
        words = np.array([1, 2**64 - 1, 12345], dtype=np.uint64)
        host = comm.allreduce_(words.copy()).tolist()
        d = torch.arange(1000, dtype=torch.int64, device="cuda")
        s = torch.cuda.current_stream()
        check(lib.fq_state_allreduce(comm.h, C.c_void_p(d.data_ptr()), d.numel(), C.c_void_p(s.cuda_stream)))
        torch.cuda.synchronize()
        dev_ok = bool((d.cpu() == torch.arange(1000)).all())
        with Engine(device=0) as eng:
            out = [(fqd.execute(eng, sql % n, comm).rows, eng.execute(sql % n).rows) for sql in SQLS]
        comm.close()
        out_q.put(((r.value, w.value), host, dev_ok, out))
    finally:
        dist.destroy_process_group()


def test_native_rccl_comm_single_rank():
    """The library's own RCCL communicator (fq_comm_init / fq_state_allreduce /
    fq_engine_execute_rccl) at world 1 -- the box has one GPU and RCCL refuses
    two ranks on one device; bench.py runs the same calls at 2..8 ranks."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=rccl_worker, args=(free_port(), 3_000_017, q))
    p.start()
    info, host, dev_ok, out = q.get(timeout=300)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert info == (0, 1)
    assert host == [1, 2**64 - 1, 12345]
    assert dev_ok
    for dist_rows, local_rows in out:
        assert dist_rows == local_rows


def test_world8_bench_rehearsal_on_one_gpu():
    """bench.py's world > 1 path at the C5 shape, started the way the driver's
    bench command is (`python3 bench.py --gpus 8 ...`, NO external launcher:
    bench.py starts the 8 ranks itself): the ranks (gloo) share the box's one
    GPU, numbers_mt(1e10) split into one 10 GB partition per rank (80 GB
    resident in total), the partial states exchanged through the native
    protocol in one all-reduce sized to them, every rank's final checked against
    the closed form inside bench.py (it exits non-zero on a mismatch).  The
    driver's 8-GPU run differs only in the transport (RCCL) and one GPU per rank."""
    import json
    import subprocess
    n = 10_000_000_000
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--rows-total", str(n),
           "--dist-backend", "gloo", "--steps", "3", "--warmup", "1", "--no-cpu-baseline"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "2"
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=280, env=env, cwd=ROOT)
    if os.path.isdir(os.path.join(ROOT, "gpurun_out")):  # evidence for profiles/
        with open(os.path.join(ROOT, "gpurun_out", "world8_rehearsal.log"), "w") as fh:
            fh.write("$ " + " ".join(cmd[1:]) + "\n" + p.stderr + p.stdout)
    assert p.returncode == 0, p.stderr[-3000:]
    assert "launching 8 ranks" in p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    out = json.loads(lines[0])
    if os.path.isdir(os.path.join(ROOT, "gpurun_out")):
        with open(os.path.join(ROOT, "gpurun_out", "world8_rehearsal.json"), "w") as fh:
            fh.write(lines[0] + "\n")
    assert out["n_gpus"] == 8 and out["ranks_seen"] == 8 and out["scaling"] == "strong"
    assert out["config"]["rows_total"] == n and out["config"]["partitions_per_gpu"] == 1
    s = n * (n - 1) // 2 % 2**64
    assert out["result"] == [s // n, n - 1, 0]
    assert "== closed form" in p.stderr
    h = out["host_ms_per_step"]
    # one all-reduce per step, of 8 ranks x (8 B length + 96 B of C3 states)
    assert h["exchange_rounds"] == 1 and h["exchange_bytes"] == 8 * 104
    assert h["exchange"] > 0 and h["partial"] > 0 and h["final"] > 0


_ABSENT_PEER_CHILD = r"""
import ctypes as C, json, sys, time
sys.path.insert(0, %r)
import torch
from fq_amd import abi
from fq_amd._lib import lib
from fq_amd import dist as fqd
uid = C.create_string_buffer(fqd.COMM_ID_BYTES)
assert lib.fq_comm_unique_id(uid) == abi.FQ_OK
h = C.c_void_p()
t0 = time.monotonic()
st = lib.fq_comm_init_timeout(0, 2, 0, uid, 3000, C.byref(h))
print(json.dumps({"status": st, "msg": lib.fq_last_error().decode(), "elapsed": time.monotonic() - t0}), flush=True)
"""


def test_rccl_init_with_a_rank_that_never_arrives_fails_within_the_deadline():
    """RCCL's own path to the deadline (fq_comm.cpp comm_wait): rank 0 of a
    world-2 communicator whose rank 1 never arrives.  The non-blocking init
    polls ncclCommGetAsyncError; after the 3 s deadline the communicator is
    aborted and the call fails with FQ_E_RCCL naming the rank and the step --
    no wait without end.  (Run in a child process with its own time limit: a
    regression here must fail the test, not hang the suite.)"""
    import json
    import subprocess
    code = _ABSENT_PEER_CHILD % os.path.join(ROOT, "fuse-query_amd")
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=90, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    from fq_amd import abi
    assert out["status"] == abi.FQ_E_RCCL, out
    assert out["msg"].startswith("rank 0 of 2: ") and "did not complete within 3000 ms" in out["msg"], out
    assert 2.5 <= out["elapsed"] < 30, out
