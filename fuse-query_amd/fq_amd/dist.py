"""Multi-GPU AggregateFinal: one process per GPU, numbers_mt partitions
sharded [8r/G, 8(r+1)/G), and the partial states exchanged with a
SINGLE all-reduce -- RCCL over xGMI on GPUs (torch.distributed backend
"nccl"), gloo on CPU.

The reference's only "exchange" is the in-process MergeProcessor channel of
JSON states (processor_merge.rs:45-63, transform_aggregate_partial.rs:61-72).
Here every rank serialises its merged partial states (fixed 16-byte
DataValue records, a few hundred bytes), writes them into ITS OWN row of a
zeroed [world, cap/8] int64 buffer, and one all-reduce(SUM) turns that into an
all-gather: each element has exactly one non-zero contributor, so the sum is
bit-exact for any payload.  The merge itself then runs in rank order on every
rank (AggregateFinalTransform), so all ranks agree on the result.
"""
import torch
import torch.distributed as dist

STATE_CAP = 4096  # bytes per rank; a query's states are 8 + 16 per value + 8 per function


def allgather_states(states, group=None, device=None, cap=STATE_CAP):
    """bytes of this rank -> [bytes of rank 0, ..., rank world-1] (one all-reduce;
    payloads above `cap` -- GROUP BY states grow with the number of groups --
    first agree on the largest length with a second, 8-byte-per-rank one)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if device is None:
        device = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
    if len(states) > cap or cap != STATE_CAP:
        lens = torch.zeros(world, dtype=torch.int64, device=device)
        lens[rank] = len(states)
        dist.all_reduce(lens, op=dist.ReduceOp.SUM, group=group)
        cap = max(cap, (int(lens.max().item()) + 7) // 8 * 8)
    buf = torch.zeros((world, cap // 8), dtype=torch.int64, device=device)
    row = torch.frombuffer(bytearray(states.ljust(cap, b"\0")), dtype=torch.int64)
    buf[rank].copy_(row)
    dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
    host = buf.cpu().numpy()
    return [host[r].tobytes() for r in range(world)]


def execute(engine, sql, group=None):
    """Run an aggregate query across all ranks of `group`: local partial on this
    rank's shard -> one all-reduce -> AggregateFinal merge in rank order."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    local = engine.execute_partial(sql, rank, world)
    everyone = allgather_states(local, group)
    return engine.execute_final(sql, everyone)
