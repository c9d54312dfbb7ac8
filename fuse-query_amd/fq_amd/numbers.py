"""system.numbers_mt partitioning (host logic of the device SourceTransform).

NumbersTable::generate_parts (src/datasources/system/numbers_table.rs:29-55)
cuts N into 8 named ranges "N-start-end" (1 range when N < 8; the last one
takes the remainder).  NumbersStream::create (numbers_stream.rs:27-62) cuts a
range into 10,000-row blocks and, when count % 10000 != 0 and count >= 10000,
ends the LAST block at block_begin + remain -- so a partition yields one
contiguous run [begin, begin + rows) with rows = 10000*(k-1) + remain + 1
(SURVEY.md finding 8).  The device Source materialises exactly that run; the
scan kernels replay the 10,000-row block boundaries (block_rows).
"""
BLOCK_SIZE = 10000  # numbers_stream.rs:29
WORKERS = 8  # numbers_table.rs:30


def generate_parts(total):
    """[(name, begin, end_inclusive)] exactly as generate_parts names them."""
    if total <= 0:
        raise ValueError("numbers_mt(0) is not supported (the reference computes total-1 "
                         "in u64 and materialises 2^64 rows)")
    chunk = total // WORKERS
    if chunk == 0:
        return [("%d-%d-%d" % (total, 0, total - 1), 0, total - 1)]
    remain = total % WORKERS
    parts = []
    for p in range(WORKERS):
        start = p * chunk
        end = (p + 1) * chunk - 1
        if p == WORKERS - 1 and remain > 0:
            end += remain
        parts.append(("%d-%d-%d" % (total, start, end), start, end))
    return parts


def stream_rows(begin, end):
    """Rows NumbersStream yields for partition [begin, end] (contiguous from begin)."""
    count = end - begin + 1
    nblocks, remain = divmod(count, BLOCK_SIZE)
    if nblocks == 0:
        return count
    if remain == 0:
        return count
    return BLOCK_SIZE * (nblocks - 1) + remain + 1


def stream_blocks(begin, end):
    """Number of DataBlocks NumbersStream yields for the partition."""
    nblocks = (end - begin + 1) // BLOCK_SIZE
    return nblocks if nblocks > 0 else 1


def shard(parts, rank, world):
    """Partitions owned by `rank` of `world` GPUs: [8r/G, 8(r+1)/G).
    With fewer partitions than ranks, the extra ranks own none."""
    n = len(parts)
    lo = (n * rank) // world
    hi = (n * (rank + 1)) // world
    return parts[lo:hi]
