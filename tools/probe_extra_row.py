import os, sys, json
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, os.path.join(ROOT, "fuse-query_amd"))
import numpy as np
from fq_amd import ops
from fq_amd.engine import Engine
ops.require_gpu()
SQL = "SELECT number FROM system.numbers_mt(4000000000) WHERE number % 1000000007 = 3"
for trial in range(2):
    e = Engine(streams=2)
    e.trim_memory()
    n = 8_000_000_000
    r = e.execute("SELECT number%%100000, count(number) FROM system.numbers_mt(%d) GROUP BY number%%100000" % n)
    print("groupby rows", len(r.rows), flush=True)
    for q in range(3):
        out = []
        with e.execute_blocks(SQL) as st:
            for b in st:
                if b.rows:
                    cols = ops.device_block_to_numpy(b)
                    vals = [int(v) for blk in cols[0] for v in blk] if b.block_rows > 0 else [int(v) for v in cols[0]]
                    out.append((b.pipe, b.block_rows, b.n_blocks, b.rows, vals[:8]))
        print("trial", trial, "query", q, json.dumps(out), flush=True)
        r = e.execute(SQL)
        print("   execute rows", sorted(v for (v,) in r.rows), flush=True)
    e.close()
