"""The drop-in boundary from a plain C host (tests/native/fq_c_client.c,
built by `make -C fuse-query_amd` into lib/fq_c_client): kernel ABI
(fq_fill_numbers_u64 + fq_aggregate), error text, and the engine ABI (C3
statement through fq_engine_execute) without Python or torch in the process."""
import os
import subprocess

import pytest

BIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fuse-query_amd", "lib", "fq_c_client")


def run(*args):
    return subprocess.run([BIN, *map(str, args)], capture_output=True, text=True, timeout=120)


def test_c_client_binary_is_built():
    assert os.access(BIN, os.X_OK), "build with make -C fuse-query_amd"


@pytest.mark.gpu
# totals whose numbers_mt partitions keep every row (numbers_stream.rs:44-46
# drops rows when a partition is >= 10,000 rows and not a multiple of them)
@pytest.mark.parametrize("n,total", [(100_000_003, 1_000_000_000), (1, 8), (4097, 800_000)])
def test_c_client_on_gpu(n, total):
    p = run(n, total)
    assert p.returncode == 0, p.stderr
    lines = p.stdout.splitlines()
    prefixes = ["OK abi version", "OK kernel abi", "OK error text", "OK engine abi", "OK engine error"]
    assert len(lines) == len(prefixes) and all(l.startswith(x) for l, x in zip(lines, prefixes)), lines
    assert "Unsupported Function: foo" in lines[-1]


def test_c_client_fails_loudly_without_gpu():
    # no device here: the first HIP-backed call reports an error, exit status 1
    if os.path.exists("/dev/kfd"):
        pytest.skip("a GPU is visible")
    p = run()
    assert p.returncode == 1 and "FAIL" in p.stderr
