"""Sweep helper: applies FQ_TUNE_<KNOB>=<value> environment variables to the
library's launch-shape knobs through fq_tune_set (abi.TUNE names).  The
library itself reads no environment for them; only the tools do, here."""
import os


def apply_env():
    from fq_amd import abi, ops
    applied = {}
    for name in abi.TUNE:
        v = os.environ.get("FQ_TUNE_" + name)
        if v is not None:
            ops.tune_set(name, int(v))
            applied[name] = int(v)
    return applied
