"""Test-only helpers: run the host API over the CPU oracle (oracle/build/libsgoracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use the oracle.
"""
import importlib
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_LIB = os.path.join(ROOT, "oracle", "build", "libsgoracle.so")

sa = importlib.import_module("siddhi-1_amd")


def build_oracle():
    if not os.path.exists(ORACLE_LIB) or \
            os.path.getmtime(ORACLE_LIB) < os.path.getmtime(os.path.join(ROOT, "oracle", "sg_oracle.cpp")):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    return sa.load_library(ORACLE_LIB)


def oracle_factory(**kw):
    lib = build_oracle()

    def make(ir, n_keys):
        return sa.NativeEngine(lib, "sgo_", ir, n_keys=n_keys, **kw)
    return make


def oracle_manager(**kw):
    return sa.SiddhiManager(engine_factory=oracle_factory(**kw))
