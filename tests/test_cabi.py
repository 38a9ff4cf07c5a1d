"""The C-ABI libraries load and export every entry point include/siddhi_gpu.h declares (no GPU needed)."""
import ctypes
import importlib
import os
import re

from oracle_backend import ROOT, build_oracle

sa = importlib.import_module("siddhi-1_amd")


def declared():
    src = open(os.path.join(ROOT, "include", "siddhi_gpu.h")).read()
    return sorted(set(re.findall(r"\b(sg_[a-z_]+)\s*\(", src)))


def test_header_declares_the_boundary():
    names = declared()
    for n in ("sg_engine_create", "sg_push_batch", "sg_advance_time", "sg_poll_matches",
              "sg_release_matches", "sg_snapshot", "sg_restore", "sg_reset_keys", "sg_engine_destroy",
              "sg_last_error"):
        assert n in names


def test_hip_library_exports_every_symbol():
    lib = sa.load_hip_library()
    for n in declared():
        assert hasattr(lib, n), n
    lib.sg_abi_version.restype = ctypes.c_int
    assert lib.sg_abi_version() == 1


def test_oracle_exports_the_same_entry_points():
    lib = build_oracle()
    for n in ("engine_create", "push_batch", "poll_matches", "release_matches", "get_stats",
              "engine_destroy", "last_error", "advance_time", "reset_keys"):
        assert hasattr(lib, "sgo_" + n), n


def test_engine_create_rejects_garbage_ir():
    lib = build_oracle()
    try:
        sa.NativeEngine(lib, "sgo_", b"\x00" * 64)
    except sa.EngineError as ex:
        assert "magic" in str(ex) or "IR" in str(ex)
    else:
        raise AssertionError("garbage IR accepted")


def test_no_result_changing_knobs_in_the_shipped_library():
    """the ablation knobs that produce wrong results (ordering / grouping ablations, JIT-time defines) are
    compiled only into EXTRA=-DSG_EXPERIMENTS builds: the shipped library does not read them"""
    path = os.path.join(ROOT, "siddhi-1_amd", "lib", "libsiddhi_gpu.so")
    blob = open(path, "rb").read()
    for name in (b"SG_ORDER_EXP", b"SG_GRP_EXP", b"SG_JIT_EXTRA"):
        assert name not in blob, name
