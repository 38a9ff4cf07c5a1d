"""bench.py's compact contract line (no GPU): every headline field kept, other legs summarised, <= 8 KB even
with many legs, the headline never dropped."""
import importlib.util
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _full(n_legs):
    rf = {"bound": "hbm", "achieved": 1234.5678, "peak": 8000.0, "unit": "GB/s", "frac": 1234.5678 / 8000.0,
          "traffic": 6.9e8, "kernel": "k_adv_m", "alg_bytes_per_launch": 8.1e8, "kernel_ms_per_launch": 0.6,
          "note": "x" * 500, "isolated": {"kernel_ms_per_launch": 0.5, "achieved": 1600.0, "frac": 0.2}}
    leg = {"value": 1e10, "unit": "events/s", "ms_per_step": 0.4, "kernels": ["k"] * 50, "workload": "w" * 300,
           "roofline": {"frac": 0.1, "traffic": 3e8, "alg_bytes_per_step": 1e8, "kernel": "k" * 200},
           "cpu_baseline": {"value": 1e6, "sample": "s" * 400}}
    return {"metric": "m", "value": 1.6e10, "unit": "events/s", "n_gpus": 1, "steps": 64, "warmup": 3,
            "ms_per_step": 1.0, "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic", "config": {"workload": "C2", "keys_per_gpu": 1 << 20, "batch_events_per_gpu": 1 << 24,
                                            "events_per_ms": 2000, "parallelism": "key-sharded x1"},
            "roofline": rf, "stages_ms_per_step": {"group": 0.3, "advance": 0.6, "order": 0.2},
            "stages_ms_isolated": {"group": 0.3, "advance": 0.5, "order": 0.2},
            "cpu_baseline": {"value": 4.7e5, "unit": "events/s", "cores": 1, "kind": "port",
                             "sample": "first 5767168 events of the C2 stream (1048576 keys), CPU oracle (...)",
                             "partition_parallel": {"value": 6.4e6, "threads": 16, "pinned_cpus": list(range(16))}},
            "other_configs": {f"L{i}": dict(leg) for i in range(n_legs)},
            "fanout_one_gpu": {"value": 1e9, "ms_per_step": 4.0, "ratio_to_single": 0.6, "host_syncs_per_push": 0.0}}


def test_compact_line_fields_and_size():
    b = _bench()
    s = b.compact_line(_full(12), "profiles/d.json")
    assert len(s) <= b.LINE_MAX
    d = json.loads(s)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "detail"):
        assert k in d, k
    assert d["value"] == 1.6e10 and d["detail"] == "profiles/d.json"
    rf = d["roofline"]
    assert rf["traffic"] == 6.9e8 and abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-12
    assert d["cpu_baseline"]["cores"] == 1 and d["cpu_baseline"]["partition_parallel"]["threads"] == 16
    assert d["extra"]["L0"] == {"value": 1e10, "ms_per_step": 0.4, "frac": 0.1, "traffic_ratio": 3.0, "cpu": 1e6}
    assert d["extra"]["fanout_one_gpu"]["ratio_to_single"] == 0.6


def test_compact_line_drops_summaries_before_the_headline():
    b = _bench()
    s = b.compact_line(_full(400), None)
    assert len(s) <= b.LINE_MAX
    d = json.loads(s)
    assert "extra" not in d and d["value"] == 1.6e10 and "roofline" in d
