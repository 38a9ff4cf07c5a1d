"""bench.py's contract on a small C2 shape: one JSON line with the metric, roofline and CPU baseline
fields the driver and the judge read (run as a child process, as the driver runs it)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def test_bench_emits_one_contract_line():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1", "--batch",
           str(1 << 18), "--keys", str(1 << 12), "--cpu-seconds", "0.5", "--no-extra"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    assert len(lines[0]) <= 8192   # the driver parses the line from a bounded stdout tail
    d = json.loads(lines[0])
    assert os.path.exists(os.path.join(ROOT, d["detail"]))
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1 and d["value"] > 0
    assert d["unit"] == "events/s" and d["higher_is_better"] is True and d["scaling"] == "weak"
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and 0 < rf["frac"] < 1
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-9
    assert d["cpu_baseline"]["kind"] == "port" and d["cpu_baseline"]["cores"] == 1
    assert d["cpu_baseline"]["value"] > 0
    # events/s = events of the timed steps over the timed wall time
    assert abs(d["value"] * d["ms_per_step"] / 1e3 - (1 << 18)) / (1 << 18) < 1e-6
