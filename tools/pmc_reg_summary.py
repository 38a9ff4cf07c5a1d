"""Summary of tools/pmc_reg.sh: per register-window kernel the average over dispatches of each PMC counter,
HBM traffic per dispatch (FETCH_SIZE x 2 on gfx950 + WRITE_SIZE, MI355X_MICROARCH.md) and per input event of
the batch (4,194,304 events per dispatch at the bench size), and the kernel-trace averages.
    python tools/pmc_reg_summary.py [dir]"""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                         "gpurun_out", "pmc_reg")
EV = 4194304
for cfg in ("C4", "C3_min1"):
    vals = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, f"{cfg}_g*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            vals[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    print(f"== {cfg}")
    kernels = sorted({k for k, _ in vals})
    for k in kernels:
        c = {n: sum(v) / len(v) for (kk, n), v in vals.items() if kk == k}
        nd = max(len(v) for (kk, n), v in vals.items() if kk == k)
        line = f"  {k} ({nd} dispatches): " + ", ".join(f"{n}={v:.4g}" for n, v in sorted(c.items()))
        print(line)
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            hbm = 2 * 1024 * c["FETCH_SIZE"] + 1024 * c["WRITE_SIZE"]
            print(f"    HBM bytes per dispatch {hbm:.4g} (fetch x2 {2048 * c['FETCH_SIZE']:.4g} + write "
                  f"{1024 * c['WRITE_SIZE']:.4g}); per batch event {hbm / EV:.1f} B")
    st = os.path.join(d, f"{cfg}_trace", "run_kernel_stats.csv")
    if os.path.exists(st):
        rows = list(csv.DictReader(open(st)))
        for r in rows[:8]:
            print(f"  trace {r['Name'][:70]:70s} calls {r['Calls']:>4s} avg {float(r['AverageNs']) / 1e3:9.1f} us "
                  f"{r['Percentage']}%")
