"""Summarise the PMC passes of tools/pmc_c2.sh (gpurun_out/pmc) for the advance kernel.

Writes tools/pmc_traffic.json (read by bench.py for roofline.traffic) and copies the counter CSVs to
profiles/<tag>_pmc/.  HBM bytes per launch follow MI355X_MICROARCH.md's HBM/rocprofv3 section:
FETCH_SIZE (KB) counts half the bytes of wide coalesced reads on gfx950 (x2), WRITE_SIZE (KB) is
exact for 16-B-per-lane stores; separate passes.  The first dispatch (cold state) is excluded.

    python tools/pmc_summary.py <tag>
"""
import csv
import hashlib
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PMC = os.path.join(ROOT, "gpurun_out", "pmc")


def counter(name):
    for g in sorted(os.listdir(PMC)):
        f = os.path.join(PMC, g, "run_counter_collection.csv")
        if not os.path.isfile(f):
            continue
        vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f))
                if r["Counter_Name"] == name and r["Kernel_Name"] == "k_adv_m"]
        if vals:
            return vals[1:] if len(vals) > 1 else vals
    return None


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    fetch, write = counter("FETCH_SIZE"), counter("WRITE_SIZE")
    if not fetch or not write:
        sys.exit("FETCH_SIZE / WRITE_SIZE passes missing under gpurun_out/pmc")
    fb = 2.0 * 1024.0 * sum(fetch) / len(fetch)
    wb = 1024.0 * sum(write) / len(write)
    src = open(os.path.join(ROOT, "siddhi-1_amd", "csrc", "p2_jit.hip"), "rb").read()
    out = {"kernel": "k_adv_m", "workload": "C2 (2^20 keys, 2^24-event batches)",
           "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb, "traffic_bytes_per_launch": fb + wb,
           "kernel_src_sha1": hashlib.sha1(src).hexdigest(), "profiles": f"profiles/{tag}_pmc",
           "method": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950) and WRITE_SIZE in separate passes, tools/pmc_c2.sh"}
    json.dump(out, open(os.path.join(ROOT, "tools", "pmc_traffic.json"), "w"), indent=1)
    dst = os.path.join(ROOT, "profiles", f"{tag}_pmc")
    os.makedirs(dst, exist_ok=True)
    for g in sorted(os.listdir(PMC)):
        f = os.path.join(PMC, g, "run_counter_collection.csv")
        if os.path.isfile(f):
            shutil.copy(f, os.path.join(dst, f"c2_adv_{g}.csv"))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
