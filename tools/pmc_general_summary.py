"""Summary of tools/pmc_general.sh: per config the NFA kernels that ran (from the kernel trace), per kernel the
average of each PMC counter over its dispatches, HBM traffic (FETCH_SIZE x 2 on gfx950 + WRITE_SIZE,
MI355X_MICROARCH.md) per dispatch, and per config the NFA kernels' traffic per pushed batch (every dispatch's
bytes / the pushes) and per input event.  Writes <dir>/summary.txt and, with --json, the per-config traffic
that bench.py reports as `other_configs.*.roofline.traffic` (tools/pmc_traffic_general.json, tagged with the
hash of the kernel sources it was measured on).
    python tools/pmc_general_summary.py gpurun_out/pmc_gen [--json tools/pmc_traffic_general.json --profiles p]"""
import argparse
import csv
import glob
import hashlib
import json
import os
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the sources the general configs' NFA kernels are built from (bench.py checks the same hash)
SOURCES = ["abs_kernels.hip", "absd_kernels.hip", "cnt_kernels.hip", "chn_kernels.hip", "gen_kernels.hip",
           "gen_host.hip", "reg_common.h", "gen_engine.h", "java_ops.h", "pack.h"]
# the configs' pushed batch size (bench.py other_configs)
EVENTS = {"C3": 1 << 22, "C3_min1": 1 << 22, "C3_and": 1 << 22, "P3": 1 << 22, "C4": 1 << 22, "C4_deep": 1 << 22, "C4_deep_state": 1 << 16}
BATCH_KERNELS = ("k_cnt_batch", "k_abs_batch", "k_chn_batch", "k_gen_batch")
# --variants: the C2 workload variants (tools/pmc_variants.sh): the two-state engine's advance kernels, all in the
# query-specialised p2_jit.hip (staged pass, HBM passes, hot-key pipeline)
VAR_SOURCES = ["p2_jit.hip"]
VAR_EVENTS = {"C2_zipf": 1 << 24, "C2_walk": 1 << 24}
VAR_BATCH_KERNELS = ("k_adv_m",)


def sources_hash(sources):
    h = hashlib.sha1()
    for f in sources:
        h.update(open(os.path.join(ROOT, "siddhi-1_amd", "csrc", f), "rb").read())
    return h.hexdigest()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--json")
    ap.add_argument("--profiles", default=None)
    ap.add_argument("--variants", action="store_true")
    args = ap.parse_args()
    global EVENTS, BATCH_KERNELS
    sources = SOURCES
    if args.variants:
        EVENTS, BATCH_KERNELS, sources = VAR_EVENTS, VAR_BATCH_KERNELS, VAR_SOURCES
    lines, out = [], {}
    for cfg in EVENTS:
        files = sorted(glob.glob(os.path.join(args.dir, f"{cfg}_g*", "run_counter_collection.csv")))
        if not files:
            continue
        vals = defaultdict(list)
        for f in files:
            for r in csv.DictReader(open(f)):
                vals[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
        calls = {}
        st = os.path.join(args.dir, f"{cfg}_trace", "run_kernel_stats.csv")
        trace = list(csv.DictReader(open(st))) if os.path.exists(st) else []
        for r in trace:
            calls[r["Name"]] = (int(r["Calls"]), float(r["AverageNs"]))
        pushes = max((c for n, (c, _) in calls.items() if n.startswith(BATCH_KERNELS)), default=0)
        lines.append(f"== {cfg}: {pushes} pushed batches of {EVENTS[cfg]} events (trace)")
        total, kern = 0.0, {}
        for k in sorted({k for k, _ in vals}):
            c = {n: sum(v) / len(v) for (kk, n), v in vals.items() if kk == k}
            nd = calls.get(k, (max(len(v) for (kk, n), v in vals.items() if kk == k), 0.0))[0]
            lines.append(f"  {k} ({nd} dispatches, avg {calls.get(k, (0, 0.0))[1] / 1e3:.1f} us): " +
                         ", ".join(f"{n}={v:.4g}" for n, v in sorted(c.items())))
            if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
                hbm = 2 * 1024 * c["FETCH_SIZE"] + 1024 * c["WRITE_SIZE"]
                lines.append(f"    HBM bytes per dispatch {hbm:.4g} (fetch x2 {2048 * c['FETCH_SIZE']:.4g} + write "
                             f"{1024 * c['WRITE_SIZE']:.4g})")
                total += hbm * nd
                kern[k] = {"dispatches": nd, "avg_us": calls.get(k, (0, 0.0))[1] / 1e3,
                           "hbm_bytes_per_dispatch": hbm,
                           "valu": c.get("SQ_INSTS_VALU"), "salu": c.get("SQ_INSTS_SALU"),
                           "wait_frac": (c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]) if c.get("SQ_WAVE_CYCLES") else None}
        if pushes:
            per = total / pushes
            lines.append(f"  NFA kernels: {per:.4g} B per pushed batch = {per / EVENTS[cfg]:.1f} B per input event")
            out[cfg] = {"traffic_bytes_per_step": per, "traffic_bytes_per_event": per / EVENTS[cfg],
                        "kernels": kern, "pushes": pushes}
        for r in trace[:10]:
            lines.append(f"  trace {r['Name'][:72]:72s} calls {r['Calls']:>4s} avg {float(r['AverageNs']) / 1e3:9.1f} us "
                         f"{r['Percentage']}%")
    text = "\n".join(lines)
    print(text)
    open(os.path.join(args.dir, "summary.txt"), "w").write(text + "\n")
    if args.json:
        json.dump({"configs": out, "kernel_src_sha1": sources_hash(sources), "sources": sources,
                   "profiles": args.profiles or args.dir,
                   "method": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950) and WRITE_SIZE in separate passes over " +
                             ("tools/exp_variants.py, tools/pmc_variants.sh" if args.variants else
                              "tools/exp_gen.py <cfg>, tools/pmc_general.sh") + "; bytes of every NFA-kernel dispatch "
                             "/ pushed batches"}, open(args.json, "w"), indent=1)


if __name__ == "__main__":
    main()
