"""Summarise a rocprofv3 --kernel-trace database (rocpd sqlite): mean duration per (kernel, grid, LDS) in dispatch order.

usage: python tools/rocpd_summary.py <results.db> [name-filter]
"""
import collections
import re
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
flt = sys.argv[2] if len(sys.argv) > 2 else ""
rows = db.execute("select name, start, end, grid_x, lds_size, scratch_size from kernels order by start").fetchall()
agg = collections.OrderedDict()
for name, s, e, grid, lds, scr in rows:
    n = re.sub(r"\(.*", "", name)
    n = re.sub(r".*anonymous namespace\)::", "", n)
    if flt and not re.search(flt, n):
        continue
    agg.setdefault((n[:90], grid, lds, scr), []).append((e - s) / 1e3)
for (n, grid, lds, scr), v in agg.items():
    print("%6d x %9.1f us (min %8.1f)  grid=%-9d lds=%-6d scratch=%-5d %s" % (len(v), sum(v) / len(v), min(v), grid, lds, scr, n))
