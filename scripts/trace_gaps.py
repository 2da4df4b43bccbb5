#!/usr/bin/env python
"""Idle time between kernels in a rocprofv3 kernel trace (last K analysis kernels)."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
ana = [r for r in rows if "analysis" in r["Kernel_Name"] and "_kernel" in r["Kernel_Name"]][-K:]
t0, t1 = int(ana[0]["Start_Timestamp"]), int(ana[-1]["End_Timestamp"])
sel = [r for r in rows if t0 <= int(r["Start_Timestamp"]) <= t1]
busy_end, idle = t0, 0
for r in sel:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    idle += max(0, s - busy_end)
    busy_end = max(busy_end, e)
ak = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in ana)
print(f"{K} analysis kernels: span {(t1 - t0) / 1e3:.1f} us, analysis {ak / 1e3:.1f} us, "
      f"idle {idle / 1e3:.1f} us ({idle / (t1 - t0):.1%})")
