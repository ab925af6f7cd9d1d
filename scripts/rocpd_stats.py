"""Kernel stats (rocprofv3 --stats CSV columns) from a rocprofv3 rocpd SQLite database, for runs made
without --output-format csv:  python scripts/rocpd_stats.py <results.db> [out.csv]"""
import collections
import csv
import sqlite3
import shutil
import statistics
import subprocess
import sys


def demangle(names):
    tool = shutil.which("c++filt") or shutil.which("llvm-cxxfilt")
    if not tool:
        return names
    out = subprocess.run([tool], input="\n".join(names), capture_output=True, text=True).stdout.splitlines()
    return out if len(out) == len(names) else names


con = sqlite3.connect(sys.argv[1])
rows = con.execute("select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d "
                   "join rocpd_info_kernel_symbol s on d.kernel_id = s.id").fetchall()
agg = collections.defaultdict(list)
for name, a, b in rows:
    agg[name.removesuffix(".kd")].append(b - a)
total = sum(sum(v) for v in agg.values())
out = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
w = csv.writer(out, quoting=csv.QUOTE_NONNUMERIC)
w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
items = sorted(agg.items(), key=lambda kv: -sum(kv[1]))
for name, (_, v) in zip(demangle([k for k, _ in items]), items):
    w.writerow([name, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / total, min(v), max(v),
                statistics.pstdev(v)])
