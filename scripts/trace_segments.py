"""Per-kernel durations from a rocprofv3 --kernel-trace CSV, split into bench.py's segments.

    python scripts/trace_segments.py gpurun_out/<tag>/prof --iso 30 --out profiles/r1_segments_c2.md

bench.py runs its timed region with several frames in flight, then `--iso-steps` single-stream
steps whose HIP-event times give `roofline`.  This prints, per kernel, the average duration of
the last `--iso` dispatches (that single-stream segment, to compare with roofline.avg_launch_us)
and of all earlier dispatches (warmup + timed region, kernels overlapping across streams).
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import os
import re


def short(name: str) -> str:
    m = re.search(r"sdr::(\w+)(<[^(]*>)?", name)
    return (m.group(1) + (m.group(2) or "").replace(" ", "")) if m else name.split("(")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("--iso", type=int, default=30)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    f = glob.glob(os.path.join(a.prof_dir, "*kernel_trace.csv"))[0]
    per = collections.defaultdict(list)
    with open(f) as fh:
        for r in csv.DictReader(fh):
            per[short(r["Kernel_Name"])].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    lines = [f"# rocprofv3 kernel trace split into bench.py segments ({os.path.basename(f)})", "",
             f"Single-stream segment = the last {a.iso} dispatches of each kernel (bench.py --iso-steps); "
             "in flight = every earlier dispatch (warmup + timed region, streams overlapping).", "",
             "| kernel | dispatches | single-stream avg us | in-flight avg us |", "|---|---|---|---|"]
    for k, v in sorted(per.items(), key=lambda kv: -sum(e - s for s, e in kv[1])):
        v.sort()
        d = [(e - s) / 1e3 for s, e in v]
        iso = d[-a.iso:] if len(d) >= a.iso else d
        rest = d[:-a.iso] if len(d) > a.iso else []
        lines.append(f"| {k} | {len(d)} | {sum(iso) / len(iso):.1f} | "
                     f"{(sum(rest) / len(rest)) if rest else float('nan'):.1f} |")
    with open(a.out, "w") as fh:
        fh.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
