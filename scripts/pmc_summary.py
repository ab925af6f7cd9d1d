"""Summarise rocprofv3 --pmc passes (scripts/pmc_profile.sh) into profiles/.

    python scripts/pmc_summary.py gpurun_out/pmc2 --tag c2 --out profiles/r1_pmc_c2

Writes <out>.md (per-kernel average counter value per dispatch) and merges the HBM traffic of
each kernel into profiles/pmc_traffic.json under "<tag>:<kernel>" (what bench.py reports as
roofline.traffic).  HBM bytes per launch follow MI355X_MICROARCH.md "HBM [CDNA4]":
FETCH_SIZE and WRITE_SIZE are KiB from the L2 memory-side request counters; on gfx950
FETCH_SIZE tallies wide streaming reads at half their bytes, so it is doubled; WRITE_SIZE is
exact for wide streaming stores.  The two come from separate passes (they do not fit one).
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import re


def short(name: str) -> str:
    m = re.search(r"sdr::(\w+)(<[^(]*>)?", name)
    return (m.group(1) + (m.group(2) or "").replace(" ", "")) if m else name.split("(")[0]


def load(d: str):
    # (kernel, counter) -> [values per dispatch]
    vals = collections.defaultdict(list)
    meta = {}
    for f in sorted(glob.glob(os.path.join(d, "p*", "*counter_collection.csv"))):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = short(r["Kernel_Name"])
                vals[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
                meta.setdefault(k, {"vgpr": r["VGPR_Count"], "sgpr": r["SGPR_Count"],
                                    "lds": r["LDS_Block_Size"], "grid": r["Grid_Size"],
                                    "wg": r["Workgroup_Size"]})
    return vals, meta


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("--tag", default="c2")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    vals, meta = load(a.pmc_dir)
    kernels = sorted({k for k, _ in vals})
    counters = sorted({c for _, c in vals})
    avg = {(k, c): sum(v) / len(v) for (k, c), v in vals.items()}
    lines = [f"# PMC summary ({a.pmc_dir}, config {a.tag})", "",
             "Average counter value per dispatch. FETCH_SIZE/WRITE_SIZE in KiB (raw, before the "
             "gfx950 x2 FETCH correction); SQ_* cycle counters in quad-cycles.", "",
             "| kernel | vgpr | sgpr | lds B | " + " | ".join(counters) + " |",
             "|---" * (4 + len(counters)) + "|"]
    for k in kernels:
        m = meta[k]
        row = [k, m["vgpr"], m["sgpr"], m["lds"]]
        for c in counters:
            v = avg.get((k, c))
            row.append("" if v is None else f"{v:,.0f}")
        lines.append("| " + " | ".join(row) + " |")
    traffic_path = os.path.join(os.path.dirname(a.out) or ".", "pmc_traffic.json")
    try:
        with open(traffic_path) as fh:
            traffic = json.load(fh)
    except FileNotFoundError:
        traffic = {}
    lines += ["", "HBM bytes per launch = 2 x FETCH_SIZE x 1024 + WRITE_SIZE x 1024:", ""]
    # this tag's entries are replaced as a whole (kernels the pipeline no longer runs drop out);
    # several instances of one kernel (k_sweep's up and down passes) average per launch
    traffic = {key: v for key, v in traffic.items() if not key.startswith(a.tag + ":")}
    per_base = collections.defaultdict(list)
    for k in kernels:
        f, w = avg.get((k, "FETCH_SIZE")), avg.get((k, "WRITE_SIZE"))
        if f is None or w is None:
            continue
        b = int(2 * f * 1024 + w * 1024)
        base = k.split("<")[0]
        if base == "k_sweep16":  # the MODE_HH sweep passes, timed apart by bench.py: up / down
            base = "k_sweep" if k.rstrip(">").endswith("true") else "k_sweep_down"
        per_base[base].append((k, b, int(2 * f * 1024), int(w * 1024)))
        lines.append(f"- {k}: {b / 1e9:.4f} GB (read {2 * f * 1024 / 1e9:.4f}, write {w * 1024 / 1e9:.4f})")
    for base, inst in per_base.items():
        n = len(inst)
        traffic[f"{a.tag}:{base}"] = {"hbm_bytes_per_launch": sum(i[1] for i in inst) // n,
                                      "read_bytes": sum(i[2] for i in inst) // n,
                                      "write_bytes": sum(i[3] for i in inst) // n,
                                      "instance": " + ".join(i[0] for i in inst),
                                      "source": os.path.basename(a.out) + ".md"}
    with open(a.out + ".md", "w") as fh:
        fh.write("\n".join(lines) + "\n")
    with open(traffic_path, "w") as fh:
        json.dump(traffic, fh, indent=1, sort_keys=True)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
