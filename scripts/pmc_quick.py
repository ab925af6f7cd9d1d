"""Average rocprofv3 --pmc counter values per dispatch, per kernel and grid size:
python scripts/pmc_quick.py <dir>"""
import collections
import csv
import glob
import re
import sys

vals = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")[:36] + " g" + r.get("Grid_Size", "?")
        vals[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(vals.items()):
    print(f"{k:48s} {c:22s} n={len(v):4d} avg={sum(v) / len(v):14.1f}")
