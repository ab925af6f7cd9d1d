"""Print a rocprofv3 --stats kernel summary (CSV) compactly: python scripts/kstats.py <dir>"""
import csv
import glob
import re
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = re.sub(r"\(.*", "", r["Name"]).replace("void ", "")[:48]
    print(f"{n:48s} calls={r['Calls']:>6} avg_us={float(r['AverageNs']) / 1e3:9.2f} "
          f"pct={float(r['Percentage']):6.2f}")
