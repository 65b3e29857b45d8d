"""Print calls / average microseconds of the kernels in rocprofv3 kernel_stats
CSVs whose names contain any of the given substrings.
Usage: python tools/kstats.py LABEL CSV [SUBSTR ...]"""
import csv
import sys

label, path = sys.argv[1], sys.argv[2]
subs = sys.argv[3:] or ["k_"]
for r in csv.DictReader(open(path)):
    n = r["Name"]
    if any(s in n for s in subs):
        short = n.split("(")[0].replace("void ", "").replace("cwq::", "")
        print(f"{label:10s} {short:36s} calls {int(r['Calls']):5d} avg_us "
              f"{float(r['AverageNs']) / 1e3:9.2f} total_us {float(r['TotalDurationNs']) / 1e3:10.1f}")
