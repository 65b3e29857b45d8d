"""Averages a c3_batch_laps.py stderr log into a timeline: each library lap's
monotonic time relative to the Python call's start, then the Python exit.

  python tools/laps_timeline.py laps.err"""
import collections
import re
import sys

acc = collections.defaultdict(list)
start = None
for ln in open(sys.argv[1]):
    m = re.match(r"\[py\] (start|end) monotonic ([\d.]+)", ln)
    if m:
        if m.group(1) == "start":
            start = float(m.group(2))
        elif start is not None:
            acc["py end"].append(float(m.group(2)) - start)
        continue
    m = re.match(r"\[(cwq[^\]]*)\] (.+?)\s+(?:chunk\s+(\d+)\s+)?at\s+[\d.]+ us \(monotonic ([\d.]+) us\)",
                 ln)
    if m and start is not None:
        key = f"{m.group(1)} {m.group(2).strip()}" + (f" c{m.group(3)}" if m.group(3) else "")
        acc[key].append(float(m.group(4)) - start)
rows = sorted(((sum(v) / len(v), k, len(v)) for k, v in acc.items()))
for t, k, n in rows:
    print(f"{t:9.1f} us  {k}  (n={n})")
