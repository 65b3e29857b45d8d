"""Device timeline of the last few ms of a rocprofv3 run (kernel and memory
copy traces): every dispatch / copy after the last T0 marker window, relative
to the first event of that window.  Usage:
  python tools/timeline.py DIR [window_ms]   (DIR holds *kernel_trace.csv and
  optionally *memory_copy_trace.csv)"""
import csv
import glob
import sys

d = sys.argv[1]
win = float(sys.argv[2]) if len(sys.argv) > 2 else 8.0
ev = []
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + r["Kernel_Name"][:70]))
for f in glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                   "C " + r.get("Direction", "?") + " " + r.get("Size", "")))
ev.sort()
end = max(e[1] for e in ev)
sel = [e for e in ev if e[0] >= end - win * 1e6]
t0 = sel[0][0]
for s, e, n in sel:
    print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {n}")
# device-busy fraction of the window: the union of the dispatch intervals
busy, cur_s, cur_e = 0, None, None
for s, e, n in sel:
    if not n.startswith("K"):
        continue
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
if cur_e is not None:
    busy += cur_e - cur_s
span = sel[-1][1] - t0
print(f"# window {span / 1e3:.1f} us, kernels busy {busy / 1e3:.1f} us = {busy / span:.1%}")
