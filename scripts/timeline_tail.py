"""Print the tail of a rocprofv3 kernel + memory-copy trace as one timeline.

    python scripts/timeline_tail.py OUT_DIR [N]

OUT_DIR holds rocprofv3 --kernel-trace --memory-copy-trace --output-format csv
output; writes OUT_DIR/finish_timeline.txt: the last N events (default 60)
with start / end relative to the first of them (us), duration, and the kernel
name or copy direction and size.  Used for the streaming finish's timeline
(scripts/stream_probe.py) and the device round's (segwin_layout_probe.py).
"""
import csv
import glob
import sys

O = sys.argv[1]
N = int(sys.argv[2]) if len(sys.argv) > 2 else 60
ev = []
for f in glob.glob(f"{O}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + r["Kernel_Name"][:50]))
for f in glob.glob(f"{O}/**/*memory_copy_trace.csv", recursive=True):
    rows = list(csv.DictReader(open(f)))
    if rows:
        print("copy columns:", list(rows[0].keys()))
    for r in rows:
        what = " ".join(str(r.get(k, "")) for k in ("Direction", "Operation", "Kind") if r.get(k))
        sz = r.get("Size") or r.get("Bytes") or r.get("Copy_Bytes") or ""
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), f"C {what} {sz}"))
ev.sort()
tail = ev[-N:]
t0 = tail[0][0]
with open(f"{O}/finish_timeline.txt", "w") as out:
    for s, e, n in tail:
        out.write(f"{(s - t0) / 1e3:10.2f} {(e - t0) / 1e3:10.2f} {(e - s) / 1e3:8.2f}  {n}\n")
print(open(f"{O}/finish_timeline.txt").read())
