"""Runs of copy events in a rocprofv3 trace (blit kernels vs DMA copies), for
scripts/d2h_engine_probe.py: python scripts/copy_engine_runs.py OUT_DIR."""
import csv, glob, sys
O = sys.argv[1]
ev = []
for f in glob.glob(f"{O}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "copyBuffer" in r["Kernel_Name"] or "fillBuffer" in r["Kernel_Name"]:
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "blit"))
for f in glob.glob(f"{O}/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "dma:" + r["Direction"].replace("MEMORY_COPY_", "")))
ev.sort()
runs = []
for s, e, n in ev:
    d = (e - s) / 1e3
    if runs and runs[-1][0] == n:
        runs[-1][1] += 1; runs[-1][2].append(d)
    else:
        runs.append([n, 1, [d]])
for n, c, ds in runs[-20:]:
    ds.sort()
    print(f"{n:28s} x{c:3d}  median {ds[len(ds)//2]:9.2f} us")
