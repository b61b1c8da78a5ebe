"""Print the kernel timeline of the last N frames from a rocprofv3 kernel_trace.csv (dev tool).

A frame starts at a k_generate dispatch.  Columns: start offset from the
frame's first kernel (us), duration (us), gap since the previous kernel on the
same queue ended (us), queue, kernel.
usage: python tools/timeline.py <run_kernel_trace.csv> [frames=1]
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
nf = int(sys.argv[2]) if len(sys.argv) > 2 else 1
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
gens = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("k_generate")]
if not gens:
    sys.exit("no k_generate dispatch")
first = gens[-nf] if len(gens) >= nf else gens[0]
# include the prep/memset kernels just before the frame's first generate on other queues
sel = rows[first:]
t0 = int(sel[0]["Start_Timestamp"])
last_end = {}
busy = 0
for r in sel:
    s, e, q = int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"]
    gap = (s - last_end[q]) / 1e3 if q in last_end else float("nan")
    last_end[q] = e
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    print(f"{(s - t0) / 1e3:10.1f} {(e - s) / 1e3:9.1f} {gap:8.1f} q{q:>2} {name}")
end = max(int(r["End_Timestamp"]) for r in sel)
print(f"span {(end - t0) / 1e3:.1f} us over {len(sel)} kernels")
