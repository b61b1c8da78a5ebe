"""Instruction mix per wave iteration of k_extend, per bounce (dev tool, here).

Reads a tools/profile.sh output dir with the `mix` (and optionally `mix2`) PMC
passes of a bench run whose k_extend launches all carry the same fused frames
(profile.sh: STEPS passes, as many warmup passes, no sync/gui/isolated steps),
and the bench line of that run (for the exact wave iterations per bounce of the
instrumented pass).  A chunk's uninstrumented launches come in bounce order
(bounce 0: the camera instance, 1: the 64-B loop, 2..: the two-level loop), so
the k-th k_extend<false,...> dispatch of a chunk is bounce k.  Prints a markdown
table: per bounce, instructions of each kind per wave iteration, and the
counters' raw per-launch means.
usage: python tools/mix_per_bounce.py <profile dir> <frames per launch> [depth=5] > profiles/<tag>_mix.md
"""
import collections
import csv
import json
import os
import sys

src, fpl = sys.argv[1], float(sys.argv[2])
depth = int(sys.argv[3]) if len(sys.argv) > 3 else 5
bench = None
for name in ("mix_bench.json", "trace_bench.json"):
    p = os.path.join(src, name)
    if os.path.exists(p):
        txt = [ln for ln in open(p).read().splitlines() if ln.startswith("{")]
        if txt:
            bench = json.loads(txt[-1])
            break
iters = {b["bounce"]: b["wave_iters"] for b in bench["frame"]["per_bounce"]} if bench else {}
rows = collections.defaultdict(lambda: collections.defaultdict(list))
for pas in ("mix", "mix2"):
    f = os.path.join(src, pas, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    disp = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        kn = r["Kernel_Name"]
        if not kn.startswith("void k_extend<false"):
            continue
        disp[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    for i, d in enumerate(sorted(disp)):
        b = i % depth
        for k, v in disp[d].items():
            rows[b][k].append(v)
keys = ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_BRANCH", "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS", "SQ_INSTS_SMEM",
        "SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA", "SQ_WAIT_ANY",
        "SQ_ACTIVE_INST_ANY", "SQ_INSTS_VALU_TRANS_F32", "SQ_BUSY_CYCLES"]
print(f"# k_extend instruction mix per wave iteration ({src}, {fpl:g} frames per launch)\n")
print("Per bounce: counter mean over the run's launches of that bounce / (wave iterations per frame of the "
      "instrumented pass x frames per launch).  SQ_INSTS_* count wave instructions; *_CYCLES and SQ_WAIT_* are "
      "summed over waves (quad-cycle units per the rocprofv3 definitions).\n")
have = [k for k in keys if any(k in rows[b] for b in rows)]
print("| bounce | wave iters / launch | " + " | ".join(k.replace("SQ_", "") for k in have) + " |")
print("|---|---|" + "---|" * len(have))
for b in sorted(rows):
    wi = iters.get(b, 0) * fpl
    cells = []
    for k in have:
        v = rows[b].get(k)
        if not v or not wi:
            cells.append("-")
            continue
        cells.append(f"{sum(v) / len(v) / wi:.1f}")
    print(f"| {b} | {wi:.4g} | " + " | ".join(cells) + " |")
print("\nRaw per-launch means:\n")
for b in sorted(rows):
    print(f"- bounce {b}: " + ", ".join(f"{k}={sum(v) / len(v):.4g} (n={len(v)})" for k, v in sorted(rows[b].items())))
