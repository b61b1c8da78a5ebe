"""Summarise a tools/profile.sh output dir into profiles/<tag>_summary.md + pmc JSON.

FETCH_SIZE / WRITE_SIZE are in KB (rocprofv3); per MI355X_MICROARCH.md §HBM,
FETCH_SIZE reads 1/2 of the bytes of wide (16 B/lane) reads on gfx950, so the
corrected read traffic is 2 x FETCH_SIZE; WRITE_SIZE is taken as is.
"""
import csv, collections, json, os, sys

src, tag = sys.argv[1], sys.argv[2]
dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles")
os.makedirs(dst, exist_ok=True)
lines = [f"# rocprofv3 summary {tag}", ""]
stats = os.path.join(src, "trace", "run_kernel_stats.csv")
if os.path.exists(stats):
    lines += ["## kernel trace (--kernel-trace --stats)", "", "| kernel | calls | total ms | avg ms | % |", "|---|---|---|---|---|"]
    for r in csv.DictReader(open(stats)):
        lines.append(f"| {r['Name'][:60]} | {r['Calls']} | {float(r['TotalDurationNs'])/1e6:.2f} | "
                     f"{float(r['AverageNs'])/1e6:.3f} | {float(r['Percentage']):.1f} |")
    lines.append("")
pmc = collections.defaultdict(dict)
for p in ["fetch", "write", "sq", "tcc"]:
    f = os.path.join(src, p, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    for r in csv.DictReader(open(f)):
        key = (r["Kernel_Name"].split("(")[0].replace("void ", ""), p, int(r["Dispatch_Id"]))
        pmc[key][r["Counter_Name"]] = float(r["Counter_Value"])
        pmc[key]["dur_ms"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        pmc[key]["scratch"] = r.get("Scratch_Size"); pmc[key]["vgpr"] = r.get("VGPR_Count"); pmc[key]["lds"] = r.get("LDS_Block_Size")
out = {}
if pmc:
    lines += ["## PMC (separate passes; last timed frame's launches = uninstrumented kernels)", "",
              "| kernel | pass | dispatch | counters | ms |", "|---|---|---|---|---|"]
    for (k, p, d), v in sorted(pmc.items(), key=lambda x: (x[0][1], x[0][2])):
        cs = " ".join(f"{a}={b:.4g}" for a, b in v.items() if a not in ("dur_ms", "scratch", "vgpr", "lds"))
        lines.append(f"| {k} | {p} | {d} | {cs} vgpr={v['vgpr']} scratch={v['scratch']} lds={v['lds']} | {v['dur_ms']:.2f} |")
    # per-launch HBM traffic of the uninstrumented extend kernel (average over its launches)
    def avg(kname, pas, cn):
        vals = [v[cn] for (k, p, d), v in pmc.items() if k == kname and p == pas and cn in v]
        return sum(vals) / len(vals) if vals else None
    f_ = avg("k_extend<false>", "fetch", "FETCH_SIZE")
    w_ = avg("k_extend<false>", "write", "WRITE_SIZE")
    if f_ is not None and w_ is not None:
        out = {"kernel": "k_extend<false>", "fetch_kb_raw": f_, "write_kb": w_,
               "bytes_per_launch": int((2 * f_ + w_) * 1024),
               "note": "read = 2 x FETCH_SIZE (gfx950 half-count correction, MI355X_MICROARCH.md §HBM) + WRITE_SIZE; KB units"}
        json.dump(out, open(os.path.join(dst, f"pmc_extend_{tag}.json"), "w"), indent=1)
        lines += ["", f"extend per-launch HBM traffic (corrected): {out['bytes_per_launch']/1e9:.2f} GB"]
open(os.path.join(dst, f"{tag}_summary.md"), "w").write("\n".join(lines) + "\n")
print("\n".join(lines[:30]))
