"""Per-dispatch PMC table for the traversal kernels of a tools/profile.sh run,
normalised per wave iteration (iterations from the bench JSON's per-bounce stats).
usage: python tools/pmc_table.py gpurun_out/prof_<tag> gpurun_out/bench.json"""
import csv, collections, json, os, sys

src = sys.argv[1]
bench = json.load(open(sys.argv[2])) if len(sys.argv) > 2 else None
d = collections.defaultdict(dict)
for p in os.listdir(src):
    f = os.path.join(src, p, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    for r in csv.DictReader(open(f)):
        k = (int(r["Dispatch_Id"]), r["Kernel_Name"].split("(")[0].replace("void ", ""))
        d[k][r["Counter_Name"]] = float(r["Counter_Value"])
iters = {}
if bench:
    for b in bench["frame"]["per_bounce"]:
        iters[("k_extend", b["bounce"])] = b.get("wave_iters")
        iters[("k_shadow", b["bounce"])] = b.get("shadow_wave_iters")
cnt = collections.Counter()
for k in sorted(d):
    name = k[1]
    if not (name.startswith("k_extend<false") or name.startswith("k_shadow<false")):
        continue
    base = name.split("<")[0]
    b = cnt[base]
    cnt[base] += 1
    c = d[k]
    it = iters.get((base, b))
    row = [f"{name:16s} b{b}"]
    for key in ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_BRANCH", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD"]:
        if key in c:
            row.append(f"{key[9:]}={c[key]:.3g}" + (f" ({c[key] / it:.0f}/it)" if it else ""))
    wc = c.get("SQ_WAVE_CYCLES")
    if wc:
        for key in ["SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA"]:
            if key in c:
                row.append(f"{key[3:]}={c[key] / wc:.2f}")
    print(" ".join(row))
