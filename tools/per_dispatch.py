"""Per-dispatch view of a profile dir: python tools/per_dispatch.py gpurun_out/prof_<tag> [passes...]"""
import csv, collections, sys
src = sys.argv[1]
passes = sys.argv[2:] or ["ta", "tas", "tcp", "tcpa", "sq", "lat", "ea", "tcc", "mix", "mix2"]
per = collections.defaultdict(lambda: collections.defaultdict(dict))
for p in passes:
    try:
        rows = list(csv.DictReader(open(f"{src}/{p}/run_counter_collection.csv")))
    except OSError:
        continue
    for kname in ("k_extend<false>", "k_shadow<false>"):
        ks = [r for r in rows if r["Kernel_Name"].split("(")[0].replace("void ", "") == kname]
        ids = sorted(set(int(r["Dispatch_Id"]) for r in ks))
        for r in ks:
            b = ids.index(int(r["Dispatch_Id"]))
            d = per[kname][b]
            d[r["Counter_Name"] + ("@" + p if r["Counter_Name"] == "GRBM_GUI_ACTIVE" else "")] = float(r["Counter_Value"])
            d["ms"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
for k, dd in per.items():
    for b, v in sorted(dd.items()):
        out = [f"{k} b{b} ms={v['ms']:.2f}"]
        for cn, pas, scale in (("TA_BUSY_avr", "ta", 1), ("TA_ADDR_STALLED_BY_TC_CYCLES_sum", "tas", 256),
                               ("TCP_PENDING_STALL_CYCLES_sum", "tcp", 256)):
            if cn in v and "GRBM_GUI_ACTIVE@" + pas in v:
                out.append(f"{cn.split('_sum')[0].split('_avr')[0]}={v[cn] / v['GRBM_GUI_ACTIVE@' + pas] / scale:.2f}")
        for cn in ("TCP_TOTAL_CACHE_ACCESSES_sum", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH",
                   "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY",
                   "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_LDS",
                   "SQ_WAIT_INST_LDS", "SQ_INSTS_VALU_TRANS_F32"):
            if cn in v:
                out.append(f"{cn}={v[cn]:.3g}")
        print(" ".join(out))
