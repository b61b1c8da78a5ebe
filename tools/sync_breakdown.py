"""Gap / tail breakdown of synchronous khp_render calls from a rocprofv3 trace (dev tool).

Input: the kernel_trace.csv (and memory_copy_trace.csv, if present) of
tools/sync_trace.py, plus its JSON line.  A call starts at its k_start (or
k_generate, or k_path) dispatch.  Per call: the device span (first kernel start to the
last kernel/copy end), the time some kernel or copy was running (union), the
idle time inside the span (host waits, launch gaps), and the launches by
kernel with their summed durations; k_extend / k_shadow durations per bounce.
usage: python tools/sync_breakdown.py <trace_dir> <calls.json> [out.md]
"""
import csv
import glob
import json
import os
import sys


def rows_of(pattern):
    fs = glob.glob(pattern, recursive=True)
    return list(csv.DictReader(open(fs[0]))) if fs else []


def union(iv):
    iv = sorted(iv)
    tot, lo, hi = 0, None, None
    for a, b in iv:
        if hi is None or a > hi:
            if hi is not None:
                tot += hi - lo
            lo, hi = a, b
        else:
            hi = max(hi, b)
    if hi is not None:
        tot += hi - lo
    return tot


def main():
    d, calls_path = sys.argv[1], sys.argv[2]
    ks = rows_of(os.path.join(d, "**", "*kernel_trace.csv"))
    cps = rows_of(os.path.join(d, "**", "*memory_copy_trace.csv"))
    calls = json.loads([ln for ln in open(calls_path) if ln.startswith("{")][-1])
    ev = []
    for r in ks:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]
                   .replace("void ", "").split("<")[0]))
    for r in cps:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy:" + r.get("Direction", "?")))
    ev.sort()
    starts = [i for i, e in enumerate(ev) if e[2] in ("k_start", "k_generate", "k_path")]
    n_calls = len(calls["gui"]) + len(calls["sync"])
    starts = starts[-n_calls:]
    names = ["gui"] * len(calls["gui"]) + ["sync"] * len(calls["sync"])
    lines = ["| call | host wall ms | device span ms | busy (union) ms | idle in span ms | k_extend ms by bounce "
             "| k_shadow+finish ms | k_shade ms | launches |", "|---|---|---|---|---|---|---|---|---|"]
    per_kind = {}
    for ci, si in enumerate(starts):
        ei = starts[ci + 1] if ci + 1 < len(starts) else len(ev)
        seg = ev[si:ei]
        # copies/kernels that belong to the call but began before its k_start (memsets) are ignored
        t0 = seg[0][0]
        t1 = max(e[1] for e in seg)
        busy = union([(a, b) for a, b, _ in seg])
        ext = [(b - a) / 1e3 for a, b, n in seg if n == "k_extend"]
        sh = sum((b - a) for a, b, n in seg if n in ("k_shadow", "k_shadow_finish")) / 1e6
        shade = sum((b - a) for a, b, n in seg if n == "k_shade") / 1e6
        kind = names[ci]
        host = calls[kind][ci if kind == "gui" else ci - len(calls["gui"])]
        lines.append(f"| {kind} {ci} | {host['wall_ms']:.2f} | {(t1 - t0) / 1e6:.2f} | {busy / 1e6:.2f} | "
                     f"{(t1 - t0 - busy) / 1e6:.2f} | {' / '.join(f'{x / 1e3:.2f}' for x in ext)} | {sh:.2f} | "
                     f"{shade:.2f} | {len(seg)} |")
        agg = per_kind.setdefault(kind, {})
        for a, b, n in seg:
            s = agg.setdefault(n, [0, 0.0])
            s[0] += 1
            s[1] += (b - a) / 1e6
    lines.append("")
    for kind, agg in per_kind.items():
        nc = len(calls[kind])
        lines.append(f"**{kind}** (per call, mean of {nc}): " + ", ".join(
            f"{n} {v[0] / nc:.1f}x {v[1] / nc:.3f} ms" for n, v in sorted(agg.items(), key=lambda x: -x[1][1])))
        lines.append("")
    txt = "\n".join(lines)
    print(txt)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(txt + "\n")


if __name__ == "__main__":
    main()
