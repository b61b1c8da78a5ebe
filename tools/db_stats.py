"""Dev tool: per-kernel totals from a rocprofv3 SQLite output (.db).

    python tools/db_stats.py gpurun_out/bprof/xxx_results.db [name-regex]
"""
import re
import sqlite3
import sys
from collections import defaultdict

db = sys.argv[1]
pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
c = sqlite3.connect(db)
agg = defaultdict(lambda: [0, 0.0, 0.0])
for name, dur in c.execute("select name, duration from kernels"):
    short = re.sub(r"\(.*", "", name)
    if pat and not pat.search(short):
        continue
    a = agg[short]
    a[0] += 1
    a[1] += dur / 1e6
    a[2] = max(a[2], dur / 1e6)
tot = sum(v[1] for v in agg.values())
print(f"{'kernel':70s} {'calls':>6s} {'total ms':>10s} {'avg ms':>9s} {'max ms':>9s} {'%':>6s}")
for k, (n, t, mx) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{k[:70]:70s} {n:6d} {t:10.3f} {t / n:9.4f} {mx:9.4f} {100 * t / tot:6.1f}")
print(f"total {tot:.3f} ms")
