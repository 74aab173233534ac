"""Per-kernel summary (calls, total/avg ms) from a rocprofv3 results database."""
import collections
import sqlite3
import sys

db = sys.argv[1]
c = sqlite3.connect(db)
agg = collections.defaultdict(list)
for name, dur in c.execute("select name, duration from kernels"):
    agg[name.split("(")[0]].append(dur / 1e6)
tot = sum(sum(v) for v in agg.values())
print(f"{'kernel':40s} {'calls':>6s} {'total_ms':>10s} {'avg_ms':>9s} {'pct':>6s}")
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k:40s} {len(v):6d} {sum(v):10.3f} {sum(v)/len(v):9.3f} {100*sum(v)/tot:6.1f}")
