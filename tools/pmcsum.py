"""Per-kernel PMC summary from rocprofv3 --pmc result databases (one line per kernel/counter)."""
import collections
import sqlite3
import sys

rows = collections.defaultdict(dict)
for db in sys.argv[1:]:
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(counters_collection)")]
    q = "select kernel_name, counter_name, sum(value), count(distinct dispatch_id) from counters_collection group by kernel_name, counter_name"
    for k, cn, v, nd in c.execute(q):
        rows[k.split("(")[0]][cn] = (v, nd)
for k in sorted(rows):
    if "hbx::" not in k:
        continue
    items = ", ".join(f"{cn}={v / nd:.4g}" for cn, (v, nd) in sorted(rows[k].items()))
    print(f"{k}: {items}")
