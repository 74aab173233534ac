"""HBM bytes per launch of one kernel from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE), as
the JSON record bench.py's `traffic` field reads (profiles/<tag>_pmc_hbm.json).

    python tools/pmc_json.py <fetch results.db> <write results.db> <kernel>[,<kernel>...] <commit> [--skip-empty] > out.json

Several comma-separated kernel names make one region (the one-lane share check is the Miller
kernel + seven step kernels + the fallback launch): its bytes are the sum of each kernel's bytes
per launch.

Units and the gfx950 correction follow /opt/skills/guides/MI355X_MICROARCH.md (HBM section):
FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts half the bytes of wide reads
(TCC_EA0_RDREQ x 64 B for 128-B requests), so it is doubled; WRITE_SIZE is taken as is.  Both are
memory-side (L2 -> fabric) counters, so Infinity-Cache hits are included: an upper bound on HBM
bytes."""
import json
import sqlite3
import sys


SKIP_EMPTY = "--skip-empty" in sys.argv  # launches that return at once (a retry pass with nothing
                                        # to retry) are not launches of the region


def per_launch(db, counter, kernel):
    c = sqlite3.connect(db)
    q = ("select dispatch_id, sum(value) from counters_collection "
         "where counter_name = ? and kernel_name like ? group by dispatch_id")
    vals = [v for _, v in c.execute(q, (counter, f"%{kernel}%")).fetchall()]
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel} in {db}")
    if SKIP_EMPTY:
        top = max(vals)
        vals = [v for v in vals if v > 0.01 * top] or vals
    return sum(vals) / len(vals), len(vals)


def main():
    fdb, wdb, kernel, commit = [a for a in sys.argv[1:] if not a.startswith("--")][:4]
    f_kib = w_kib = 0.0
    nf, nw = [], []
    parts = {}
    for k in kernel.split(","):
        fk, a = per_launch(fdb, "FETCH_SIZE", k)
        wk, b = per_launch(wdb, "WRITE_SIZE", k)
        f_kib += fk
        w_kib += wk
        nf.append(a)
        nw.append(b)
        parts[k] = round(2 * fk * 1024 + wk * 1024)
    nf, nw = (nf[0], nw[0]) if len(nf) == 1 else (nf, nw)
    fetch = 2 * f_kib * 1024
    write = w_kib * 1024
    print(json.dumps({"kernel": kernel, "bytes_per_launch": round(fetch + write), "fetch_bytes": round(fetch),
                      "write_bytes": round(write), "fetch_size_kib_raw": f_kib, "write_size_kib_raw": w_kib,
                      "launches": [nf, nw], "fetch_correction": 2, "commit": commit,
                      **({"parts": parts} if len(parts) > 1 else {}),
                      "note": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes; FETCH doubled (gfx950)"}))


if __name__ == "__main__":
    main()
