"""Summarise a rocprofv3 results.db (kernel trace) into a per-kernel table."""
import sqlite3
import sys


def summarize(db, top=30):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else None)
    rows = c.execute(f"select {name_col}, count(*), sum(end-start), avg(end-start), max(end-start) "
                     f"from kernels group by {name_col} order by sum(end-start) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    out = [f"{'kernel':70s} {'calls':>6s} {'total_ms':>10s} {'avg_us':>10s} {'max_us':>10s} {'pct':>6s}"]
    for name, n, tot, avg, mx in rows[:top]:
        short = (name or "?")[:70]
        out.append(f"{short:70s} {n:6d} {tot/1e6:10.3f} {avg/1e3:10.1f} {mx/1e3:10.1f} {100*tot/total:6.1f}")
    out.append(f"{'TOTAL':70s} {sum(r[1] for r in rows):6d} {total/1e6:10.3f}")
    return "\n".join(out)


if __name__ == "__main__":
    print(summarize(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 30))
