"""Per-kernel summary of a rocprofv3 SQLite (rocpd) database: calls, total / average / max
duration and share of GPU time, sorted by total time.

Usage: python tools/rocpd_summary.py <run_results.db> [--top N]
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=20)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), max(duration) from kernels "
                     "group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    print(f"{'kernel':100s} {'calls':>6s} {'total_ms':>10s} {'avg_us':>10s} {'max_us':>10s} {'pct':>6s}")
    for name, n, tot, avg, mx in rows[:a.top]:
        print(f"{name[:100]:100s} {n:6d} {tot / 1e6:10.3f} {avg / 1e3:10.1f} {mx / 1e3:10.1f} {100 * tot / total:6.1f}")


if __name__ == "__main__":
    main()
