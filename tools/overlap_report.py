"""Overlap of the asynchronous transport's delay kernels with the join kernels in a
rocprofv3 kernel trace (results.db): for every k_spin_delay interval, the compute
kernels that ran while it was in flight.  Used for profiles/async_overlap_*.txt."""
import sqlite3
import sys


def report(db):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, start, end from kernels order by start").fetchall()
    spins = [(s, e) for n, s, e in rows if "k_spin_delay" in (n or "")]
    work = [(n, s, e) for n, s, e in rows if "k_spin_delay" not in (n or "") and "rocclr" not in (n or "")]
    out = [f"{len(spins)} delay kernels, {len(work)} compute kernels"]
    total_ov = 0
    for i, (s, e) in enumerate(spins):
        ov = [(n, max(s, ws), min(e, we)) for n, ws, we in work if ws < e and we > s]
        t = sum(b - a for _, a, b in ov)
        total_ov += t
        names = sorted({(n or "?").split("(")[0].split("<")[0].replace("void ", "")[-40:] for n, _, _ in ov})
        out.append(f"delay {i:3d}: {(e - s) / 1e3:9.1f} us in flight, {len(ov):4d} compute kernels overlapping "
                   f"for {t / 1e3:9.1f} us: {', '.join(names[:6])}")
    span = sum(e - s for s, e in spins)
    out.append(f"TOTAL delay-in-flight {span / 1e6:.3f} ms, compute overlapped with it {total_ov / 1e6:.3f} ms")
    return "\n".join(out)


if __name__ == "__main__":
    print(report(sys.argv[1]))
