"""Overlap of transfer kernels with compute kernels in a rocprofv3 kernel trace (results.db):
for every transfer-kernel interval, the compute kernels that ran while it was in flight.

  python tools/overlap_report.py <results.db> [transfer substring, default k_spin_delay] [steps] [skip]

skip: leading transfer kernels to ignore (1 for a distributed context's RCCL warm-up exchange).

steps: the trace holds that many equal steps (e.g. 2 for --warmup 1 --steps 1): the transfers are
split into that many consecutive groups and each group's overlap is reported (the first step also
pays the communicator's first-use setup).

k_spin_delay = the asynchronous delay transport (profiles/async_overlap_*.txt);
rcclGenericKernel = the RCCL all-to-all kernels of a forced / multi-rank shuffle
(profiles/rccl_forced_*.txt)."""
import sqlite3
import sys


def short(n):
    return (n or "?").split("(")[0].replace("void ", "").replace("cylon::hip::", "")[:48]


def report(db, pat="k_spin_delay", steps=1, skip=0):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, start, end from kernels order by start").fetchall()
    xfer = [(n, s, e) for n, s, e in rows if pat in (n or "")][skip:]  # skip: the context's warm-up exchange
    work = [(n, s, e) for n, s, e in rows if pat not in (n or "") and "rocclr" not in (n or "")]
    out = [f"{len(xfer)} transfer kernels ({pat}), {len(work)} compute kernels"]
    total_ov = 0
    per = []
    t0 = rows[0][1] if rows else 0
    for i, (n, s, e) in enumerate(xfer):
        ov = [(wn, max(s, ws), min(e, we)) for wn, ws, we in work if ws < e and we > s]
        t = sum(b - a for _, a, b in ov)
        total_ov += t
        per.append((e - s, t))
        names = sorted({short(wn) for wn, _, _ in ov})
        out.append(f"xfer {i:3d} @ {(s - t0) / 1e6:9.3f} ms: {(e - s) / 1e3:9.1f} us in flight, {len(ov):4d} compute "
                   f"kernels overlapping for {t / 1e3:9.1f} us: {', '.join(names[:5])}")
    span = sum(e - s for _, s, e in xfer)
    out.append(f"TOTAL transfer-in-flight {span / 1e6:.3f} ms, compute overlapped with it {total_ov / 1e6:.3f} ms")
    if steps > 1 and per:
        g = len(per) // steps
        for k in range(steps):
            part = per[k * g:(k + 1) * g] if k + 1 < steps else per[k * g:]
            fl, ov = sum(p[0] for p in part), sum(p[1] for p in part)
            out.append(f"STEP {k}: {len(part)} transfers, in flight {fl / 1e6:.3f} ms, overlapped {ov / 1e6:.3f} ms "
                       f"({100.0 * ov / max(fl, 1):.1f} %)")
    return "\n".join(out)


if __name__ == "__main__":
    print(report(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "k_spin_delay",
                 int(sys.argv[3]) if len(sys.argv) > 3 else 1, int(sys.argv[4]) if len(sys.argv) > 4 else 0))
