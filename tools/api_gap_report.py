"""Host-side HIP API time per step of a rocprofv3 --kernel-trace --hip-trace database, and what the
host was inside while the compute stream sat idle (the first-step overlap question: transfers in
flight, no compute kernel to overlap them with).

  python tools/api_gap_report.py <results.db> [transfer substring, default rcclGenericKernel] [steps] [skip]

Steps are found as in overlap_report.py (transfer kernels split into `steps` equal groups).  For
every step: the HIP API calls by total time, the longest single calls, and every gap > 2 ms
between consecutive non-transfer kernels with the API calls that overlapped it."""
import collections
import sqlite3
import sys


def short(n, k=60):
    return (n or "?").split("(")[0].replace("void ", "").replace("cylon::hip::", "")[:k]


def main():
    db = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else "rcclGenericKernel"
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    skip = int(sys.argv[4]) if len(sys.argv) > 4 else 0  # leading transfers (the context's warm-up exchange)
    c = sqlite3.connect(db)
    ks = c.execute("select name, start, end from kernels order by start").fetchall()
    api = c.execute("select name, start, end from regions order by start").fetchall()
    # the kernel each launch call dispatched (correlation id)
    kcorr = dict(c.execute("select corr_id, name from kernels").fetchall())
    acorr = {(n, st): cid for n, st, cid in c.execute("select name, start, corr_id from regions").fetchall()}
    if not ks:
        print("no kernels")
        return
    t0 = ks[0][1]
    xfer = [k for k in ks if pat in (k[0] or "")][skip:]
    work = [k for k in ks if pat not in (k[0] or "") and "rocclr" not in (k[0] or "")]
    per = max(1, len(xfer) // steps)
    print(f"{len(ks)} kernels, {len(api)} HIP API calls, {len(xfer)} transfer kernels ({pat})")
    for s in range(steps):
        grp = xfer[s * per:(s + 1) * per]
        if not grp:
            continue
        a, b = grp[0][1], grp[-1][2]
        print(f"\n== step {s}: transfers {(a - t0) / 1e6:.1f} .. {(b - t0) / 1e6:.1f} ms")
        inwin = [x for x in api if x[2] > a and x[1] < b]
        tot = collections.Counter()
        cnt = collections.Counter()
        for n, st, en in inwin:
            tot[n] += (min(en, b) - max(st, a)) / 1e6
            cnt[n] += 1
        print("  HIP API time inside the transfer window (ms, calls):")
        for n, v in tot.most_common(8):
            print(f"    {v:9.2f} {cnt[n]:6d}  {n}")
        print("  longest calls:")
        for n, st, en in sorted(inwin, key=lambda x: x[1] - x[2])[:6]:
            k = kcorr.get(acorr.get((n, st)), "")
            print(f"    {(en - st) / 1e6:9.2f} ms at {(st - t0) / 1e6:9.1f}  {n}  {short(k, 70)}")
        wk = [k for k in work if k[2] > a and k[1] < b]
        for (n1, s1, e1), (n2, s2, e2) in zip(wk, wk[1:]):
            gap = (s2 - e1) / 1e6
            if gap > 2.0:
                hold = collections.Counter()
                for n, st, en in api:
                    if en > e1 and st < s2:
                        hold[n] += (min(en, s2) - max(st, e1)) / 1e6
                top = ", ".join(f"{n} {v:.1f}" for n, v in hold.most_common(3))
                print(f"  idle {gap:7.2f} ms after {short(n1, 40)} @ {(e1 - t0) / 1e6:.1f}: {top}")


if __name__ == "__main__":
    main()
