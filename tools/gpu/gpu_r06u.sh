# round 6: kernel split of the first-pass-chunk bounded join (1B x 1B x 6 payload columns, released inputs)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r06u}
mkdir -p $O
. tools/gpu/lib.sh
step bprof 900 rocprofv3 --kernel-trace --stats -d $O/bprof -o p -- python tools/retain_probe.py --rows 1000000000 --payload-cols 6 --steps 1 --warmup 2 --retain 0
python tools/rocpd_summary.py $O/bprof/p_results.db --top 30 > $O/bprof.summary.txt 2>&1 || true
python - $O/bprof/p_results.db > $O/bprof.gaps.txt 2>&1 <<'PY' || true
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name = "kernel_name" if "kernel_name" in cols else "name"
rows = c.execute(f"select {name}, start, end from kernels order by start").fetchall()
# the last step: from the last first-pass chunk pass (k_rows_pass PartDigitN with >= 1 s before) onwards
idx = [i for i, r in enumerate(rows) if "k_rows_pass" in (r[0] or "") and "PartDigitN" in (r[0] or "")]
first = idx[-1]
# walk back to the start of the last join (a gap > 50 ms before a PartDigitN pass)
for i in reversed(idx):
    j = i
    if i > 0 and rows[i][1] - rows[i - 1][2] > 50e6:
        first = i
        break
seg = rows[first:]
busy = sum(e - s for _, s, e in seg)
span = seg[-1][2] - seg[0][1]
print(f"last join: span {span/1e6:.2f} ms, kernel busy {busy/1e6:.2f} ms, idle {100*(span-busy)/span:.1f} %")
PY
head -30 $O/bprof.summary.txt | cut -c1-70,100-175
cat $O/bprof.gaps.txt
rm -rf $O/bprof
