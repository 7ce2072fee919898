"""Stream -> hardware queue map and transfer/compute overlap of a rocprofv3 kernel trace.
  python tools/queue_map.py <results.db> [transfer substring]"""
import sqlite3
import sys

sys.path.insert(0, __import__("os").path.dirname(__file__))
from overlap_report import report  # noqa: E402

db = sys.argv[1]
c = sqlite3.connect(db)
print("stream_id queue_id kernels:", c.execute("select stream_id, queue_id, count(*) from kernels "
                                                 "where name not like '%rocclr%' group by stream_id, queue_id").fetchall())
print(report(db, sys.argv[2] if len(sys.argv) > 2 else "rcclGenericKernel").splitlines()[-1])
