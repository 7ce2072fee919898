import os, sys
sys.path.insert(0, os.getcwd())
os.environ["CYLON_RADIX_SETOP_MIN_ROWS"] = "1"
import numpy as np, pyarrow as pa
sys.path.insert(0, "tests")
from test_gpu_ops import _setop_frames
from cylon_amd import CylonContext, Table
g = CylonContext(device="cuda:0"); c = CylonContext(device="cpu")
a, b = _setop_frames(60_000, 40_000, 5)
a, b = a.drop(["s"]), b.drop(["s"])
for n in (100, 1000, 10000, 60000):
    aa = a.slice(0, n)
    G = Table(aa, g).unique(None).to_pandas(); C = Table(aa, c).unique(None).to_pandas()
    print(n, len(G), len(C))
aa = a.slice(0, 1000)
G = Table(aa, g).unique(None).to_pandas(); C = Table(aa, c).unique(None).to_pandas()
key = lambda df: set(map(lambda r: tuple("nan" if isinstance(x, float) and x != x else x for x in r), df.itertuples(index=False)))
miss = key(C) - key(G)
print("missing", list(miss)[:10])
df = aa.to_pandas()
for m in list(miss)[:3]:
    print(m, df[(df.x == m[0])])
