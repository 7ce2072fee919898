"""pandas-style DataFrame API: merge, join on index, concat, drop_duplicates, sort_values,
groupby, device moves (reference: python/examples/dataframe/*.py).

    python examples/python/dataframe_ops.py [--device cpu|cuda:0]
"""
import pandas as pd

from _common import device_from_argv, report
from cylon_amd import DataFrame

dev = device_from_argv()
df1 = DataFrame(pd.DataFrame({"key": [1, 2, 3, 4, 5], "a": [10, 20, 30, 40, 50]})).to_device(dev)
df2 = DataFrame(pd.DataFrame({"key": [2, 3, 5, 7], "b": [0.2, 0.3, 0.5, 0.7]})).to_device(dev)

m = df1.merge(df2, how="inner", on="key")
report("merge_rows", len(m))
report("left_merge_rows", len(df1.merge(df2, how="left", on="key")))

# axis=0 concat is the reference's set union of the frames (frame.py:1610-1634): duplicates fold
extra = DataFrame(pd.DataFrame({"key": [5, 6], "a": [50, 60]})).to_device(dev)
report("concat_rows", len(DataFrame.concat([df1, extra])))

s = df1.sort_values(by="a", ascending=False).to_pandas()
report("sort_first_a", int(s["a"].iloc[0]))

g = DataFrame(pd.DataFrame({"g": [1, 1, 2, 2, 2], "v": [1.0, 2.0, 3.0, 4.0, 5.0]})).to_device(dev)
out = g.groupby(by="g", agg={"v": "sum"}).to_pandas().sort_values("g")
report("group_sums", ",".join(str(float(x)) for x in out.iloc[:, -1]))
report("dedup_rows", len(g.drop_duplicates(subset="g")))

j = df1.set_index("key").join(df2.set_index("key"), how="inner")
report("index_join_rows", len(j))
report("on_host", df1.to_cpu().is_cpu())
