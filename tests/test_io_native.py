"""Native C++ CSV reader/writer (cylon/io/csv.cpp, C25) vs Arrow's CSV reader."""
import glob
import os

import pandas as pd
import pytest

from cylon_amd import C
from cylon_amd.io import CSVReadOptions, read_csv

DATA = os.path.join(os.path.dirname(__file__), "data")


def _both(ctx, path, opts_fn=lambda: CSVReadOptions(), monkeypatch=None):
    monkeypatch.setenv("CYLON_CSV_READER", "native")
    a = read_csv(ctx, path, opts_fn()).to_pandas()
    monkeypatch.setenv("CYLON_CSV_READER", "arrow")
    b = read_csv(ctx, path, opts_fn()).to_pandas()
    return a, b


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(DATA, "input", "*.csv"))))
def test_native_reader_matches_arrow_on_fixtures(ctx, path, monkeypatch):
    a, b = _both(ctx, path, monkeypatch=monkeypatch)
    pd.testing.assert_frame_equal(a, b)


def test_native_reader_edge_cases(ctx, tmp_path, monkeypatch):
    p = tmp_path / "e.csv"
    p.write_bytes(b'junk line\r\nid,name,score,flag,mixed\r\n1,"a, b",1.5,true,x\r\n\r\n'
                  b'2,"say ""hi""",,false,3\r\n3,NA,2,TRUE,\r\n-4,plain,1e3,false,4.5\r\n')
    def opts():
        return CSVReadOptions().skip_rows(1)
    a, b = _both(ctx, str(p), opts, monkeypatch)
    pd.testing.assert_frame_equal(a, b)
    assert a["name"].tolist() == ["a, b", 'say "hi"', "NA", "plain"]
    assert a["flag"].tolist() == [True, False, True, False]
    # subset + renamed + tab-delimited + strings_can_be_null
    q = tmp_path / "t.tsv"
    q.write_text("1\tx\t5\n2\t\t6\n")
    def opts2():
        return (CSVReadOptions().with_delimiter("\t").column_names(["a", "b", "c"]).use_cols(["c", "b"])
                .strings_can_be_null(True))
    a, b = _both(ctx, str(q), opts2, monkeypatch)
    pd.testing.assert_frame_equal(a, b)
    assert list(a.columns) == ["c", "b"] and a["b"].isna().tolist() == [False, True]


def test_native_multi_file_and_writer_roundtrip(ctx, tmp_path, monkeypatch):
    monkeypatch.setenv("CYLON_CSV_READER", "native")
    files = sorted(glob.glob(os.path.join(DATA, "input", "csv1_*.csv")))
    tabs = read_csv(ctx, files)
    assert len(tabs) == len(files)
    out = tmp_path / "w.csv"
    C.write_csv(tabs[0].native, str(out))
    back = read_csv(ctx, str(out)).to_pandas()
    pd.testing.assert_frame_equal(back, tabs[0].to_pandas())


def test_native_parquet_roundtrip_all_types(ctx, tmp_path):
    """io/arrow_io.cpp (Arrow / Parquet C++): every supported type with nulls, column selection,
    concurrent multi-file reads, compression codecs."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    from cylon_amd.io import ParquetOptions, read_parquet, write_parquet
    at = pa.table({"i8": pa.array([1, None, -3], pa.int8()), "u64": pa.array([1, 2, 2**63], pa.uint64()),
                   "i": pa.array([1, None, 3], pa.int32()), "s": ["a", None, "ccc"], "f": [1.5, 2.5, None],
                   "h": pa.array([1.0, 2.0, None], pa.float16()), "b": [True, False, None],
                   "bin": pa.array([b"\x00x", None, b""], pa.binary()),
                   "ts": pa.array([1, 2, None], pa.timestamp("us", tz="UTC")),
                   "t64": pa.array([5, 6, 7], pa.time64("ns")), "dur": pa.array([1, None, 3], pa.duration("s")),
                   "fx": pa.array([b"ab", b"cd", b"ef"], pa.binary(2)), "d": pa.array([10, 20, 30], pa.date32())})
    src = str(tmp_path / "x.parquet")
    pq.write_table(at, src)
    t = read_parquet(ctx, src)
    assert t.to_arrow().equals(at)
    for codec in ("snappy", "zstd", "none"):
        out = str(tmp_path / f"y_{codec}.parquet")
        write_parquet(t, out, ParquetOptions(compression=codec, chunk_size=2))
        back = pq.read_table(out)
        assert back.equals(at) and pq.ParquetFile(out).metadata.num_row_groups == 2
    ts = read_parquet(ctx, [src, str(tmp_path / "y_zstd.parquet")], ParquetOptions(columns=["s", "i8"]))
    assert [x.column_names for x in ts] == [["s", "i8"], ["s", "i8"]]
    assert ts[1].to_pydict() == {"s": ["a", None, "ccc"], "i8": [1, None, -3]}
    with pytest.raises(Exception):
        read_parquet(ctx, src, ParquetOptions(columns=["nope"]))
    with pytest.raises(Exception):
        read_parquet(ctx, str(tmp_path / "missing.parquet"))


def test_native_parquet_large_strings(ctx, tmp_path):
    import pyarrow as pa
    import pyarrow.parquet as pq
    from cylon_amd.io import read_parquet
    at = pa.table({"s": pa.array(["x" * 5, "yy", None], pa.large_string())})
    p = str(tmp_path / "l.parquet")
    pq.write_table(at, p)
    assert read_parquet(ctx, p).to_pydict() == {"s": ["xxxxx", "yy", None]}


def test_native_reader_escaping_and_multiline_values(ctx, tmp_path, monkeypatch):
    """Escape characters and quoted values spanning lines (HasNewLinesInValues) parse
    natively the way Arrow's reader parses them."""
    p = tmp_path / "m.csv"
    p.write_bytes(b'id,text,v\n1,"line one\nline two",1.5\n2,plain\\,comma,2.5\n3,"say \\"hi\\"",3.0\n'
                  b'4,"a\r\nb",4.0\n')
    opts = lambda: CSVReadOptions().use_escaping().has_new_lines_in_values()  # noqa: E731
    a, b = _both(ctx, str(p), opts, monkeypatch)
    pd.testing.assert_frame_equal(a, b)
    assert a["text"].tolist()[:3] == ["line one\nline two", "plain,comma", 'say "hi"']


def test_native_reader_column_types_and_missing_columns(ctx, tmp_path, monkeypatch):
    import pyarrow as pa
    p = tmp_path / "t.csv"
    p.write_text("a,b,c,d\n1,2.5,x,1\n-3,,y,0\n7,4.25,,1\n")
    opts = lambda: (CSVReadOptions()  # noqa: E731
                    .with_column_types({"a": pa.int32(), "b": pa.float32(), "d": pa.bool_(), "e": pa.int16()})
                    .use_cols(["d", "a", "e", "b"]).include_missing_columns())
    a, b = _both(ctx, str(p), opts, monkeypatch)
    pd.testing.assert_frame_equal(a, b)
    t = read_csv(ctx, str(p), opts())
    assert [str(x) for x in t.to_arrow().schema.types] == ["bool", "int32", "int16", "float"]
    assert t.to_pandas()["e"].isna().all()


def test_native_reader_rejects_bad_typed_values(ctx, tmp_path, monkeypatch):
    import pyarrow as pa
    p = tmp_path / "bad.csv"
    p.write_text("a,b\n1,2\nx,3\n")
    monkeypatch.setenv("CYLON_CSV_READER", "native")
    with pytest.raises(Exception, match="conversion"):
        read_csv(ctx, str(p), CSVReadOptions().with_column_types({"a": pa.int64()}))
