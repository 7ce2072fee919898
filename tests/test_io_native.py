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
