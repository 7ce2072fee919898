"""Arrow boundary: validity bitmaps packed / unpacked by the engine's kernels, the Arrow C
Device Data Interface (zero-copy HBM hand-off) and the PyCapsule stream export
(reference: util/copy_arrray.cpp:24-110 builds bitmaps on the host; arrow/arrow_builder.cpp:31-161
builds tables zero-copy from raw buffers)."""
import numpy as np
import pyarrow as pa
import pytest
import torch

from cylon_amd import Table
from cylon_amd._lib import C


def _all_types(n=500, seed=0):
    rng = np.random.default_rng(seed)
    mask = rng.random(n) < 0.2
    return pa.table({
        "i64": pa.array(rng.integers(-9, 9, n), mask=mask),
        "f32": pa.array(rng.random(n).astype(np.float32)),
        "u16": pa.array(rng.integers(0, 60000, n).astype(np.uint16), mask=mask),
        "b": pa.array(rng.random(n) < 0.5, mask=rng.random(n) < 0.1),
        "s": pa.array([None if m else f"v{x}" for x, m in zip(rng.integers(0, 99, n), mask)]),
        "ts": pa.array(rng.integers(0, 1 << 40, n), pa.timestamp("us", tz="UTC")),
        "l": pa.array([None if m else list(map(int, rng.integers(0, 5, x))) for x, m in
                       zip(rng.integers(0, 4, n), mask)], pa.list_(pa.int32())),
        "fsl": pa.array([list(map(float, v)) for v in rng.random((n, 2))], pa.list_(pa.float64(), 2)),
    })


@pytest.mark.parametrize("n,off", [(1, 0), (63, 5), (64, 0), (1000, 13), (4097, 7)])
def test_bitmap_pack_unpack_kernels(ctx, n, off):
    rng = np.random.default_rng(n)
    v = (rng.random(n) < 0.7).astype(np.uint8)
    words, nulls = C.pack_validity(torch.from_numpy(v).to(ctx.device))
    assert nulls == int(n - v.sum())
    assert words.cpu().numpy().view(np.uint8)[: (n + 7) // 8].tobytes() == np.packbits(v, bitorder="little").tobytes()
    padded = np.concatenate([np.zeros(off, np.uint8), v])
    bits = torch.from_numpy(np.packbits(padded, bitorder="little")).to(ctx.device)
    assert np.array_equal(C.unpack_validity(bits, off, n).cpu().numpy(), v)


def test_c_device_interface_roundtrip_cpu(ctx):
    at = _all_types()
    t = Table(at, ctx)
    rb = pa.RecordBatch._import_from_c_device_capsule(*t.__arrow_c_device_array__())  # pyarrow as the consumer
    for name in at.column_names:
        assert rb.column(name).to_pylist() == at.column(name).to_pylist(), name
    back = Table.from_arrow_device(ctx, t).to_arrow()
    assert back.to_pydict() == at.to_pydict()
    assert pa.table(t).to_pydict() == at.to_pydict()  # __arrow_c_stream__


def test_c_device_interface_import_sliced_pyarrow(ctx):
    at = _all_types(300, 1).slice(17, 200)
    rb = at.combine_chunks().to_batches()[0]
    got = Table.from_arrow_device(ctx, rb).to_arrow()
    assert got.to_pydict() == at.to_pydict()


@pytest.mark.gpu
def test_c_device_interface_zero_copy_on_device(gpu_ctx):
    at = _all_types(100_000, 2)
    t = Table(at, gpu_ctx)
    caps = t.__arrow_c_device_array__()
    t2 = Table.from_arrow_device(gpu_ctx, caps)
    assert t2.to_arrow().to_pydict() == at.to_pydict()
    # fixed-width values and string bytes are the same HBM buffers (no copy)
    n1, n2 = t.native.columns(), t2.native.columns()
    for c1, c2 in zip(n1, n2):
        if c1.name in ("i64", "f32", "u16", "ts", "s", "fsl"):
            assert c1.data.data_ptr() == c2.data.data_ptr(), c1.name
    torch.cuda.synchronize()
