// Bindings for the extended relational operators (set ops, unique, group-by,
// aggregates, range partition, distributed sort).
#include <map>
#include <torch/extension.h>

#include "cylon/kernels/kernels.hpp"
#include <tuple>

#include "cylon/api.hpp"
#include "cylon/io/arrow_io.hpp"
#include "cylon/io/csv.hpp"
#include "cylon/indexing/index.hpp"
#include "cylon/io/device_interop.hpp"
#include "cylon/io/h2d.hpp"
#include "cylon/knobs.hpp"
#include "cylon/ops/api_ext.hpp"
#include "cylon/ops/graph.hpp"
#include "cylon/ops/relational.hpp"
#include "cylon/ops/util.hpp"
#include "cylon/table.hpp"

namespace py = pybind11;
using namespace cylon;

static std::vector<ops::AggSpec> make_specs(const std::vector<int> &cols, const std::vector<int> &op_ids,
                                            const std::vector<double> &qs, const std::vector<int> &ddofs) {
  CYLON_CHECK(cols.size() == op_ids.size(), Code::Invalid, "aggregate columns and ops differ in length");
  std::vector<ops::AggSpec> specs;
  for (size_t i = 0; i < cols.size(); ++i) {
    ops::AggSpec s{cols[i], op_ids[i]};
    if (i < qs.size()) s.quantile = qs[i];
    if (i < ddofs.size()) s.ddof = ddofs[i];
    specs.push_back(s);
  }
  return specs;
}

void register_extended_ops(py::module &m) {
  auto rel = py::call_guard<py::gil_scoped_release>();

  m.def("index_lookup", &ops::IndexLookup, py::arg("ctx"), py::arg("index"), py::arg("labels"), rel);

  // ---- device self-check behind the radix passes' wave-atomic stable ranking (radix_join.hip)
  m.def("rp_set_ranking", [](int mode) { hip::rp_set_ranking(mode); });
  m.def("partition_digit_bits", [](int bits) { ops::SetPartitionDigitBits(bits); });
  m.def("knob_registry", []() {  // (name without CYLON_, group, effect) of every native knob
    std::vector<std::tuple<std::string, std::string, std::string>> r;
    for (const auto &k : knobs::Registry()) r.emplace_back(k.name, k.group, k.effect);
    return r;
  });
  m.def("rp_take_order_violation", [](const std::string &device) {
    ops::Exec ex{at::Device(device)};
    CYLON_CHECK(ex.gpu, Code::Invalid, "rp_take_order_violation needs a GPU device");
    return hip::rp_take_order_violation(ex.stream);
  });
  m.def("lds_lane_order_violations", [](const std::string &device, int blocks, int rounds) {
    ops::Exec ex{at::Device(device)};
    CYLON_CHECK(ex.gpu, Code::Invalid, "lds_lane_order_violations needs a GPU device");
    return hip::lds_lane_order_violations(blocks, rounds, ex.stream);
  }, py::arg("device") = "cuda:0", py::arg("blocks") = 256, py::arg("rounds") = 4096,
     py::call_guard<py::gil_scoped_release>());

  // ---- validity bitmaps <-> byte masks at the Arrow boundary (bitmap.hip)
  m.def("pack_validity", [](at::Tensor bytes) {
    ops::Exec ex(bytes.device());
    bytes = bytes.contiguous().to(at::kByte);
    const int64_t n = bytes.numel();
    at::Tensor words = at::empty({std::max<int64_t>((n + 63) / 64, 1)}, ex.opts(at::kLong));
    at::Tensor nulls = at::zeros({1}, ex.opts(at::kLong));
    KCALL(ex, pack_validity, bytes.data_ptr<uint8_t>(), n, reinterpret_cast<uint64_t *>(words.data_ptr<int64_t>()),
          nulls.data_ptr<int64_t>());
    return std::make_pair(words.slice(0, 0, (n + 63) / 64), nulls.item<int64_t>());
  }, py::call_guard<py::gil_scoped_release>());
  m.def("unpack_validity", [](at::Tensor bits, int64_t bit_offset, int64_t n) {
    ops::Exec ex(bits.device());
    bits = bits.contiguous();
    at::Tensor out = at::empty({n}, ex.opts(at::kByte));
    if (n) KCALL(ex, unpack_validity, reinterpret_cast<const uint8_t *>(bits.data_ptr()), bit_offset, n,
                 out.data_ptr<uint8_t>());
    return out;
  }, py::call_guard<py::gil_scoped_release>());

  m.def("merge_sorted_runs", &ops::MergeSortedRuns, py::arg("runs"), py::arg("run_rows"), py::arg("col"),
        py::arg("ascending") = true, rel);

  // ---- pinned, pipelined host -> device ingest (io/h2d.cpp); src = host address of nbytes
  m.def("h2d_copy", [](uintptr_t src, int64_t nbytes, at::Tensor dst, int threads) {
    CYLON_CHECK(dst.is_cuda() && dst.is_contiguous(), Code::Invalid, "h2d_copy: contiguous device tensor expected");
    CYLON_CHECK(nbytes >= 0 && nbytes <= (int64_t)(dst.numel() * dst.element_size()), Code::Invalid,
                "h2d_copy: " << nbytes << " bytes do not fit the destination");
    io::H2DStats st;
    io::StagedH2D(reinterpret_cast<const void *>(src), dst.data_ptr(), (size_t)nbytes, dst.device().index(), threads,
                  &st);
    return st.seconds;
  }, py::arg("src"), py::arg("nbytes"), py::arg("dst"), py::arg("threads") = 0,
     py::call_guard<py::gil_scoped_release>());

  // ---- Arrow C Device Data Interface (PyCapsules "arrow_schema" / "arrow_device_array")
  m.def("export_device_table", [](const TablePtr &t) {
    auto *sch = new ArrowSchema();
    auto *arr = new ArrowDeviceArray();
    {
      py::gil_scoped_release nogil;
      io::ExportDeviceTable(t, sch, arr);
    }
    PyObject *cs = PyCapsule_New(sch, "arrow_schema", [](PyObject *o) {
      auto *p = static_cast<ArrowSchema *>(PyCapsule_GetPointer(o, "arrow_schema"));
      if (p && p->release) p->release(p);
      delete p;
    });
    PyObject *ca = PyCapsule_New(arr, "arrow_device_array", [](PyObject *o) {
      auto *p = static_cast<ArrowDeviceArray *>(PyCapsule_GetPointer(o, "arrow_device_array"));
      if (p && p->array.release) p->array.release(&p->array);
      delete p;
    });
    return py::make_tuple(py::reinterpret_steal<py::object>(cs), py::reinterpret_steal<py::object>(ca));
  });
  m.def("import_device_table", [](std::shared_ptr<CylonContext> ctx, py::object schema, py::object array) {
    auto *sch = static_cast<ArrowSchema *>(PyCapsule_GetPointer(schema.ptr(), "arrow_schema"));
    auto *arr = static_cast<ArrowDeviceArray *>(PyCapsule_GetPointer(array.ptr(), "arrow_device_array"));
    CYLON_CHECK(sch && arr, Code::Invalid, "expected 'arrow_schema' and 'arrow_device_array' capsules");
    py::gil_scoped_release nogil;
    return io::ImportDeviceTable(ctx, sch, arr);  // moves the structs (the capsules then only free them)
  });

  // ---- C27 persistent indexes + loc / iloc indexers (cylon/indexing/index.hpp)
  py::enum_<indexing::IndexingSchema>(m, "IndexingSchema")
      .value("RANGE", indexing::IndexingSchema::Range)
      .value("LINEAR", indexing::IndexingSchema::Linear)
      .value("HASH", indexing::IndexingSchema::Hash)
      .value("BINARYTREE", indexing::IndexingSchema::BinaryTree)
      .value("BTREE", indexing::IndexingSchema::BTree);
  py::class_<indexing::BaseIndex, std::shared_ptr<indexing::BaseIndex>>(m, "NativeIndex")
      .def("locations_of", &indexing::BaseIndex::LocationsOf, rel)
      .def("range_of", &indexing::BaseIndex::RangeOf, rel)
      .def("schema", &indexing::BaseIndex::GetSchema)
      .def("size", &indexing::BaseIndex::Size)
      .def("persistent_rows", [](const indexing::BaseIndex &i) {
        auto *s = dynamic_cast<const indexing::SortedIndex *>(&i);
        return s ? s->BuiltRows() : int64_t(0);
      });
  m.def("build_index", &indexing::BuildIndex, py::arg("table"), py::arg("col"), py::arg("schema"), rel);
  m.def("index_from_column", [](std::shared_ptr<CylonContext> ctx, const Column &c, indexing::IndexingSchema schema) {
    return indexing::BuildIndex(Table::Make(ctx, {c}), 0, schema);
  }, rel);
  m.def("table_set_index", [](const TablePtr &t, std::shared_ptr<indexing::BaseIndex> i) { t->SetIndex(i); }, rel);
  m.def("table_get_index", [](const TablePtr &t) { return t->GetIndex(); }, rel);
  m.def("table_reset_index", [](const TablePtr &t) { t->ResetIndex(); }, rel);
  m.def("loc", [](const TablePtr &t, const Column &values, const std::vector<int> &cols, indexing::IndexingSchema s) {
    return indexing::LocIndexer(s).Loc(t, values, cols);
  }, rel);
  m.def("loc_range", [](const TablePtr &t, const Column &start, const Column &end, const std::vector<int> &cols,
                        indexing::IndexingSchema s) { return indexing::LocIndexer(s).LocRange(t, start, end, cols); },
        rel);
  m.def("iloc", [](const TablePtr &t, at::Tensor pos, const std::vector<int> &cols) {
    return indexing::ILocIndexer().ILoc(t, pos, cols);
  }, rel);

  // ---- C25 native CSV I/O
  m.def(
      "read_csv",
      [](const std::shared_ptr<CylonContext> &ctx, const std::vector<std::string> &paths, const std::string &delimiter,
         bool header, bool autogen, const std::vector<std::string> &column_names, int64_t skip_rows,
         bool ignore_empty_lines, const std::vector<std::string> &include_columns,
         const std::vector<std::string> &null_values, const std::vector<std::string> &true_values,
         const std::vector<std::string> &false_values, bool strings_can_be_null, bool quoting,
         const std::string &quote_char, bool double_quote, int threads, bool escaping, const std::string &escape_char,
         bool newlines_in_values, const std::map<std::string, int> &column_types, bool include_missing_columns,
         int64_t block_size, bool concurrent_file_reads) {
        io::CSVReadOptions o;
        o.escaping = escaping;
        if (!escape_char.empty()) o.escape_char = escape_char[0];
        o.newlines_in_values = newlines_in_values;
        for (const auto &kv : column_types) o.column_types.emplace(kv.first, DataType(static_cast<Type>(kv.second)));
        o.include_missing_columns = include_missing_columns;
        o.block_size = (int32_t)std::min<int64_t>(block_size, INT32_MAX);
        o.concurrent_file_reads = concurrent_file_reads;
        o.delimiter = delimiter.empty() ? ',' : delimiter[0];
        o.header = header;
        o.autogenerate_column_names = autogen;
        o.column_names = column_names;
        o.skip_rows = skip_rows;
        o.ignore_empty_lines = ignore_empty_lines;
        o.include_columns = include_columns;
        o.null_values = null_values;
        if (!true_values.empty()) o.true_values = true_values;
        if (!false_values.empty()) o.false_values = false_values;
        o.strings_can_be_null = strings_can_be_null;
        o.quoting = quoting;
        o.quote_char = quote_char.empty() ? '"' : quote_char[0];
        o.double_quote = double_quote;
        o.threads = threads;
        return io::ReadCSVs(ctx, paths, o);
      },
      py::arg("ctx"), py::arg("paths"), py::arg("delimiter") = ",", py::arg("header") = true,
      py::arg("autogenerate_column_names") = false, py::arg("column_names") = std::vector<std::string>{},
      py::arg("skip_rows") = 0, py::arg("ignore_empty_lines") = true,
      py::arg("include_columns") = std::vector<std::string>{}, py::arg("null_values") = std::vector<std::string>{},
      py::arg("true_values") = std::vector<std::string>{}, py::arg("false_values") = std::vector<std::string>{},
      py::arg("strings_can_be_null") = false, py::arg("quoting") = true, py::arg("quote_char") = "\"",
      py::arg("double_quote") = true, py::arg("threads") = 0, py::arg("escaping") = false,
      py::arg("escape_char") = "\\", py::arg("newlines_in_values") = false,
      py::arg("column_types") = std::map<std::string, int>{}, py::arg("include_missing_columns") = false,
      py::arg("block_size") = int64_t(1) << 20, py::arg("concurrent_file_reads") = true, rel);
  m.def(
      "write_csv",
      [](const TablePtr &t, const std::string &path, const std::string &delimiter,
         const std::vector<std::string> &names) {
        io::CSVWriteOptions o;
        o.delimiter = delimiter.empty() ? ',' : delimiter[0];
        o.column_names = names;
        io::WriteCSV(t, path, o);
      },
      py::arg("table"), py::arg("path"), py::arg("delimiter") = ",",
      py::arg("column_names") = std::vector<std::string>{}, rel);

  // ---- C25 native Parquet I/O (Arrow / Parquet C++ from pyarrow's libraries)
  m.def(
      "read_parquet",
      [](const std::shared_ptr<CylonContext> &ctx, const std::vector<std::string> &paths,
         const std::vector<std::string> &columns, bool use_threads, bool concurrent_file_reads) {
        io::ParquetOptions o;
        o.columns = columns;
        o.use_threads = use_threads;
        o.concurrent_file_reads = concurrent_file_reads;
        return io::ReadParquets(ctx, paths, o);
      },
      py::arg("ctx"), py::arg("paths"), py::arg("columns") = std::vector<std::string>{},
      py::arg("use_threads") = true, py::arg("concurrent_file_reads") = true, rel);
  m.def(
      "write_parquet",
      [](const TablePtr &t, const std::string &path, const std::string &compression, int64_t chunk_size) {
        io::ParquetOptions o;
        o.compression = compression;
        o.chunk_size = chunk_size;
        io::WriteParquet(t, path, o);
      },
      py::arg("table"), py::arg("path"), py::arg("compression") = "snappy", py::arg("chunk_size") = 1 << 20, rel);

  py::enum_<AggOp>(m, "AggregationOp")
      .value("SUM", AGG_SUM).value("MIN", AGG_MIN).value("MAX", AGG_MAX).value("COUNT", AGG_COUNT)
      .value("MEAN", AGG_MEAN).value("VAR", AGG_VAR).value("NUNIQUE", AGG_NUNIQUE)
      .value("QUANTILE", AGG_QUANTILE).value("STDDEV", AGG_STDDEV);

  m.def("union", &ops::Union, rel);
  m.def("subtract", &ops::Subtract, rel);
  m.def("intersect", &ops::Intersect, rel);
  m.def("distributed_union", &ops::DistributedUnion, rel);
  m.def("distributed_subtract", &ops::DistributedSubtract, rel);
  m.def("distributed_intersect", &ops::DistributedIntersect, rel);
  m.def("unique", &ops::Unique, rel);
  m.def("distributed_unique", &ops::DistributedUnique, rel);

  m.def("group_ids", [](const TablePtr &t, const std::vector<int> &cols, bool presorted) {
    auto g = ops::GroupIds(t, cols, presorted);
    return std::make_tuple(g.gid, g.ngroups, g.first_rows);
  }, py::call_guard<py::gil_scoped_release>());

  auto groupby_fn = [](TablePtr (*fn)(const TablePtr &, const std::vector<int> &, const std::vector<ops::AggSpec> &)) {
    return [fn](const TablePtr &t, const std::vector<int> &keys, const std::vector<int> &cols,
                const std::vector<int> &op_ids, const std::vector<double> &qs, const std::vector<int> &ddofs) {
      return fn(t, keys, make_specs(cols, op_ids, qs, ddofs));
    };
  };
  m.def("hash_groupby", groupby_fn(&ops::HashGroupBy), py::call_guard<py::gil_scoped_release>());
  m.def("pipeline_groupby", groupby_fn(&ops::PipelineGroupBy), py::call_guard<py::gil_scoped_release>());
  m.def("distributed_hash_groupby", groupby_fn(&ops::DistributedHashGroupBy), py::call_guard<py::gil_scoped_release>());
  m.def("distributed_pipeline_groupby", groupby_fn(&ops::DistributedPipelineGroupBy), py::call_guard<py::gil_scoped_release>());

  m.def("aggregate", &ops::Aggregate, py::arg("table"), py::arg("col"), py::arg("op"), py::arg("quantile") = 0.5,
        py::arg("ddof") = 1, py::arg("distributed") = true, rel);

  m.def(
      "distributed_sort",
      [](const TablePtr &t, const std::vector<int> &cols, const std::vector<bool> &asc, uint32_t num_bins,
         uint64_t num_samples) {
        SortOptions o;
        o.num_bins = num_bins;
        o.num_samples = num_samples;
        return ops::DistributedSort(t, cols, asc, o);
      },
      rel);
  // ---- streaming op graph (C24) ------------------------------------------
  m.def(
      "dis_join_op",
      [](std::shared_ptr<CylonContext> ctx, const std::vector<TablePtr> &lefts, const std::vector<TablePtr> &rights,
         const std::string &type, const std::string &algo, const std::vector<int> &lc, const std::vector<int> &rc,
         const std::string &lp, const std::string &rp, int num_splits) {
        using namespace join::config;
        const JoinType jt = type == "left" ? LEFT : type == "right" ? RIGHT : type == "outer" ? FULL_OUTER : INNER;
        const JoinAlgorithm ja = algo == "hash" ? HASH : SORT;
        graph::DisJoinOpConfig cfg{num_splits, JoinConfig(jt, lc, rc, ja, lp, rp)};
        std::vector<TablePtr> out;
        graph::DisJoinOP op(ctx, 0, [&out](int, const TablePtr &t) { out.push_back(t); }, cfg);
        for (const auto &t : lefts) op.InsertTable(graph::DisJoinOP::kLeftTag, t);
        for (const auto &t : rights) op.InsertTable(graph::DisJoinOP::kRightTag, t);
        op.WaitForCompletion();
        return out;
      },
      rel);
  m.def(
      "dis_union_op",
      [](std::shared_ptr<CylonContext> ctx, const std::vector<TablePtr> &tables) {
        std::vector<TablePtr> out;
        graph::DisUnionOp op(ctx, 0, [&out](int, const TablePtr &t) { out.push_back(t); });
        for (const auto &t : tables) op.InsertTable(0, t);
        op.WaitForCompletion();
        return out;
      },
      rel);

  // ---- string-ID registry (reference table_api.hpp) ----------------------------
  m.def("registry_put", &PutTable, py::call_guard<py::gil_scoped_release>());
  m.def("registry_get", &GetTable, py::call_guard<py::gil_scoped_release>());
  m.def("registry_remove", &RemoveTable, py::call_guard<py::gil_scoped_release>());
  m.def("registry_list", &ListTables, py::call_guard<py::gil_scoped_release>());
  m.def("registry_row_count", &RowCount, py::call_guard<py::gil_scoped_release>());
  m.def("registry_column_count", &ColumnCount, py::call_guard<py::gil_scoped_release>());
  m.def(
      "registry_join",
      [](const std::string &l, const std::string &r, const std::string &type, const std::string &algo,
         const std::vector<int> &lc, const std::vector<int> &rc, const std::string &dest, bool distributed) {
        using namespace join::config;
        const JoinType jt = type == "left" ? LEFT : type == "right" ? RIGHT : type == "outer" ? FULL_OUTER : INNER;
        JoinConfig cfg(jt, lc, rc, algo == "hash" ? HASH : SORT);
        Status s = distributed ? DistributedJoinTables(l, r, cfg, dest) : JoinTables(l, r, cfg, dest);
        return std::make_pair(s.get_code(), s.get_msg());  // converted after the GIL is re-acquired
      },
      rel);
  m.def(
      "registry_union",
      [](const std::string &a, const std::string &b, const std::string &dest, bool distributed) {
        Status s = UnionTables(a, b, dest, distributed);
        return std::make_pair(s.get_code(), s.get_msg());  // converted after the GIL is re-acquired
      },
      rel);

  // ---- all-to-all with the reference's insert/finish/isComplete protocol ----------
  struct A2AHandle {
    std::vector<std::tuple<int, TablePtr, int>> received;
    std::unique_ptr<TableAllToAll> impl;
  };
  py::class_<A2AHandle, std::shared_ptr<A2AHandle>>(m, "TableAllToAll")
      .def(py::init([](std::shared_ptr<CylonContext> ctx) {
        auto h = std::make_shared<A2AHandle>();
        A2AHandle *raw = h.get();
        h->impl = std::make_unique<TableAllToAll>(ctx, [raw](int src, const TablePtr &t, int ref) {
          raw->received.emplace_back(src, t, ref);
          return true;
        });
        return h;
      }), py::call_guard<py::gil_scoped_release>())
      .def("insert", [](A2AHandle &h, const TablePtr &t, int target, int ref) { return h.impl->insert(t, target, ref); },
           py::arg("table"), py::arg("target"), py::arg("reference") = 0, py::call_guard<py::gil_scoped_release>())
      .def("finish", [](A2AHandle &h) { h.impl->finish(); }, py::call_guard<py::gil_scoped_release>())
      .def("is_complete", [](A2AHandle &h) { return h.impl->isComplete(); }, rel)
      .def("close", [](A2AHandle &h) { h.impl->close(); }, py::call_guard<py::gil_scoped_release>())
      .def("received", [](A2AHandle &h) { return h.received; }, py::call_guard<py::gil_scoped_release>());

  m.def("map_to_sort_partitions", &ops::MapToSortPartitions, rel);
  m.def("partition_reorder", &ops::PartitionReorder, rel);
  m.def("shuffle_partition", &ops::ShufflePartition, rel);
  m.def("all_to_all_table", &ops::AllToAllTable, rel);
}
