// Python binding of the native engine (module cylon_amd._C).
// Reference: python/pycylon/*.pyx (Cython binding of libcylon) and
// python/pycylon/api/lib.pyx (C-API wrap/unwrap).  Here pybind11 over the
// C++ core; the pandas-like frontends (Table, DataFrame) are Python on top.
#include <torch/extension.h>
#include <torch/csrc/distributed/c10d/ProcessGroup.hpp>
#include <torch/csrc/utils/pybind.h>

#include "cylon/net/async_delay_communicator.hpp"
#include "cylon/ctx/cylon_context.hpp"
#include "cylon/net/channel.hpp"
#include "cylon/net/communicator.hpp"
#include "cylon/ops/api_ext.hpp"
#include "cylon/table.hpp"
#include "cylon/trace.hpp"

namespace py = pybind11;
using namespace cylon;

namespace {

// Python subclasses of the channel callbacks (reference net/channel.hpp callbacks)
class PyRecvCb : public net::ChannelReceiveCallback {
 public:
  void receivedHeader(int source, int finished, const std::vector<int32_t> &header) override {
    PYBIND11_OVERRIDE_PURE_NAME(void, net::ChannelReceiveCallback, "received_header", receivedHeader, source,
                                finished, header);
  }
  void receivedData(int source, const at::Tensor &buffer) override {
    PYBIND11_OVERRIDE_PURE_NAME(void, net::ChannelReceiveCallback, "received_data", receivedData, source, buffer);
  }
};

class PySendCb : public net::ChannelSendCallback {
 public:
  void sendComplete(const std::shared_ptr<net::TxRequest> &req) override {
    PYBIND11_OVERRIDE_PURE_NAME(void, net::ChannelSendCallback, "send_complete", sendComplete, req);
  }
  void sendFinishComplete(const std::shared_ptr<net::TxRequest> &req) override {
    PYBIND11_OVERRIDE_PURE_NAME(void, net::ChannelSendCallback, "send_finish_complete", sendFinishComplete, req);
  }
};

at::Device parse_device(const std::string &s) { return at::Device(s); }

join::config::JoinType parse_join_type(const std::string &t) {
  if (t == "inner") return join::config::INNER;
  if (t == "left") return join::config::LEFT;
  if (t == "right") return join::config::RIGHT;
  if (t == "outer" || t == "full_outer" || t == "fullouter") return join::config::FULL_OUTER;
  CYLON_THROW(Code::Invalid, "unsupported join type '" << t << "'");
}

join::config::JoinAlgorithm parse_join_algo(const std::string &a) {
  if (a == "hash") return join::config::HASH;
  if (a == "sort") return join::config::SORT;
  CYLON_THROW(Code::Invalid, "unsupported join algorithm '" << a << "'");
}

join::config::JoinConfig make_jc(const std::string &type, const std::string &algo, const std::vector<int> &l,
                                 const std::vector<int> &r, const std::string &lp, const std::string &rp) {
  return join::config::JoinConfig(parse_join_type(type), l, r, parse_join_algo(algo), lp, rp);
}

}  // namespace

PYBIND11_MODULE(_C, m) {
  // release the GIL inside every blocking transport wait (net::EnterBlocking)
  net::SetBlockingHook([]() -> std::unique_ptr<net::BlockingRegion> {
    struct GilRelease : net::BlockingRegion {
      PyThreadState *st = nullptr;
      GilRelease() {
        // holds the GIL iff it has a current thread state (PyGILState_Check is not reliable
        // after pybind11's gil_scoped_release)
        if (Py_IsInitialized() && _PyThreadState_UncheckedGet() != nullptr) st = PyEval_SaveThread();
      }
      ~GilRelease() override {
        if (st) PyEval_RestoreThread(st);
      }
    };
    return std::make_unique<GilRelease>();
  });

  m.doc() = "cylon_amd native engine: MI355X HIP kernels + RCCL shuffle";

  static py::exception<CylonError> exc(m, "CylonError", PyExc_RuntimeError);
  py::register_exception_translator([](std::exception_ptr p) {
    try {
      if (p) std::rethrow_exception(p);
    } catch (const CylonError &e) {
      PyErr_SetObject(exc.ptr(), Py_BuildValue("(si)", e.what(), e.code()));
    }
  });

  py::enum_<Type>(m, "Type")
      .value("BOOL", Type::BOOL).value("UINT8", Type::UINT8).value("INT8", Type::INT8)
      .value("UINT16", Type::UINT16).value("INT16", Type::INT16).value("UINT32", Type::UINT32)
      .value("INT32", Type::INT32).value("UINT64", Type::UINT64).value("INT64", Type::INT64)
      .value("HALF_FLOAT", Type::HALF_FLOAT).value("FLOAT", Type::FLOAT).value("DOUBLE", Type::DOUBLE)
      .value("STRING", Type::STRING).value("BINARY", Type::BINARY)
      .value("FIXED_SIZE_BINARY", Type::FIXED_SIZE_BINARY).value("DATE32", Type::DATE32)
      .value("DATE64", Type::DATE64).value("TIMESTAMP", Type::TIMESTAMP).value("TIME32", Type::TIME32)
      .value("TIME64", Type::TIME64).value("INTERVAL", Type::INTERVAL).value("DECIMAL", Type::DECIMAL)
      .value("LIST", Type::LIST).value("EXTENSION", Type::EXTENSION)
      .value("FIXED_SIZE_LIST", Type::FIXED_SIZE_LIST).value("DURATION", Type::DURATION);

  py::enum_<Layout>(m, "Layout").value("FIXED_WIDTH", Layout::FIXED_WIDTH).value("VARIABLE_WIDTH", Layout::VARIABLE_WIDTH);

  py::class_<DataType>(m, "DataType")
      .def(py::init<>(), py::call_guard<py::gil_scoped_release>())
      .def(py::init<Type>(), py::call_guard<py::gil_scoped_release>())
      .def(py::init<Type, int32_t>(), py::call_guard<py::gil_scoped_release>())
      .def_readwrite("type", &DataType::type)
      .def_readwrite("byte_width", &DataType::byte_width)
      .def_property("unit", [](const DataType &d) { return static_cast<int>(d.unit); },
                    [](DataType &d, int u) { d.unit = static_cast<TimeUnit>(u); })
      .def_readwrite("timezone", &DataType::timezone)
      .def_readwrite("value_type", &DataType::value_type)
      .def_readwrite("list_size", &DataType::list_size)
      .def_readwrite("precision", &DataType::precision)
      .def_readwrite("scale", &DataType::scale)
      .def("value_width", &DataType::value_width)
      .def_static("list_of", &DataType::List)
      .def_static("fixed_size_list_of", &DataType::FixedSizeList)
      .def("width", &DataType::width, py::call_guard<py::gil_scoped_release>())
      .def("layout", &DataType::layout, py::call_guard<py::gil_scoped_release>())
      .def("is_numeric", &DataType::is_numeric, py::call_guard<py::gil_scoped_release>())
      .def("__eq__", [](const DataType &a, const DataType &b) { return a == b; }, py::call_guard<py::gil_scoped_release>())
      .def("__repr__", &DataType::ToString, py::call_guard<py::gil_scoped_release>())
      .def("__str__", &DataType::ToString, py::call_guard<py::gil_scoped_release>());

  py::class_<Column>(m, "Column")
      .def(py::init([](const std::string &name, const DataType &t, int64_t length, at::Tensor data,
                       c10::optional<at::Tensor> offsets, c10::optional<at::Tensor> validity) {
             return Column(name, t, length, data, offsets ? *offsets : at::Tensor(), validity ? *validity : at::Tensor());
           }),
           py::arg("name"), py::arg("type"), py::arg("length"), py::arg("data"), py::arg("offsets") = py::none(),
           py::arg("validity") = py::none())
      .def_readwrite("name", &Column::name)
      .def_readonly("type", &Column::type)
      .def_readonly("length", &Column::length)
      .def_property_readonly("data", [](const Column &c) { return c.data; })
      .def_property_readonly("offsets", [](const Column &c) -> py::object {
        return c.offsets.defined() ? py::cast(c.offsets) : py::none();
      })
      .def_property_readonly("validity", [](const Column &c) -> py::object {
        return c.validity.defined() ? py::cast(c.validity) : py::none();
      })
      .def("null_count", &Column::null_count, py::call_guard<py::gil_scoped_release>())
      .def("nbytes", &Column::nbytes, py::call_guard<py::gil_scoped_release>())
      .def("to", [](const Column &c, const std::string &d) { return c.to(parse_device(d)); }, py::call_guard<py::gil_scoped_release>())
      .def("slice", &Column::slice, py::call_guard<py::gil_scoped_release>())
      .def("with_name", &Column::with_name, py::call_guard<py::gil_scoped_release>());

  py::enum_<net::CommType>(m, "CommType")
      .value("LOCAL", net::CommType::LOCAL).value("MPI", net::CommType::MPI).value("TCP", net::CommType::TCP)
      .value("UCX", net::CommType::UCX).value("RCCL", net::CommType::RCCL).value("GLOO", net::CommType::GLOO);

  // ---- P8 C-API: opaque capsules for third-party native code (reference python/pycylon/api/lib.pyx)
  m.def("table_to_capsule", [](const TablePtr &t) {
    return py::capsule(new TablePtr(t), "cylon_amd.Table", [](PyObject *o) {
      delete static_cast<TablePtr *>(PyCapsule_GetPointer(o, "cylon_amd.Table"));
    });
  });
  m.def("table_from_capsule", [](py::capsule c) {
    CYLON_CHECK(std::string(c.name()) == "cylon_amd.Table", Code::Invalid, "not a cylon_amd.Table capsule");
    return *static_cast<TablePtr *>(c.get_pointer());
  });
  m.def("context_to_capsule", [](const std::shared_ptr<CylonContext> &ctx) {
    return py::capsule(new std::shared_ptr<CylonContext>(ctx), "cylon_amd.Context", [](PyObject *o) {
      delete static_cast<std::shared_ptr<CylonContext> *>(PyCapsule_GetPointer(o, "cylon_amd.Context"));
    });
  });
  m.def("context_from_capsule", [](py::capsule c) {
    CYLON_CHECK(std::string(c.name()) == "cylon_amd.Context", Code::Invalid, "not a cylon_amd.Context capsule");
    return *static_cast<std::shared_ptr<CylonContext> *>(c.get_pointer());
  });

  py::class_<net::TxRequest, std::shared_ptr<net::TxRequest>>(m, "TxRequest")
      .def(py::init<>(), py::call_guard<py::gil_scoped_release>())
      .def(py::init([](int target, py::object buffer, std::vector<int32_t> header) {
             at::Tensor b = buffer.is_none() ? at::Tensor() : buffer.cast<at::Tensor>();
             return std::make_shared<net::TxRequest>(target, b, header);
           }),
           py::arg("target"), py::arg("buffer") = py::none(), py::arg("header") = std::vector<int32_t>{})
      .def_readwrite("target", &net::TxRequest::target)
      .def_readwrite("header", &net::TxRequest::header)
      .def_property(
          "buffer", [](const net::TxRequest &r) -> py::object {
            return r.buffer.defined() ? py::cast(r.buffer) : py::none();
          },
          [](net::TxRequest &r, at::Tensor b) { r.buffer = b; });
  py::class_<net::ChannelReceiveCallback, PyRecvCb>(m, "ChannelReceiveCallback").def(py::init<>(), py::call_guard<py::gil_scoped_release>());
  py::class_<net::ChannelSendCallback, PySendCb>(m, "ChannelSendCallback").def(py::init<>(), py::call_guard<py::gil_scoped_release>());
  py::class_<net::Channel, std::shared_ptr<net::Channel>>(m, "Channel")
      .def(py::init([](const std::shared_ptr<CylonContext> &ctx) {
        return std::make_shared<net::Channel>(ctx->GetCommunicator(), ctx->GetDevice());
      }), py::call_guard<py::gil_scoped_release>())
      .def("init", &net::Channel::init, py::arg("edge"), py::arg("receives"), py::arg("send_ids"),
           py::arg("receive_callback"), py::arg("send_callback"), py::keep_alive<1, 5>(), py::keep_alive<1, 6>(), py::call_guard<py::gil_scoped_release>())
      .def("send", &net::Channel::send, py::call_guard<py::gil_scoped_release>())
      .def("send_fin", &net::Channel::sendFin, py::call_guard<py::gil_scoped_release>())
      .def("progress_sends", &net::Channel::progressSends, py::call_guard<py::gil_scoped_release>())
      .def("progress_receives", &net::Channel::progressReceives, py::call_guard<py::gil_scoped_release>())
      .def("is_complete", &net::Channel::isComplete, py::call_guard<py::gil_scoped_release>())
      .def("close", &net::Channel::close, py::call_guard<py::gil_scoped_release>());

  py::class_<MemoryPool, std::shared_ptr<MemoryPool>>(m, "MemoryPool")
      .def("bytes_allocated", &MemoryPool::bytes_allocated, py::call_guard<py::gil_scoped_release>())
      .def("max_memory", &MemoryPool::max_memory, py::call_guard<py::gil_scoped_release>())
      .def("backend_name", &MemoryPool::backend_name, py::call_guard<py::gil_scoped_release>())
      .def("device", [](const MemoryPool &p) { return p.device().str(); }, py::call_guard<py::gil_scoped_release>())
      .def(
          "empty",
          [](const std::shared_ptr<MemoryPool> &p, std::vector<int64_t> shape, const std::string &dtype) {
            static const std::map<std::string, at::ScalarType> m{
                {"int8", at::kChar},  {"uint8", at::kByte},   {"int16", at::kShort},   {"int32", at::kInt},
                {"int64", at::kLong}, {"float16", at::kHalf}, {"float32", at::kFloat}, {"float64", at::kDouble},
                {"bool", at::kBool}};
            auto it = m.find(dtype);
            CYLON_CHECK(it != m.end(), Code::Invalid, "unsupported dtype " << dtype);
            return EmptyFromPool(p, shape, it->second);
          },
          py::arg("shape"), py::arg("dtype"), "tensor whose storage is allocated from this pool", py::call_guard<py::gil_scoped_release>());
  m.def("host_memory_pool", []() { return std::shared_ptr<MemoryPool>(std::make_shared<HostMemoryPool>()); }, py::call_guard<py::gil_scoped_release>());
  m.def("device_memory_pool", [](const std::string &dev) {
    return std::shared_ptr<MemoryPool>(std::make_shared<DeviceMemoryPool>(parse_device(dev)));
  }, py::call_guard<py::gil_scoped_release>());

  py::class_<CylonContext, std::shared_ptr<CylonContext>>(m, "Context")
      .def("memory_pool", &CylonContext::GetMemoryPool, py::call_guard<py::gil_scoped_release>())
      .def("set_memory_pool", &CylonContext::SetMemoryPool, py::call_guard<py::gil_scoped_release>())
      .def_static("init_local", [](const std::string &dev) { return CylonContext::Init(parse_device(dev)); },
                  py::arg("device") = "cpu", py::call_guard<py::gil_scoped_release>())
      .def_static("init_distributed",
                  [](c10::intrusive_ptr<c10d::ProcessGroup> pg, const std::string &backend, const std::string &dev) {
                    const auto ct = backend == "nccl" || backend == "rccl" ? net::CommType::RCCL : net::CommType::GLOO;
                    const at::Device device = parse_device(dev);
                    const at::Device comm_device = ct == net::CommType::RCCL ? device : at::Device(at::kCPU);
                    auto comm = std::make_shared<net::ProcessGroupCommunicator>(pg, ct, comm_device);
                    comm->WarmUp();
                    return CylonContext::InitDistributed(comm, device);
                  }, py::call_guard<py::gil_scoped_release>())
      .def_static("init_native",
                  [](const std::string &comm, int rank, int world, const std::string &dev, double timeout_s) {
                    net::CommConfig cfg;
                    cfg.type = comm == "tcp" || comm == "gloo" ? net::CommType::TCP
                               : comm == "mpi"                 ? net::CommType::MPI
                                                               : net::CommType::RCCL;
                    cfg.rank = rank;
                    cfg.world_size = world;
                    cfg.device = dev;
                    cfg.timeout_s = timeout_s;
                    return CylonContext::InitDistributed(cfg);
                  },
                  py::arg("comm"), py::arg("rank") = -1, py::arg("world_size") = -1, py::arg("device") = "",
                  py::arg("timeout_s") = 1800.0, py::call_guard<py::gil_scoped_release>())
      .def("get_rank", &CylonContext::GetRank, py::call_guard<py::gil_scoped_release>())
      .def("get_world_size", &CylonContext::GetWorldSize, py::call_guard<py::gil_scoped_release>())
      .def("get_neighbours", &CylonContext::GetNeighbours, py::call_guard<py::gil_scoped_release>())
      .def("get_next_sequence", &CylonContext::GetNextSequence, py::call_guard<py::gil_scoped_release>())
      .def("is_distributed", &CylonContext::IsDistributed, py::call_guard<py::gil_scoped_release>())
      .def("get_comm_type", &CylonContext::GetCommType, py::call_guard<py::gil_scoped_release>())
      .def("barrier", &CylonContext::Barrier, py::call_guard<py::gil_scoped_release>())
      .def("finalize", &CylonContext::Finalize, py::call_guard<py::gil_scoped_release>())
      .def("add_config", &CylonContext::AddConfig, py::call_guard<py::gil_scoped_release>())
      .def("get_config", &CylonContext::GetConfig, py::arg("key"), py::arg("default") = "", py::call_guard<py::gil_scoped_release>())
      .def("get_configs", &CylonContext::GetConfigs, py::call_guard<py::gil_scoped_release>())
      .def("device", [](const CylonContext &c) { return c.GetDevice().str(); }, py::call_guard<py::gil_scoped_release>())
      .def("inject_faults",
           [](CylonContext &c, int64_t fail_at_call) {
             c.setCommunicator(std::make_shared<net::FaultInjectionCommunicator>(c.GetCommunicator(), fail_at_call));
           }, py::call_guard<py::gil_scoped_release>())
      .def("use_async_delay_transport",
           [](CylonContext &c, double delay_us) {
             c.setCommunicator(std::make_shared<net::AsyncDelayCommunicator>(c.GetCommunicator(), delay_us));
           }, py::call_guard<py::gil_scoped_release>())
      .def("async_transport_stats",
           [](CylonContext &c) {
             auto a = std::dynamic_pointer_cast<net::AsyncDelayCommunicator>(c.GetCommunicator());
             CYLON_CHECK(a != nullptr, Code::Invalid, "context does not use the async delay transport");
             return std::make_pair(a->posted(), a->observed_in_flight());
           }, py::call_guard<py::gil_scoped_release>())
      .def("bytes_allocated", &CylonContext::BytesAllocated, py::call_guard<py::gil_scoped_release>())
      .def("max_memory", &CylonContext::MaxMemory, py::call_guard<py::gil_scoped_release>())
      .def("allreduce", [](CylonContext &c, at::Tensor t, int op) {
        c.GetCommunicator()->AllReduce(t, static_cast<net::ReduceOp>(op));
        return t;
      }, py::call_guard<py::gil_scoped_release>())
      .def("allgather", [](CylonContext &c, at::Tensor t) { return c.GetCommunicator()->AllGather(t); }, py::call_guard<py::gil_scoped_release>())
      .def("allgatherv", [](CylonContext &c, at::Tensor t) { return c.GetCommunicator()->AllGatherV(t); }, py::call_guard<py::gil_scoped_release>())
      .def("broadcast", [](CylonContext &c, at::Tensor t, int root) {
        c.GetCommunicator()->Broadcast(t, root);
        return t;
      }, py::call_guard<py::gil_scoped_release>())
      .def("alltoallv", [](CylonContext &c, at::Tensor t, std::vector<int64_t> sc) {
        auto comm = c.GetCommunicator();
        auto rc = comm->ExchangeCounts(sc);
        return comm->AllToAllV(t, sc, rc);
      }, py::call_guard<py::gil_scoped_release>());

  py::class_<Table, std::shared_ptr<Table>>(m, "Table")
      .def(py::init([](std::shared_ptr<CylonContext> ctx, std::vector<Column> cols) {
        return std::make_shared<Table>(std::move(ctx), std::move(cols));
      }), py::call_guard<py::gil_scoped_release>())
      .def("rows", &Table::Rows, py::call_guard<py::gil_scoped_release>())
      .def("num_columns", &Table::Columns, py::call_guard<py::gil_scoped_release>())
      .def("column_names", &Table::ColumnNames, py::call_guard<py::gil_scoped_release>())
      .def("column", &Table::column, py::call_guard<py::gil_scoped_release>())
      .def("columns", &Table::columns, py::call_guard<py::gil_scoped_release>())
      .def("column_index", &Table::ColumnIndex, py::call_guard<py::gil_scoped_release>())
      .def("context", &Table::GetContext, py::call_guard<py::gil_scoped_release>())
      .def("device", [](const Table &t) { return t.device().str(); }, py::call_guard<py::gil_scoped_release>())
      .def("retain_memory", &Table::retainMemory, py::call_guard<py::gil_scoped_release>())
      .def("is_retain", &Table::IsRetain, py::call_guard<py::gil_scoped_release>())
      .def("clear", &Table::Clear, py::call_guard<py::gil_scoped_release>())
      .def("nbytes", &Table::nbytes, py::call_guard<py::gil_scoped_release>())
      .def("to", [](const Table &t, const std::string &d) { return t.to(parse_device(d)); }, py::call_guard<py::gil_scoped_release>());

  // ---- operators (GIL released: kernels + collectives) -----------------------
  auto rel = py::call_guard<py::gil_scoped_release>();
  m.def("gather", &ops::Gather, rel);
  m.def("gather_nullable", &ops::GatherNullable, rel);
  m.def("select_var", &ops::SelectVar, py::arg("a"), py::arg("b"), py::arg("cond"), rel);
  m.def("cast_string_to_number", &ops::CastStringToNumber, py::arg("col"), py::arg("target"), rel);
  m.def("cast_integer_to_string", &ops::CastIntegerToString, py::arg("col"), py::arg("target"), rel);
  m.def("project", &ops::Project, rel);
  m.def("merge", &ops::Merge, rel);
  m.def("slice", &ops::Slice, rel);
  m.def("filter_by_mask", &ops::FilterByMask, rel);
  m.def("mask_to_indices", &ops::MaskToIndices, py::arg("mask"), py::arg("invert") = false, rel);
  m.def("map_to_hash_partitions", &ops::MapToHashPartitions, rel);
  m.def("split", &ops::Split, rel);
  m.def("hash_partition", &ops::HashPartition, rel);
  m.def("shuffle", &ops::Shuffle, rel);
  m.def("sort_indices", &ops::SortIndices, rel);
  m.def("sort", &ops::Sort, rel);
  m.def(
      "join",
      [](const TablePtr &l, const TablePtr &r, const std::string &type, const std::string &algo,
         const std::vector<int> &lc, const std::vector<int> &rc, const std::string &lp, const std::string &rp) {
        return ops::Join(l, r, make_jc(type, algo, lc, rc, lp, rp));
      },
      rel);
  m.def(
      "distributed_join",
      [](const TablePtr &l, const TablePtr &r, const std::string &type, const std::string &algo,
         const std::vector<int> &lc, const std::vector<int> &rc, const std::string &lp, const std::string &rp) {
        return ops::DistributedJoin(l, r, make_jc(type, algo, lc, rc, lp, rp));
      },
      rel);
  m.def(
      "join_indices",
      [](const TablePtr &l, const TablePtr &r, const std::string &type, const std::string &algo,
         const std::vector<int> &lc, const std::vector<int> &rc) {
        return ops::JoinIndices(l, r, make_jc(type, algo, lc, rc, "", ""));
      },
      rel);

  // ---- tracing / metrics -----------------------------------------------------
  m.def("trace_enable", &trace::set_enabled, py::call_guard<py::gil_scoped_release>());
  m.def("trace_enabled", &trace::enabled, py::call_guard<py::gil_scoped_release>());
  m.def("trace_phases", [] {
    std::map<std::string, std::pair<double, int64_t>> out;
    for (auto &kv : trace::phases()) out[kv.first] = {kv.second.total_ms, kv.second.calls};
    return out;
  }, py::call_guard<py::gil_scoped_release>());
  m.def("trace_counters", &trace::counters, py::call_guard<py::gil_scoped_release>());
  m.def("trace_reset", &trace::reset, py::call_guard<py::gil_scoped_release>());
  m.def("log", &trace::log, py::call_guard<py::gil_scoped_release>());

  register_extended_ops(m);
}
