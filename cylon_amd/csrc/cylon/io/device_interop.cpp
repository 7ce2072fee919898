// Arrow C Device Data Interface export / import (see device_interop.hpp).
#include "device_interop.hpp"

#include <hip/hip_runtime.h>

#include <ATen/hip/HIPContext.h>
#include <cstring>
#include <cstdio>
#include <map>

#include "../ops/util.hpp"

#define HIP_EVENT_CHECK(expr)                                                                        \
  do {                                                                                               \
    hipError_t _e = (expr);                                                                          \
    CYLON_CHECK(_e == hipSuccess, Code::ExecutionError, #expr << ": " << hipGetErrorString(_e));     \
  } while (0)

namespace cylon {
namespace io {

using ops::Exec;
using ops::ptr;

namespace {

char unit_char(TimeUnit u) {
  switch (u) {
    case TimeUnit::SECOND: return 's';
    case TimeUnit::MILLI: return 'm';
    case TimeUnit::MICRO: return 'u';
    case TimeUnit::NANO: return 'n';
  }
  return 'm';
}

TimeUnit unit_of_char(char c) {
  switch (c) {
    case 's': return TimeUnit::SECOND;
    case 'm': return TimeUnit::MILLI;
    case 'u': return TimeUnit::MICRO;
    default: return TimeUnit::NANO;
  }
}

std::string format_of(const DataType &t) {
  switch (t.type) {
    case Type::BOOL: return "b";
    case Type::UINT8: return "C";
    case Type::INT8: return "c";
    case Type::UINT16: return "S";
    case Type::INT16: return "s";
    case Type::UINT32: return "I";
    case Type::INT32: return "i";
    case Type::UINT64: return "L";
    case Type::INT64: return "l";
    case Type::HALF_FLOAT: return "e";
    case Type::FLOAT: return "f";
    case Type::DOUBLE: return "g";
    case Type::STRING: return "U";
    case Type::BINARY: return "Z";
    case Type::FIXED_SIZE_BINARY: return "w:" + std::to_string(t.byte_width);
    case Type::DECIMAL:  // "d:precision,scale[,bitwidth]"
      return "d:" + std::to_string(t.precision ? t.precision : (t.byte_width == 32 ? 76 : 38)) + "," +
             std::to_string(t.scale) + (t.byte_width == 32 ? ",256" : "");
    case Type::DATE32: return "tdD";
    case Type::DATE64: return "tdm";
    case Type::TIMESTAMP: return std::string("ts") + unit_char(t.unit) + ":" + t.timezone;
    case Type::TIME32: return std::string("tt") + unit_char(t.unit);
    case Type::TIME64: return std::string("tt") + unit_char(t.unit);
    case Type::DURATION: return std::string("tD") + unit_char(t.unit);
    case Type::LIST: return "+L";
    case Type::FIXED_SIZE_LIST: return "+w:" + std::to_string(t.list_size);
    default: CYLON_THROW(Code::NotImplemented, "no Arrow C format for " << t.ToString());
  }
}

DataType type_of_format(const std::string &f, const ArrowSchema *s) {
  static const std::map<std::string, Type> simple = {
      {"b", Type::BOOL},   {"C", Type::UINT8},  {"c", Type::INT8},   {"S", Type::UINT16},     {"s", Type::INT16},
      {"I", Type::UINT32}, {"i", Type::INT32},  {"L", Type::UINT64}, {"l", Type::INT64},      {"e", Type::HALF_FLOAT},
      {"f", Type::FLOAT},  {"g", Type::DOUBLE}, {"U", Type::STRING}, {"u", Type::STRING},     {"Z", Type::BINARY},
      {"z", Type::BINARY}, {"tdD", Type::DATE32}, {"tdm", Type::DATE64}};
  auto it = simple.find(f);
  if (it != simple.end()) return DataType(it->second);
  if (f.rfind("w:", 0) == 0) return DataType::FixedSizeBinary(std::atoi(f.c_str() + 2));
  if (f.rfind("d:", 0) == 0) {
    int p = 0, sc = 0, bits = 128;
    std::sscanf(f.c_str() + 2, "%d,%d,%d", &p, &sc, &bits);
    CYLON_CHECK(bits == 128 || bits == 256, Code::NotImplemented, "decimal bit width " << bits);
    DataType d(Type::DECIMAL, bits / 8);
    d.precision = p;
    d.scale = sc;
    return d;
  }
  if (f.rfind("ts", 0) == 0 && f.size() >= 4) {
    DataType d = DataType::Timestamp(unit_of_char(f[2]), f.size() > 4 ? f.substr(4) : "");
    return d;
  }
  if (f.rfind("tt", 0) == 0 && f.size() == 3) {
    DataType d(f[2] == 's' || f[2] == 'm' ? Type::TIME32 : Type::TIME64);
    d.unit = unit_of_char(f[2]);
    return d;
  }
  if (f.rfind("tD", 0) == 0 && f.size() == 3) {
    DataType d(Type::DURATION);
    d.unit = unit_of_char(f[2]);
    return d;
  }
  if (f == "+L" || f == "+l") {
    CYLON_CHECK(s->n_children == 1, Code::Invalid, "list schema without a child");
    return DataType::List(type_of_format(s->children[0]->format, s->children[0]).type);
  }
  if (f.rfind("+w:", 0) == 0) {
    CYLON_CHECK(s->n_children == 1, Code::Invalid, "fixed-size list schema without a child");
    return DataType::FixedSizeList(type_of_format(s->children[0]->format, s->children[0]).type, std::atoi(f.c_str() + 3));
  }
  CYLON_THROW(Code::NotImplemented, "Arrow C format '" << f << "' is not supported");
}

// ---------------------------------------------------------------------------
// export
// ---------------------------------------------------------------------------
struct Node {
  std::string format, name;
  std::vector<const void *> buffers;
  std::vector<ArrowArray *> arrays;     // children
  std::vector<ArrowSchema *> schemas;   // children
  std::vector<at::Tensor> keep;
  TablePtr table;                        // root: keeps every column buffer alive
  hipEvent_t event = nullptr;            // root (device export)
};

void release_schema(ArrowSchema *s) {
  if (!s || !s->release) return;
  for (int64_t i = 0; i < s->n_children; ++i) {
    ArrowSchema *c = s->children[i];
    if (c->release) c->release(c);
    delete c;
  }
  delete static_cast<Node *>(s->private_data);
  s->release = nullptr;
}

void release_array(ArrowArray *a) {
  if (!a || !a->release) return;
  for (int64_t i = 0; i < a->n_children; ++i) {
    ArrowArray *c = a->children[i];
    if (c->release) c->release(c);
    delete c;
  }
  Node *n = static_cast<Node *>(a->private_data);
  if (n->event) (void)hipEventDestroy(n->event);
  delete n;
  a->release = nullptr;
}

void fill_schema(ArrowSchema *s, Node *n, int64_t flags) {
  s->format = n->format.c_str();
  s->name = n->name.c_str();
  s->metadata = nullptr;
  s->flags = flags;
  s->n_children = (int64_t)n->schemas.size();
  s->children = n->schemas.empty() ? nullptr : n->schemas.data();
  s->dictionary = nullptr;
  s->release = release_schema;
  s->private_data = n;
}

void fill_array(ArrowArray *a, Node *n, int64_t length, int64_t null_count) {
  a->length = length;
  a->null_count = null_count;
  a->offset = 0;
  a->n_buffers = (int64_t)n->buffers.size();
  a->n_children = (int64_t)n->arrays.size();
  a->buffers = n->buffers.data();
  a->children = n->arrays.empty() ? nullptr : n->arrays.data();
  a->dictionary = nullptr;
  a->release = release_array;
  a->private_data = n;
}

// byte mask -> Arrow bitmap (device or host), null count
std::pair<at::Tensor, int64_t> to_bitmap(const Exec &ex, const at::Tensor &bytes, int64_t n) {
  at::Tensor words = ex.empty_i64(std::max<int64_t>((n + 63) / 64, 1));
  at::Tensor nulls = at::zeros({1}, ex.opts(at::kLong));
  KCALL(ex, pack_validity, bytes.data_ptr<uint8_t>(), n, reinterpret_cast<uint64_t *>(ptr<int64_t>(words)),
        ptr<int64_t>(nulls));
  return {words, nulls.item<int64_t>()};
}

void export_column(const Exec &ex, const Column &c, ArrowSchema *s, ArrowArray *a) {
  auto *sn = new Node();
  auto *an = new Node();
  sn->format = format_of(c.type);
  sn->name = c.name;
  const int64_t n = c.length;
  int64_t nulls = 0;
  const void *validity = nullptr;
  if (c.nullable() && n) {
    auto bm = to_bitmap(ex, c.validity, n);
    nulls = bm.second;
    if (nulls) {
      an->keep.push_back(bm.first);
      validity = bm.first.data_ptr();
    }
  }
  an->buffers.push_back(validity);
  an->keep.push_back(c.data);
  if (c.type.type == Type::BOOL) {  // bit-packed values
    auto bits = to_bitmap(ex, c.data, n);
    an->keep.push_back(bits.first);
    an->buffers.push_back(bits.first.data_ptr());
  } else if (c.type.type == Type::LIST) {  // element offsets + child values
    const int64_t w = c.type.value_width();
    at::Tensor eo = c.offsets.slice(0, 0, n + 1).div(w, "trunc").contiguous();
    an->keep.push_back(eo);
    an->buffers.push_back(eo.data_ptr());
    const int64_t elems = n ? ops::read_i64(eo, n) : 0;
    ArrowSchema *cs = new ArrowSchema();
    ArrowArray *ca = new ArrowArray();
    auto *csn = new Node(), *can = new Node();
    csn->format = format_of(DataType(c.type.value_type));
    csn->name = "item";
    can->buffers = {nullptr, c.data.numel() ? c.data.data_ptr() : nullptr};
    fill_schema(cs, csn, 2 /* nullable */);
    fill_array(ca, can, elems, 0);
    sn->schemas.push_back(cs);
    an->arrays.push_back(ca);
  } else if (c.type.type == Type::FIXED_SIZE_LIST) {
    ArrowSchema *cs = new ArrowSchema();
    ArrowArray *ca = new ArrowArray();
    auto *csn = new Node(), *can = new Node();
    csn->format = format_of(DataType(c.type.value_type));
    csn->name = "item";
    can->buffers = {nullptr, c.data.numel() ? c.data.data_ptr() : nullptr};
    fill_schema(cs, csn, 2);
    fill_array(ca, can, n * c.type.list_size, 0);
    sn->schemas.push_back(cs);
    an->arrays.push_back(ca);
  } else if (c.is_var()) {  // large utf8 / binary: int64 offsets + bytes, as stored
    an->keep.push_back(c.offsets);
    an->buffers.push_back(c.offsets.data_ptr());
    an->buffers.push_back(c.data.numel() ? c.data.data_ptr() : nullptr);
  } else {
    an->buffers.push_back(c.data.numel() ? c.data.data_ptr() : nullptr);
  }
  fill_schema(s, sn, 2);
  fill_array(a, an, n, nulls);
}

// ---------------------------------------------------------------------------
// import
// ---------------------------------------------------------------------------
struct Holder {
  ArrowArray array{};
  ArrowSchema schema{};
  ~Holder() {
    if (array.release) array.release(&array);
    if (schema.release) schema.release(&schema);
  }
};

at::Tensor wrap(const std::shared_ptr<Holder> &h, const void *p, int64_t nbytes, at::Device dev) {
  if (nbytes <= 0 || !p) return at::empty({0}, at::TensorOptions().dtype(at::kByte).device(dev));
  return at::from_blob(const_cast<void *>(p), {nbytes}, [h](void *) {}, at::TensorOptions().dtype(at::kByte).device(dev));
}

Column import_column(const Exec &ex, const std::shared_ptr<Holder> &h, const ArrowSchema *s, const ArrowArray *a,
                     at::Device dev) {
  const std::string f = s->format;
  const DataType t = type_of_format(f, s);
  const int64_t n = a->length, off = a->offset;
  at::Tensor valid;
  if (a->null_count != 0 && a->n_buffers > 0 && a->buffers[0]) {
    valid = at::empty({n}, ex.opts(at::kByte));
    KCALL(ex, unpack_validity, static_cast<const uint8_t *>(a->buffers[0]), off, n, ptr<uint8_t>(valid));
  }
  auto as_dtype = [&](at::Tensor bytes) { return bytes.view(storage_dtype(t)); };
  if (t.type == Type::BOOL) {
    at::Tensor b = at::empty({n}, ex.opts(at::kByte));
    KCALL(ex, unpack_validity, static_cast<const uint8_t *>(a->buffers[1]), off, n, ptr<uint8_t>(b));
    return Column(s->name ? s->name : "", t, n, b, at::Tensor(), valid);
  }
  if (t.type == Type::STRING || t.type == Type::BINARY) {
    const bool large = f == "U" || f == "Z";
    at::Tensor o;
    if (large) {
      o = wrap(h, static_cast<const int64_t *>(a->buffers[1]) + off, (n + 1) * 8, dev).view(at::kLong);
    } else {
      o = wrap(h, static_cast<const int32_t *>(a->buffers[1]) + off, (n + 1) * 4, dev).view(at::kInt).to(at::kLong);
    }
    const int64_t first = ops::read_i64(o, 0), last = ops::read_i64(o, n);
    at::Tensor bytes = wrap(h, static_cast<const uint8_t *>(a->buffers[2]) + first, last - first, dev);
    if (first != 0) o = o - first;
    return Column(s->name ? s->name : "", t, n, bytes, o.contiguous(), valid);
  }
  if (t.type == Type::LIST) {
    const ArrowSchema *cs = s->children[0];
    const ArrowArray *ca = a->children[0];
    CYLON_CHECK(ca->null_count == 0, Code::NotImplemented, "null list elements are not supported");
    const int64_t w = t.value_width();
    const bool large = f == "+L";
    at::Tensor o = large ? wrap(h, static_cast<const int64_t *>(a->buffers[1]) + off, (n + 1) * 8, dev).view(at::kLong)
                         : wrap(h, static_cast<const int32_t *>(a->buffers[1]) + off, (n + 1) * 4, dev).view(at::kInt).to(at::kLong);
    const int64_t first = ops::read_i64(o, 0), last = ops::read_i64(o, n);
    at::Tensor bytes = wrap(h, static_cast<const uint8_t *>(ca->buffers[1]) + (ca->offset + first) * w, (last - first) * w, dev);
    (void)cs;
    return Column(s->name ? s->name : "", t, n, bytes, ((o - first) * w).contiguous(), valid);
  }
  const int64_t w = t.width();
  if (t.type == Type::FIXED_SIZE_LIST) {
    const ArrowArray *ca = a->children[0];
    const int64_t k = t.list_size, vw = t.value_width();
    at::Tensor bytes = wrap(h, static_cast<const uint8_t *>(ca->buffers[1]) + (ca->offset + off * k) * vw, n * w, dev);
    return Column(s->name ? s->name : "", t, n, bytes, at::Tensor(), valid);
  }
  at::Tensor bytes = wrap(h, static_cast<const uint8_t *>(a->buffers[1]) + off * w, n * w, dev);
  const bool raw = t.kind() == ValueKind::FIXED_BYTES;
  return Column(s->name ? s->name : "", t, n, raw ? bytes : as_dtype(bytes), at::Tensor(), valid);
}

}  // namespace

void ExportDeviceTable(const TablePtr &t, ArrowSchema *schema, ArrowDeviceArray *out) {
  Exec ex(t->device());
  auto *sn = new Node();
  auto *an = new Node();
  sn->format = "+s";
  sn->name = "";
  an->buffers = {nullptr};
  an->table = t;
  for (const auto &c : t->columns()) {
    ArrowSchema *cs = new ArrowSchema();
    ArrowArray *ca = new ArrowArray();
    export_column(ex, c, cs, ca);
    sn->schemas.push_back(cs);
    an->arrays.push_back(ca);
  }
  fill_schema(schema, sn, 0);
  std::memset(out, 0, sizeof(*out));
  fill_array(&out->array, an, t->Rows(), 0);
  if (ex.gpu) {
    HIP_EVENT_CHECK(hipEventCreateWithFlags(&an->event, hipEventDisableTiming));
    HIP_EVENT_CHECK(hipEventRecord(an->event, reinterpret_cast<hipStream_t>(ex.stream)));
    out->device_type = ARROW_DEVICE_ROCM;
    out->device_id = t->device().index();
    out->sync_event = &an->event;
  } else {
    out->device_type = ARROW_DEVICE_CPU;
    out->device_id = -1;
    out->sync_event = nullptr;
  }
}

TablePtr ImportDeviceTable(const std::shared_ptr<CylonContext> &ctx, ArrowSchema *schema, ArrowDeviceArray *in) {
  CYLON_CHECK(schema && schema->release && in && in->array.release, Code::Invalid, "released Arrow C structs");
  CYLON_CHECK(std::string(schema->format) == "+s", Code::Invalid, "a table imports from a struct array ('+s')");
  CYLON_CHECK(in->array.offset == 0, Code::NotImplemented, "sliced struct arrays are not supported");
  at::Device dev(at::kCPU);
  if (in->device_type == ARROW_DEVICE_ROCM) dev = at::Device(at::kCUDA, (c10::DeviceIndex)in->device_id);
  else CYLON_CHECK(in->device_type == ARROW_DEVICE_CPU, Code::NotImplemented,
                   "Arrow device type " << in->device_type << " is not supported");
  Exec ex(dev);
  if (in->sync_event && ex.gpu)  // the producer's buffers are ready once its event fires
    HIP_EVENT_CHECK(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(ex.stream),
                                       *static_cast<hipEvent_t *>(in->sync_event), 0));
  auto h = std::make_shared<Holder>();
  h->array = in->array;  // move
  h->schema = *schema;
  in->array.release = nullptr;
  schema->release = nullptr;
  std::vector<Column> cols;
  for (int64_t i = 0; i < h->schema.n_children; ++i)
    cols.push_back(import_column(ex, h, h->schema.children[i], h->array.children[i], dev));
  auto out = Table::Make(ctx, std::move(cols));
  return ctx->GetDevice() == dev ? out : out->to(ctx->GetDevice());
}

}  // namespace io
}  // namespace cylon
