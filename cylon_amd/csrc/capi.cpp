// C ABI (cylon_amd/include/cylon_capi.h): see the header.
#include "../include/cylon_capi.h"

#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>

#include "cylon/api.hpp"
#include "cylon/io/csv.hpp"
#include "cylon/table.hpp"

using namespace cylon;

namespace {
thread_local std::string g_err;
std::mutex g_mu;
std::shared_ptr<CylonContext> g_ctx;

std::shared_ptr<CylonContext> ctx() {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_ctx) g_ctx = CylonContext::Init(at::Device(at::kCPU));
  return g_ctx;
}

int fail(int code, const std::string &msg) {
  g_err = msg;
  return code == 0 ? (int)Code::UnknownError : code;
}

template <class F>
int guard(F &&f) {
  try {
    return f();
  } catch (const CylonError &e) {
    return fail((int)e.code(), e.what());
  } catch (const std::exception &e) {
    return fail((int)Code::UnknownError, e.what());
  }
}

int status(const Status &s) { return s.is_ok() ? 0 : fail(s.get_code(), s.get_msg()); }

join::config::JoinConfig make_cfg(int jt, int alg, int l, int r) {
  using namespace join::config;
  const JoinType t = jt == 1 ? JoinType::LEFT : jt == 2 ? JoinType::RIGHT : jt == 3 ? JoinType::FULL_OUTER
                                                                                     : JoinType::INNER;
  const JoinAlgorithm a = alg == 1 ? JoinAlgorithm::HASH : JoinAlgorithm::SORT;
  return JoinConfig(t, l, r, a);
}
}  // namespace

#define CYLON_CAPI __attribute__((visibility("default")))

extern "C" {

CYLON_CAPI int cylon_capi_version(void) { return 1; }
CYLON_CAPI const char *cylon_last_error(void) { return g_err.c_str(); }

CYLON_CAPI int cylon_init(const char *device) {
  return guard([&] {
    std::lock_guard<std::mutex> lk(g_mu);
    g_ctx = CylonContext::Init(at::Device(std::string(device ? device : "cpu")));
    return 0;
  });
}

CYLON_CAPI int cylon_init_distributed(const char *comm_type) {
  return guard([&] {
    const std::string t = comm_type ? comm_type : "rccl";
    net::CommType ct = net::CommType::RCCL;
    if (t == "tcp" || t == "gloo") ct = net::CommType::TCP;
    else if (t == "mpi") ct = net::CommType::MPI;
    else CYLON_CHECK(t == "rccl" || t == "nccl", Code::Invalid, "unknown comm type '" << t << "'");
    std::lock_guard<std::mutex> lk(g_mu);
    net::CommConfig cfg;
    cfg.type = ct;
    g_ctx = CylonContext::InitDistributed(cfg);
    return 0;
  });
}

CYLON_CAPI int cylon_get_rank(void) { return ctx()->GetRank(); }
CYLON_CAPI int cylon_get_world_size(void) { return ctx()->GetWorldSize(); }
CYLON_CAPI int cylon_barrier(void) {
  return guard([&] {
    ctx()->Barrier();
    return 0;
  });
}
CYLON_CAPI int cylon_finalize(void) {
  return guard([&] {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_ctx) g_ctx->Finalize();
    g_ctx.reset();
    return 0;
  });
}

CYLON_CAPI int cylon_read_csv(const char *path, const char *table_id) {
  return guard([&] {
    PutTable(table_id, io::ReadCSV(ctx(), path, io::CSVReadOptions()));
    return 0;
  });
}

CYLON_CAPI int cylon_write_csv(const char *table_id, const char *path) {
  return guard([&] {
    io::WriteCSV(GetTable(table_id), path, io::CSVWriteOptions());
    return 0;
  });
}

CYLON_CAPI int64_t cylon_row_count(const char *table_id) {
  try {
    return RowCount(table_id);
  } catch (const std::exception &e) {
    fail((int)Code::KeyError, e.what());
    return -1;
  }
}

CYLON_CAPI int32_t cylon_column_count(const char *table_id) {
  try {
    return ColumnCount(table_id);
  } catch (const std::exception &e) {
    fail((int)Code::KeyError, e.what());
    return -1;
  }
}

CYLON_CAPI int cylon_remove_table(const char *table_id) {
  return guard([&] {
    RemoveTable(table_id);
    return 0;
  });
}

CYLON_CAPI int cylon_join(const char *l, const char *r, int jt, int alg, int lc, int rc, const char *dest) {
  return guard([&] { return status(JoinTables(l, r, make_cfg(jt, alg, lc, rc), dest)); });
}

CYLON_CAPI int cylon_distributed_join(const char *l, const char *r, int jt, int alg, int lc, int rc,
                                      const char *dest) {
  return guard([&] { return status(DistributedJoinTables(l, r, make_cfg(jt, alg, lc, rc), dest)); });
}

CYLON_CAPI int cylon_set_op(const char *a, const char *b, int op, int distributed, const char *dest) {
  return guard([&] {
    TablePtr ta = GetTable(a), tb = GetTable(b), out;
    Status s;
    if (op == 0) s = distributed ? DistributedUnion(ta, tb, out) : Union(ta, tb, out);
    else if (op == 1) s = distributed ? DistributedSubtract(ta, tb, out) : Subtract(ta, tb, out);
    else s = distributed ? DistributedIntersect(ta, tb, out) : Intersect(ta, tb, out);
    if (s.is_ok()) PutTable(dest, out);
    return status(s);
  });
}

CYLON_CAPI int cylon_sort(const char *id, int column, int ascending, const char *dest) {
  return guard([&] { return status(SortTable(id, column, dest, ascending != 0)); });
}

CYLON_CAPI int cylon_project(const char *id, const int32_t *cols, int n, const char *dest) {
  return guard([&] {
    TablePtr out;
    Status s = Project(GetTable(id), std::vector<int32_t>(cols, cols + n), out);
    if (s.is_ok()) PutTable(dest, out);
    return status(s);
  });
}

CYLON_CAPI int cylon_merge(const char *const *ids, int n, const char *dest) {
  return guard([&] {
    std::vector<TablePtr> ts;
    for (int i = 0; i < n; ++i) ts.push_back(GetTable(ids[i]));
    TablePtr out;
    Status s = Merge(ts, out);
    if (s.is_ok()) PutTable(dest, out);
    return status(s);
  });
}

CYLON_CAPI int cylon_print(const char *id, int64_t b, int64_t e) {
  return guard([&] {
    TablePtr t = GetTable(id);
    TablePtr h = t->device().is_cuda() ? t->to(at::Device(at::kCPU)) : t;
    if (e < 0 || e > h->Rows()) e = h->Rows();
    std::vector<std::string> names = h->ColumnNames();
    for (size_t i = 0; i < names.size(); ++i) std::printf("%s%s", i ? "," : "", names[i].c_str());
    std::printf("\n");
    for (int64_t r = std::max<int64_t>(0, b); r < e; ++r) {
      Row row(h, r);
      for (int c = 0; c < h->Columns(); ++c) {
        if (c) std::printf(",");
        if (row.IsNull(c)) continue;
        const Column &col = h->column(c);
        if (col.is_var()) std::printf("%s", row.GetString(c).c_str());
        else if (col.type.kind() == ValueKind::FLOAT) std::printf("%g", row.GetDouble(c));
        else std::printf("%lld", (long long)row.GetInt64(c));
      }
      std::printf("\n");
    }
    std::fflush(stdout);
    return 0;
  });
}

CYLON_CAPI int cylon_table_from_buffers(const char *id, int ncols, const char *const *names, const int32_t *types,
                                        int64_t nrows, const void *const *data, const uint8_t *const *validity,
                                        const int32_t *const *offsets) {
  return guard([&] {
    std::vector<Column> cols;
    auto opts = [](at::ScalarType st) { return at::TensorOptions().dtype(st).device(at::kCPU); };
    for (int c = 0; c < ncols; ++c) {
      DataType dt(static_cast<Type>(types[c]));
      at::Tensor valid;
      if (validity && validity[c]) {
        valid = at::empty({nrows}, opts(at::kByte));
        uint8_t *v = valid.data_ptr<uint8_t>();
        for (int64_t r = 0; r < nrows; ++r) v[r] = (validity[c][r >> 3] >> (r & 7)) & 1;
      }
      if (dt.is_variable_width()) {
        CYLON_CHECK(offsets && offsets[c], Code::Invalid, "column " << c << " needs offsets");
        at::Tensor off = at::empty({nrows + 1}, opts(at::kLong));
        int64_t *o = off.data_ptr<int64_t>();
        const int32_t base = offsets[c][0];
        for (int64_t r = 0; r <= nrows; ++r) o[r] = offsets[c][r] - base;
        at::Tensor bytes = at::empty({o[nrows]}, opts(at::kByte));
        if (o[nrows]) std::memcpy(bytes.data_ptr(), static_cast<const uint8_t *>(data[c]) + base, (size_t)o[nrows]);
        cols.emplace_back(names[c], dt, nrows, bytes, off, valid);
      } else {
        Column col = make_fixed_column(names[c], dt, nrows, at::Device(at::kCPU), false);
        const int64_t nb = col.data.numel() * col.data.element_size();
        if (nb) std::memcpy(col.data.data_ptr(), data[c], (size_t)nb);
        col.validity = valid;
        cols.push_back(col);
      }
    }
    auto c = ctx();
    TablePtr t = Table::Make(c, std::move(cols));
    PutTable(id, c->GetDevice().is_cuda() ? t->to(c->GetDevice()) : t);
    return 0;
  });
}

struct cylon_row {
  const Row *row;
};

CYLON_CAPI int cylon_select(const char *id, cylon_row_predicate pred, void *user, const char *dest) {
  return guard([&] {
    TablePtr out;
    Status s = Select(
        GetTable(id),
        [&](const Row &r) {
          cylon_row cr{&r};
          return pred(&cr, user) != 0;
        },
        out);
    if (s.is_ok()) PutTable(dest, out);
    return status(s);
  });
}

CYLON_CAPI int64_t cylon_row_index(const cylon_row *r) { return r->row->RowIndex(); }
CYLON_CAPI int cylon_row_is_null(const cylon_row *r, int col) { return r->row->IsNull(col) ? 1 : 0; }
CYLON_CAPI int64_t cylon_row_get_int64(const cylon_row *r, int col) { return r->row->GetInt64(col); }
CYLON_CAPI double cylon_row_get_double(const cylon_row *r, int col) { return r->row->GetDouble(col); }
CYLON_CAPI int64_t cylon_row_get_string(const cylon_row *r, int col, char *buf, int64_t cap) {
  const std::string s = r->row->GetString(col);
  if (buf && cap > 0) {
    const int64_t k = std::min<int64_t>(cap - 1, (int64_t)s.size());
    std::memcpy(buf, s.data(), (size_t)k);
    buf[k] = 0;
  }
  return (int64_t)s.size();
}

}  // extern "C"
