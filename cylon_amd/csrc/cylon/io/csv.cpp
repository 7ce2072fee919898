// Native CSV reader / writer (C25): see csv.hpp.
#include "csv.hpp"
#include "cylon/trace.hpp"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <charconv>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string_view>
#include <thread>
#include <unordered_set>

namespace cylon {
namespace io {

namespace {

class MappedFile {
 public:
  explicit MappedFile(const std::string &path) {
    fd_ = ::open(path.c_str(), O_RDONLY);
    CYLON_CHECK(fd_ >= 0, Code::IOError, "cannot open " << path);
    struct stat st;
    CYLON_CHECK(::fstat(fd_, &st) == 0, Code::IOError, "cannot stat " << path);
    size_ = (size_t)st.st_size;
    if (size_ > 0) {
      void *p = ::mmap(nullptr, size_, PROT_READ, MAP_PRIVATE, fd_, 0);
      CYLON_CHECK(p != MAP_FAILED, Code::IOError, "cannot mmap " << path);
      data_ = static_cast<const char *>(p);
      ::madvise(p, size_, MADV_SEQUENTIAL);
    }
  }
  ~MappedFile() {
    if (data_) ::munmap(const_cast<char *>(data_), size_);
    if (fd_ >= 0) ::close(fd_);
  }
  const char *data() const { return data_; }
  size_t size() const { return size_; }

 private:
  int fd_ = -1;
  const char *data_ = nullptr;
  size_t size_ = 0;
};

struct Field {
  const char *p;
  uint32_t len;
  bool quoted;    // enclosed in quotes
  bool escaped;   // contains doubled quotes (needs unescaping)
};

// Split [b, e) (one line, no newline) into fields.
void split_line(const char *b, const char *e, const CSVReadOptions &o, std::vector<Field> &out) {
  out.clear();
  const char *p = b;
  while (true) {
    Field f{p, 0, false, false};
    if (o.quoting && p < e && *p == o.quote_char) {
      const char *s = ++p;
      while (p < e) {
        if (o.escaping && *p == o.escape_char && p + 1 < e) {
          f.escaped = true;
          p += 2;
          continue;
        }
        if (*p == o.quote_char) {
          if (o.double_quote && p + 1 < e && p[1] == o.quote_char) {
            f.escaped = true;
            p += 2;
            continue;
          }
          break;
        }
        ++p;
      }
      f.p = s;
      f.len = (uint32_t)(p - s);
      f.quoted = true;
      if (p < e) ++p;  // closing quote
      while (p < e && *p != o.delimiter) ++p;
    } else {
      while (p < e && *p != o.delimiter) {
        if (o.escaping && *p == o.escape_char && p + 1 < e) {
          f.escaped = true;
          ++p;
        }
        ++p;
      }
      f.len = (uint32_t)(p - f.p);
    }
    out.push_back(f);
    if (p >= e) break;
    ++p;  // delimiter
    if (p == e) {  // trailing delimiter: one more empty field
      out.push_back(Field{p, 0, false, false});
      break;
    }
  }
}

// field text with doubled quotes (inside quotes) and escape characters resolved
std::string field_string(const Field &f, const CSVReadOptions &o) {
  if (!f.escaped) return std::string(f.p, f.len);
  std::string s;
  s.reserve(f.len);
  for (uint32_t i = 0; i < f.len; ++i) {
    if (o.escaping && f.p[i] == o.escape_char && i + 1 < f.len) {
      s.push_back(f.p[++i]);
      continue;
    }
    s.push_back(f.p[i]);
    if (f.quoted && f.p[i] == o.quote_char && i + 1 < f.len && f.p[i + 1] == o.quote_char) ++i;
  }
  return s;
}

enum Seen : uint8_t { S_NULL = 1, S_INT = 2, S_BOOL = 4, S_DBL = 8, S_STR = 16 };

struct Sets {
  std::unordered_set<std::string_view> nulls, trues, falses;
  // cheap pre-filter for the null lookup: (first byte, length) of any null spelling
  bool first[256] = {};
  bool len[64] = {};
  bool empty_is_null = false;
  void index() {
    for (auto s : trues)
      if (!s.empty()) bfirst[(unsigned char)s[0]] = true;
    for (auto s : falses)
      if (!s.empty()) bfirst[(unsigned char)s[0]] = true;
    for (auto s : nulls) {
      if (s.empty()) empty_is_null = true;
      else first[(unsigned char)s[0]] = true;
      if (s.size() < 64) len[s.size()] = true;
    }
  }
  bool bfirst[256] = {};
  bool is_null(std::string_view s) const {
    if (s.empty()) return empty_is_null;
    if (s.size() >= 64 || !len[s.size()] || !first[(unsigned char)s[0]]) return false;
    return nulls.count(s) > 0;
  }
  bool maybe_bool(std::string_view s) const { return !s.empty() && bfirst[(unsigned char)s[0]]; }
};

bool parse_i64(std::string_view s, int64_t *v) {
  if (s.empty()) return false;
  const char *b = s.data(), *e = b + s.size();
  if (*b == '+') ++b;
  auto r = std::from_chars(b, e, *v);
  return r.ec == std::errc() && r.ptr == e;
}

bool parse_f64(std::string_view s, double *v) {
  if (s.empty()) return false;
  const char *b = s.data(), *e = b + s.size();
  if (*b == '+') ++b;
  auto r = std::from_chars(b, e, *v);
  if (r.ec == std::errc() && r.ptr == e) return true;
  if (s.size() > 120) return false;  // inf / nan spellings etc.: strtod
  char buf[128];
  std::memcpy(buf, s.data(), s.size());
  buf[s.size()] = 0;
  char *end = nullptr;
  *v = std::strtod(buf, &end);
  return end == buf + s.size();
}

uint8_t classify(const Field &f, const Sets &sets) {
  std::string_view s(f.p, f.len);
  if (!f.quoted && sets.is_null(s)) return S_NULL;
  if (f.escaped) return S_STR;
  // character-class fast path: plain integers and decimal numbers
  size_t k = (!s.empty() && (s[0] == '-' || s[0] == '+')) ? 1 : 0;
  bool digits = k < s.size(), numeric = k < s.size();
  for (size_t q = k; q < s.size(); ++q) {
    const char c = s[q];
    const bool dg = c >= '0' && c <= '9';
    digits &= dg;
    numeric &= dg || c == '.' || c == 'e' || c == 'E' || c == '-' || c == '+';
  }
  if (digits && s.size() - k <= 18 && !sets.maybe_bool(s)) return S_INT;
  double d;
  if (numeric && !digits && parse_f64(s, &d)) return S_DBL;
  int64_t i;
  if (parse_i64(s, &i)) return S_INT;
  if (sets.maybe_bool(s) && (sets.trues.count(s) || sets.falses.count(s))) return S_BOOL;
  if (parse_f64(s, &d)) return S_DBL;
  return S_STR;
}

enum class Kind { I64, F64, BOOL, STR };

Kind resolve(uint8_t seen) {
  if (seen & S_STR) return Kind::STR;
  if ((seen & S_BOOL) && (seen & (S_INT | S_DBL))) return Kind::STR;
  if (seen & S_BOOL) return Kind::BOOL;
  if (seen & S_DBL) return Kind::F64;
  if (seen & S_INT) return Kind::I64;
  return Kind::STR;  // only nulls
}

// line starts of [b, e): positions just after '\n' (quotes spanning lines are not supported)
void find_lines(const char *base, size_t b, size_t e, bool skip_empty, std::vector<std::pair<size_t, size_t>> &out) {
  size_t s = b;
  while (s < e) {
    const void *nl = std::memchr(base + s, '\n', e - s);
    size_t t = nl ? (size_t)(static_cast<const char *>(nl) - base) : e;
    size_t te = t;
    if (te > s && base[te - 1] == '\r') --te;
    if (!(skip_empty && te == s)) out.emplace_back(s, te);
    s = t + 1;
  }
}

// newlines_in_values: a newline inside a quoted value does not end the record
void find_records(const char *base, size_t b, size_t e, const CSVReadOptions &o,
                  std::vector<std::pair<size_t, size_t>> &out) {
  size_t s = b;
  bool inq = false;
  for (size_t i = b; i < e; ++i) {
    const char c = base[i];
    if (o.escaping && c == o.escape_char) {
      ++i;
      continue;
    }
    if (o.quoting && c == o.quote_char) inq = !inq;
    else if (c == '\n' && !inq) {
      size_t te = i;
      if (te > s && base[te - 1] == '\r') --te;
      if (!(o.ignore_empty_lines && te == s)) out.emplace_back(s, te);
      s = i + 1;
    }
  }
  if (s < e) {
    size_t te = e;
    if (base[te - 1] == '\r') --te;
    if (!(o.ignore_empty_lines && te == s)) out.emplace_back(s, te);
  }
}

Kind forced_kind(const DataType &t) {
  switch (t.type) {
    case Type::BOOL: return Kind::BOOL;
    case Type::HALF_FLOAT: case Type::FLOAT: case Type::DOUBLE: return Kind::F64;
    case Type::STRING: case Type::BINARY: return Kind::STR;
    default: break;
  }
  CYLON_CHECK(t.layout() == Layout::FIXED_WIDTH && t.type != Type::FIXED_SIZE_BINARY && t.type != Type::DECIMAL, Code::NotImplemented,
              "CSV column type " << t.ToString() << " is not supported");
  return Kind::I64;  // integers and the integer-backed temporal types
}

template <class F>
void parallel_for(int T, F &&fn) {
  if (T <= 1) {
    fn(0);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(T);
  std::vector<std::exception_ptr> errs(T);
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t]() {
      try {
        fn(t);
      } catch (...) {
        errs[t] = std::current_exception();
      }
    });
  for (auto &x : th) x.join();
  for (auto &e : errs)
    if (e) std::rethrow_exception(e);
}

}  // namespace

TablePtr ReadCSV(const std::shared_ptr<CylonContext> &ctx, const std::string &path, const CSVReadOptions &o) {
  MappedFile mf(path);
  const char *base = mf.data();
  const size_t size = mf.size();
  Sets sets;
  static const std::vector<std::string> kArrowNulls{"",     "#N/A", "#N/A N/A", "#NA", "-1.#IND", "-1.#QNAN",
                                                    "-NaN", "-nan", "1.#IND",   "1.#QNAN", "N/A", "NA",
                                                    "NULL", "NaN",  "n/a",      "nan",     "null"};
  const std::vector<std::string> &nulls = o.null_values.empty() ? kArrowNulls : o.null_values;
  for (const auto &s : nulls) sets.nulls.insert(s);
  for (const auto &s : o.true_values) sets.trues.insert(s);
  for (const auto &s : o.false_values) sets.falses.insert(s);
  sets.index();

  // skip rows, then the header
  size_t pos = 0;
  for (int64_t i = 0; i < o.skip_rows && pos < size; ++i) {
    const void *nl = std::memchr(base + pos, '\n', size - pos);
    pos = nl ? (size_t)(static_cast<const char *>(nl) - base) + 1 : size;
  }
  std::vector<std::string> names = o.column_names;
  std::vector<Field> fields;
  const bool header_row = names.empty() && !o.autogenerate_column_names && o.header;
  if (header_row) {
    while (pos < size) {  // first non-empty line
      const void *nl = std::memchr(base + pos, '\n', size - pos);
      size_t t = nl ? (size_t)(static_cast<const char *>(nl) - base) : size;
      size_t te = (t > pos && base[t - 1] == '\r') ? t - 1 : t;
      const size_t ls = pos;
      pos = t + 1;
      if (te == ls && o.ignore_empty_lines) continue;
      split_line(base + ls, base + te, o, fields);
      for (const auto &f : fields) names.push_back(field_string(f, o));
      break;
    }
  }
  // line-aligned chunks
  int T = o.threads > 0 ? o.threads : (int)std::min<unsigned>(16, std::max(1u, std::thread::hardware_concurrency()));
  const size_t data_bytes = pos < size ? size - pos : 0;
  const size_t min_block = (size_t)std::max<int32_t>(1, o.block_size);
  T = (int)std::max<size_t>(1, std::min<size_t>((size_t)T, data_bytes / min_block));  // >= block_size per thread
  if (!o.use_threads || o.newlines_in_values) T = 1;
  std::vector<size_t> cut(T + 1, size);
  cut[0] = std::min(pos, size);
  for (int t = 1; t < T; ++t) {
    size_t c = cut[0] + data_bytes * t / T;
    const void *nl = c < size ? std::memchr(base + c, '\n', size - c) : nullptr;
    cut[t] = nl ? (size_t)(static_cast<const char *>(nl) - base) + 1 : size;
    cut[t] = std::max(cut[t], cut[t - 1]);
  }
  std::vector<std::vector<std::pair<size_t, size_t>>> lines(T);
  auto tick = [t0 = std::chrono::steady_clock::now()](const char *what) {
    if (trace::log_level() >= 3)
      std::fprintf(stderr, "[csv] %-10s %.3f ms\n", what,
                   std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  };
  tick("open");
  if (o.newlines_in_values) find_records(base, cut[0], cut[1], o, lines[0]);
  else parallel_for(T, [&](int t) { find_lines(base, cut[t], cut[t + 1], o.ignore_empty_lines, lines[t]); });
  tick("lines");

  // column count
  int ncols = (int)names.size();
  if (ncols == 0) {
    for (auto &lv : lines)
      if (!lv.empty()) {
        split_line(base + lv[0].first, base + lv[0].second, o, fields);
        ncols = (int)fields.size();
        break;
      }
    for (int i = 0; i < ncols; ++i) names.push_back("f" + std::to_string(i));
  }
  // selected columns (output order)
  std::vector<int> sel;
  std::vector<std::string> missing;  // output position -> name of an absent included column ("" = parsed)
  if (o.include_columns.empty()) {
    for (int i = 0; i < ncols; ++i) sel.push_back(i);
  } else {
    for (const auto &c : o.include_columns) {
      auto it = std::find(names.begin(), names.end(), c);
      if (it == names.end()) {
        CYLON_CHECK(o.include_missing_columns, Code::KeyError, "CSV column '" << c << "' not found in " << path);
        missing.resize(sel.size() + 1);
        missing.back() = c;
        sel.push_back(-1);
        continue;
      }
      sel.push_back((int)(it - names.begin()));
    }
  }
  missing.resize(sel.size());
  const int nsel = (int)sel.size();

  // pass A: type inference
  std::vector<std::vector<uint8_t>> seen(T, std::vector<uint8_t>(nsel, 0));
  parallel_for(T, [&](int t) {
    std::vector<Field> fs;
    for (const auto &ln : lines[t]) {
      split_line(base + ln.first, base + ln.second, o, fs);
      CYLON_CHECK((int)fs.size() == ncols, Code::Invalid,
                  "CSV parse error in " << path << ": expected " << ncols << " columns, got " << fs.size());
      for (int j = 0; j < nsel; ++j)
        if (sel[j] >= 0) seen[t][j] |= classify(fs[sel[j]], sets);
    }
  });
  tick("infer");
  std::vector<Kind> kinds(nsel);
  std::vector<const DataType *> want(nsel, nullptr);  // explicit column_types entry
  for (int j = 0; j < nsel; ++j) {
    uint8_t s = 0;
    for (int t = 0; t < T; ++t) s |= seen[t][j];
    kinds[j] = resolve(s);
    auto it = o.column_types.find(sel[j] >= 0 ? names[sel[j]] : missing[j]);
    if (it != o.column_types.end()) {
      want[j] = &it->second;
      kinds[j] = forced_kind(it->second);
    }
  }
  std::vector<int64_t> row0(T + 1, 0);
  for (int t = 0; t < T; ++t) row0[t + 1] = row0[t] + (int64_t)lines[t].size();
  const int64_t n = row0[T];

  // pass B: convert
  std::vector<at::Tensor> data(nsel), valid(nsel);
  std::vector<std::vector<std::string>> sbytes(nsel, std::vector<std::string>(T));
  std::vector<std::vector<std::vector<int64_t>>> slens(nsel, std::vector<std::vector<int64_t>>(T));
  auto cpu = [](at::ScalarType st) { return at::TensorOptions().dtype(st).device(at::kCPU); };
  for (int j = 0; j < nsel; ++j) {
    valid[j] = at::ones({n}, cpu(at::kByte));
    if (kinds[j] == Kind::I64) data[j] = at::empty({n}, cpu(at::kLong));
    if (kinds[j] == Kind::F64) data[j] = at::empty({n}, cpu(at::kDouble));
    if (kinds[j] == Kind::BOOL) data[j] = at::empty({n}, cpu(storage_dtype(DataType(Type::BOOL))));
  }
  for (int j = 0; j < nsel; ++j)
    if (sel[j] < 0 && data[j].defined()) data[j].zero_();
  std::vector<uint8_t *> vptr(nsel);
  std::vector<void *> dptr(nsel, nullptr);
  for (int j = 0; j < nsel; ++j) {
    vptr[j] = valid[j].data_ptr<uint8_t>();
    if (data[j].defined()) dptr[j] = data[j].data_ptr();
  }
  std::vector<std::vector<uint8_t>> anynull(T, std::vector<uint8_t>(nsel, 0));
  tick("alloc");
  parallel_for(T, [&](int t) {
    std::vector<Field> fs;
    int64_t r = row0[t];
    for (const auto &ln : lines[t]) {
      split_line(base + ln.first, base + ln.second, o, fs);
      for (int j = 0; j < nsel; ++j) {
        uint8_t *v = vptr[j];
        if (sel[j] < 0) {  // absent included column: null
          v[r] = 0;
          anynull[t][j] = 1;
          if (kinds[j] == Kind::STR) slens[j][t].push_back(0);
          continue;
        }
        const Field &f = fs[sel[j]];
        std::string_view s(f.p, f.len);
        const bool is_null = !f.quoted && sets.is_null(s);
        const bool strict = want[j] != nullptr;  // explicit types reject unparsable values
        switch (kinds[j]) {
          case Kind::I64: {
            int64_t x = 0;
            if (is_null) v[r] = 0, anynull[t][j] = 1;
            else if (!parse_i64(s, &x) && strict)
              CYLON_THROW(Code::Invalid, "CSV conversion error in " << path << ": '" << s << "' is not an integer");
            static_cast<int64_t *>(dptr[j])[r] = x;
            break;
          }
          case Kind::F64: {
            double x = 0;
            if (is_null) v[r] = 0, anynull[t][j] = 1;
            else if (!parse_f64(s, &x) && strict)
              CYLON_THROW(Code::Invalid, "CSV conversion error in " << path << ": '" << s << "' is not a number");
            static_cast<double *>(dptr[j])[r] = x;
            break;
          }
          case Kind::BOOL: {
            uint8_t x = 0;
            if (is_null) v[r] = 0, anynull[t][j] = 1;
            else if (sets.trues.count(s)) x = 1;
            else if (strict && !sets.falses.count(s))
              CYLON_THROW(Code::Invalid, "CSV conversion error in " << path << ": '" << s << "' is not a boolean");
            static_cast<uint8_t *>(dptr[j])[r] = x;
            break;
          }
          case Kind::STR: {
            if (is_null && o.strings_can_be_null) {
              v[r] = 0;
              anynull[t][j] = 1;
              slens[j][t].push_back(0);
            } else {
              const std::string x = field_string(f, o);
              sbytes[j][t] += x;
              slens[j][t].push_back((int64_t)x.size());
            }
            break;
          }
        }
      }
      ++r;
    }
  });
  tick("convert");
  std::vector<Column> cols;
  for (int j = 0; j < nsel; ++j) {
    const std::string &name = sel[j] >= 0 ? names[sel[j]] : missing[j];
    bool any_null = false;
    for (int t = 0; t < T; ++t) any_null |= anynull[t][j] != 0;
    at::Tensor vd = any_null ? valid[j] : at::Tensor();
    if (kinds[j] == Kind::STR) {
      int64_t total = 0;
      for (int t = 0; t < T; ++t) total += (int64_t)sbytes[j][t].size();
      at::Tensor bytes = at::empty({total}, cpu(at::kByte));
      at::Tensor offs = at::empty({n + 1}, cpu(at::kLong));
      int64_t *op = offs.data_ptr<int64_t>();
      uint8_t *bp = bytes.data_ptr<uint8_t>();
      int64_t acc = 0, r = 0;
      op[0] = 0;
      for (int t = 0; t < T; ++t) {
        std::memcpy(bp + acc, sbytes[j][t].data(), sbytes[j][t].size());
        for (int64_t len : slens[j][t]) {
          acc += len;
          op[++r] = acc;
        }
      }
      cols.emplace_back(name, want[j] ? *want[j] : DataType(Type::STRING), n, bytes, offs, vd);
    } else {
      const Type ty = kinds[j] == Kind::I64 ? Type::INT64 : kinds[j] == Kind::F64 ? Type::DOUBLE : Type::BOOL;
      if (want[j] && want[j]->type != ty) {  // narrow / reinterpret to the requested type
        cols.emplace_back(name, *want[j], n, data[j].to(storage_dtype(*want[j])), at::Tensor(), vd);
        continue;
      }
      cols.emplace_back(name, DataType(ty), n, data[j], at::Tensor(), vd);
    }
  }
  tick("columns");
  TablePtr t = Table::Make(ctx, std::move(cols));
  return ctx->GetDevice().is_cuda() ? t->to(ctx->GetDevice()) : t;
}

std::vector<TablePtr> ReadCSVs(const std::shared_ptr<CylonContext> &ctx, const std::vector<std::string> &paths,
                               const CSVReadOptions &opts) {
  std::vector<TablePtr> out(paths.size());
  CSVReadOptions o = opts;
  if (o.threads == 0)
    o.threads = std::max(1, (int)std::min<size_t>(16, std::thread::hardware_concurrency()) / (int)std::max<size_t>(1, paths.size()));
  if (o.concurrent_file_reads) parallel_for((int)paths.size(), [&](int i) { out[i] = ReadCSV(ctx, paths[i], o); });
  else
    for (size_t i = 0; i < paths.size(); ++i) out[i] = ReadCSV(ctx, paths[i], o);
  return out;
}

namespace {
void put_escaped(std::string &out, const char *p, size_t len, char delim) {
  bool q = false;
  for (size_t i = 0; i < len; ++i)
    if (p[i] == delim || p[i] == '"' || p[i] == '\n' || p[i] == '\r') q = true;
  if (!q) {
    out.append(p, len);
    return;
  }
  out.push_back('"');
  for (size_t i = 0; i < len; ++i) {
    if (p[i] == '"') out.push_back('"');
    out.push_back(p[i]);
  }
  out.push_back('"');
}
}  // namespace

// CSV text of columns [col1, col2) and rows [row1, row2) of a host table
static void write_csv_rows(const TablePtr &t, int col1, int col2, int64_t row1, int64_t row2, char delim,
                           const std::vector<std::string> &names, std::ostream &f) {
  std::string out;
  for (int i = col1; i < col2; ++i) {
    if (i > col1) out.push_back(delim);
    out.push_back('"');
    out += names[i - col1];
    out.push_back('"');
  }
  out.push_back('\n');
  char buf[64];
  for (int64_t r = row1; r < row2; ++r) {
    for (int c = col1; c < col2; ++c) {
      if (c > col1) out.push_back(delim);
      const Column &col = t->column(c);
      if (col.nullable() && col.validity.data_ptr<uint8_t>()[r] == 0) continue;
      const uint8_t *d = static_cast<const uint8_t *>(col.data.data_ptr());
      if (col.is_var()) {
        const int64_t *o = col.offsets.data_ptr<int64_t>();
        put_escaped(out, reinterpret_cast<const char *>(d) + o[r], (size_t)(o[r + 1] - o[r]), delim);
        continue;
      }
      const int w = col.type.width();
      const ValueKind k = col.type.kind();
      std::to_chars_result res{buf, std::errc()};
      if (col.type.type == Type::BOOL) {
        out += d[r] ? "true" : "false";
        continue;
      }
      if (k == ValueKind::FLOAT) {
        const double x = w == 8 ? reinterpret_cast<const double *>(d)[r]
                                : w == 4 ? (double)reinterpret_cast<const float *>(d)[r] : 0.0;
        res = w == 4 ? std::to_chars(buf, buf + sizeof(buf), reinterpret_cast<const float *>(d)[r])
                     : std::to_chars(buf, buf + sizeof(buf), x);
      } else if (k == ValueKind::SIGNED_INT) {
        int64_t x = w == 1 ? (int64_t)reinterpret_cast<const int8_t *>(d)[r]
                    : w == 2 ? (int64_t)reinterpret_cast<const int16_t *>(d)[r]
                    : w == 4 ? (int64_t)reinterpret_cast<const int32_t *>(d)[r]
                             : reinterpret_cast<const int64_t *>(d)[r];
        res = std::to_chars(buf, buf + sizeof(buf), x);
      } else if (k == ValueKind::UNSIGNED_INT) {
        uint64_t x = w == 1 ? d[r]
                     : w == 2 ? reinterpret_cast<const uint16_t *>(d)[r]
                     : w == 4 ? reinterpret_cast<const uint32_t *>(d)[r]
                              : reinterpret_cast<const uint64_t *>(d)[r];
        res = std::to_chars(buf, buf + sizeof(buf), x);
      } else {
        CYLON_THROW(Code::NotImplemented, "CSV text: unsupported column type " << col.type.ToString());
      }
      out.append(buf, res.ptr);
    }
    out.push_back('\n');
    if (out.size() > (1 << 22)) {
      f.write(out.data(), (std::streamsize)out.size());
      out.clear();
    }
  }
  f.write(out.data(), (std::streamsize)out.size());
}

void WriteCSV(const TablePtr &table, const std::string &path, const CSVWriteOptions &opts) {
  TablePtr t = table->device().is_cuda() ? table->to(at::Device(at::kCPU)) : table;
  std::ofstream f(path, std::ios::binary);
  CYLON_CHECK(f.good(), Code::IOError, "cannot open " << path << " for writing");
  std::vector<std::string> names = opts.column_names.empty() ? t->ColumnNames() : opts.column_names;
  CYLON_CHECK((int)names.size() == t->Columns(), Code::Invalid, "CSV header has " << names.size() << " names for "
                                                                                   << t->Columns() << " columns");
  write_csv_rows(t, 0, t->Columns(), 0, t->Rows(), opts.delimiter, names, f);
  CYLON_CHECK(f.good(), Code::IOError, "write failed: " << path);
}

void PrintToOStream(const TablePtr &table, int col1, int col2, int64_t row1, int64_t row2, std::ostream &out,
                    char delimiter, bool use_custom_header, const std::vector<std::string> &headers) {
  col2 = col2 < 0 ? table->Columns() : std::min(col2, table->Columns());
  row2 = row2 < 0 ? table->Rows() : std::min(row2, table->Rows());
  col1 = std::max(0, std::min(col1, col2));
  row1 = std::max<int64_t>(0, std::min(row1, row2));
  // only the printed rows travel to the host
  TablePtr t = table->device().is_cuda() ? ops::Slice(table, row1, row2 - row1)->to(at::Device(at::kCPU))
                                         : ops::Slice(table, row1, row2 - row1);
  std::vector<std::string> names;
  if (use_custom_header) {
    CYLON_CHECK((int)headers.size() == col2 - col1, Code::Invalid,
                "custom header has " << headers.size() << " names for " << (col2 - col1) << " columns");
    names = headers;
  } else {
    for (int c = col1; c < col2; ++c) names.push_back(t->column(c).name);
  }
  write_csv_rows(t, col1, col2, 0, t->Rows(), delimiter, names, out);
}

}  // namespace io
}  // namespace cylon
