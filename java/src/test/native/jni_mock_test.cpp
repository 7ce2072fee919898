// Executes the JNI layer (java/src/main/native/cylon_jni.cpp, J2) without a JDK: the JNIEnv
// members it calls are implemented here over plain C++ objects (mock_jni/jni.h), and every native
// method of org.cylonamd.{CylonContext, Table, Row, ArrowTable} is called the way the Java classes
// call it, against the engine behind the C ABI (libcylon_amd.so).  Prints "key value" lines for the
// pytest driver (tests/test_jni_mock.py), which checks them against the Python API.
#include <jni.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <functional>
#include <memory>
#include <string>
#include <vector>

// ---- mock JVM objects
struct MString : _jobject {
  std::string s;
  explicit MString(std::string v) : s(std::move(v)) {}
};
struct MIntArray : _jobject {
  std::vector<jint> v;
};
struct MLongArray : _jobject {
  std::vector<jlong> v;
};
struct MObjArray : _jobject {
  std::vector<jobject> v;
};
struct MClass : _jobject {
  std::string name;
  explicit MClass(std::string n) : name(std::move(n)) {}
};
struct MRow : _jobject {  // org.cylonamd.Row: wraps the native row handle
  jlong handle;
  explicit MRow(jlong h) : handle(h) {}
};
struct MPredicate : _jobject {  // a java.util.function.Predicate<Row>
  std::function<bool(jlong)> fn;
};
struct _jmethodID {
  std::string name;
};

static std::vector<std::unique_ptr<_jobject>> g_objs;  // the "heap"
static std::vector<std::unique_ptr<_jmethodID>> g_methods;
static int g_live_local_refs = 0;
template <class T>
static T *mk(T *o) {
  g_objs.emplace_back(o);
  return o;
}
static jstring js(const std::string &s) { return mk(new MString(s)); }

const char *JNIEnv::GetStringUTFChars(jstring s, jboolean *is_copy) {
  if (is_copy) *is_copy = 0;
  return static_cast<MString *>(s)->s.c_str();
}
void JNIEnv::ReleaseStringUTFChars(jstring, const char *) {}
jstring JNIEnv::NewStringUTF(const char *c) { return js(c); }
jclass JNIEnv::FindClass(const char *name) { return mk(new MClass(name)); }
jclass JNIEnv::GetObjectClass(jobject) { return mk(new MClass("java/util/function/Predicate")); }
jmethodID JNIEnv::GetMethodID(jclass, const char *name, const char *) {
  g_methods.emplace_back(new _jmethodID{name});
  return g_methods.back().get();
}
jobject JNIEnv::NewObject(jclass cls, jmethodID ctor, ...) {
  if (static_cast<MClass *>(cls)->name != "org/cylonamd/Row" || ctor->name != "<init>") return nullptr;
  va_list ap;
  va_start(ap, ctor);
  const jlong h = va_arg(ap, jlong);
  va_end(ap);
  ++g_live_local_refs;
  return new MRow(h);  // a local reference: the layer deletes it (DeleteLocalRef)
}
jboolean JNIEnv::CallBooleanMethod(jobject o, jmethodID m, ...) {
  if (m->name != "test") return 0;
  va_list ap;
  va_start(ap, m);
  jobject row = va_arg(ap, jobject);
  va_end(ap);
  return static_cast<MPredicate *>(o)->fn(static_cast<MRow *>(row)->handle) ? 1 : 0;
}
void JNIEnv::DeleteLocalRef(jobject o) {
  --g_live_local_refs;
  delete o;
}
jsize JNIEnv::GetArrayLength(jobject a) {
  if (auto *i = dynamic_cast<MIntArray *>(a)) return (jsize)i->v.size();
  if (auto *l = dynamic_cast<MLongArray *>(a)) return (jsize)l->v.size();
  return (jsize) static_cast<MObjArray *>(a)->v.size();
}
void JNIEnv::GetIntArrayRegion(jintArray a, jsize start, jsize len, jint *buf) {
  std::memcpy(buf, static_cast<MIntArray *>(a)->v.data() + start, sizeof(jint) * len);
}
void JNIEnv::GetLongArrayRegion(jlongArray a, jsize start, jsize len, jlong *buf) {
  std::memcpy(buf, static_cast<MLongArray *>(a)->v.data() + start, sizeof(jlong) * len);
}
jobject JNIEnv::GetObjectArrayElement(jobjectArray a, jsize i) { return static_cast<MObjArray *>(a)->v[i]; }

// ---- the native methods under test (cylon_jni.cpp)
#define J(cls, name) Java_org_cylonamd_##cls##_##name
extern "C" {
jint J(CylonContext, nativeInit)(JNIEnv *, jclass, jstring);
jint J(CylonContext, nativeRank)(JNIEnv *, jclass);
jint J(CylonContext, nativeWorldSize)(JNIEnv *, jclass);
jint J(CylonContext, nativeBarrier)(JNIEnv *, jclass);
jint J(CylonContext, nativeFinalize)(JNIEnv *, jclass);
jstring J(CylonContext, nativeLastError)(JNIEnv *, jclass);
jint J(Table, nativeReadCSV)(JNIEnv *, jclass, jstring, jstring);
jint J(Table, nativeWriteCSV)(JNIEnv *, jclass, jstring, jstring);
jlong J(Table, nativeRowCount)(JNIEnv *, jclass, jstring);
jint J(Table, nativeColumnCount)(JNIEnv *, jclass, jstring);
jint J(Table, nativeJoin)(JNIEnv *, jclass, jstring, jstring, jint, jint, jint, jint, jboolean, jstring);
jint J(Table, nativeSetOp)(JNIEnv *, jclass, jstring, jstring, jint, jboolean, jstring);
jint J(Table, nativeSort)(JNIEnv *, jclass, jstring, jint, jboolean, jstring);
jint J(Table, nativeProject)(JNIEnv *, jclass, jstring, jintArray, jstring);
jint J(Table, nativeMerge)(JNIEnv *, jclass, jobjectArray, jstring);
jint J(Table, nativeSelect)(JNIEnv *, jclass, jstring, jobject, jstring);
jint J(Table, nativeRemove)(JNIEnv *, jclass, jstring);
jlong J(Row, nativeIndex)(JNIEnv *, jclass, jlong);
jboolean J(Row, nativeIsNull)(JNIEnv *, jclass, jlong, jint);
jlong J(Row, nativeGetInt64)(JNIEnv *, jclass, jlong, jint);
jdouble J(Row, nativeGetDouble)(JNIEnv *, jclass, jlong, jint);
jstring J(Row, nativeGetString)(JNIEnv *, jclass, jlong, jint);
jint J(ArrowTable, nativeFromBuffers)(JNIEnv *, jclass, jstring, jobjectArray, jintArray, jlong, jlongArray,
                                      jlongArray, jlongArray);
}

static int g_fail = 0;
#define CHECK(c)                                                      \
  do {                                                                \
    if (!(c)) {                                                       \
      std::fprintf(stderr, "CHECK failed line %d: %s\n", __LINE__, #c); \
      ++g_fail;                                                       \
    }                                                                 \
  } while (0)

int main(int argc, char **argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s <csv a> <csv b> <out dir>\n", argv[0]);
    return 2;
  }
  JNIEnv envo;
  JNIEnv *env = &envo;
  jclass cls = mk(new MClass("org/cylonamd/Table"));
  CHECK(J(CylonContext, nativeInit)(env, cls, js("cpu")) == 0);
  std::printf("world %d\nrank %d\n", J(CylonContext, nativeWorldSize)(env, cls), J(CylonContext, nativeRank)(env, cls));
  CHECK(J(CylonContext, nativeBarrier)(env, cls) == 0);
  CHECK(J(Table, nativeReadCSV)(env, cls, js(argv[1]), js("A")) == 0);
  CHECK(J(Table, nativeReadCSV)(env, cls, js(argv[2]), js("B")) == 0);
  std::printf("rows_a %lld\ncols_a %d\n", (long long)J(Table, nativeRowCount)(env, cls, js("A")),
              J(Table, nativeColumnCount)(env, cls, js("A")));
  // inner hash join on column 0 (Table.join: type 0, algorithm 1 = hash)
  CHECK(J(Table, nativeJoin)(env, cls, js("A"), js("B"), 0, 1, 0, 0, 0, js("J")) == 0);
  std::printf("join_rows %lld\njoin_cols %d\n", (long long)J(Table, nativeRowCount)(env, cls, js("J")),
              J(Table, nativeColumnCount)(env, cls, js("J")));
  CHECK(J(Table, nativeJoin)(env, cls, js("A"), js("B"), 3, 0, 0, 0, 0, js("JO")) == 0);
  std::printf("outer_rows %lld\n", (long long)J(Table, nativeRowCount)(env, cls, js("JO")));
  CHECK(J(Table, nativeSetOp)(env, cls, js("A"), js("B"), 0, 0, js("U")) == 0);
  std::printf("union_rows %lld\n", (long long)J(Table, nativeRowCount)(env, cls, js("U")));
  CHECK(J(Table, nativeSort)(env, cls, js("A"), 0, 1, js("S")) == 0);
  auto *pc = mk(new MIntArray);
  pc->v = {1};
  CHECK(J(Table, nativeProject)(env, cls, js("A"), pc, js("P")) == 0);
  std::printf("project_cols %d\n", J(Table, nativeColumnCount)(env, cls, js("P")));
  auto *ids = mk(new MObjArray);
  ids->v = {js("A"), js("B")};
  CHECK(J(Table, nativeMerge)(env, cls, ids, js("M")) == 0);
  std::printf("merge_rows %lld\n", (long long)J(Table, nativeRowCount)(env, cls, js("M")));
  // select through a Java predicate: rows of A whose column 0 is even (Row.getInt64)
  auto *even = mk(new MPredicate);
  int64_t seen = 0;
  even->fn = [&](jlong h) {
    ++seen;
    CHECK(J(Row, nativeIndex)(env, cls, h) >= 0);
    return !J(Row, nativeIsNull)(env, cls, h, 0) && J(Row, nativeGetInt64)(env, cls, h, 0) % 2 == 0;
  };
  CHECK(J(Table, nativeSelect)(env, cls, js("A"), even, js("E")) == 0);
  std::printf("select_even_rows %lld\nselect_visited %lld\nlocal_refs_left %d\n",
              (long long)J(Table, nativeRowCount)(env, cls, js("E")), (long long)seen, g_live_local_refs);
  const std::string out = std::string(argv[3]) + "/jni_sorted.csv";
  CHECK(J(Table, nativeWriteCSV)(env, cls, js("S"), js(out)) == 0);
  // ArrowTable.fromBuffers: int64 (with a null), double and string columns from host buffers
  const int64_t iv[4] = {7, 8, 9, 10};
  const uint8_t ivalid = 0b1101;  // row 1 null (LSB first)
  const double dv[4] = {0.5, 1.5, 2.5, 3.5};
  const char sbytes[] = "abbcccdddd";
  const int32_t soff[5] = {0, 1, 3, 6, 10};
  auto *names = mk(new MObjArray);
  names->v = {js("i"), js("d"), js("s")};
  auto *types = mk(new MIntArray);
  types->v = {8, 11, 12};  // INT64, DOUBLE, STRING
  auto *data = mk(new MLongArray), *valid = mk(new MLongArray), *offs = mk(new MLongArray);
  data->v = {(jlong)(intptr_t)iv, (jlong)(intptr_t)dv, (jlong)(intptr_t)sbytes};
  valid->v = {(jlong)(intptr_t)&ivalid, 0, 0};
  offs->v = {0, 0, (jlong)(intptr_t)soff};
  CHECK(J(ArrowTable, nativeFromBuffers)(env, cls, js("T"), names, types, 4, data, valid, offs) == 0);
  std::printf("buffers_rows %lld\nbuffers_cols %d\n", (long long)J(Table, nativeRowCount)(env, cls, js("T")),
              J(Table, nativeColumnCount)(env, cls, js("T")));
  auto *probe = mk(new MPredicate);
  std::string strs;
  double dsum = 0;
  int nulls = 0;
  probe->fn = [&](jlong h) {
    nulls += J(Row, nativeIsNull)(env, cls, h, 0) ? 1 : 0;
    dsum += J(Row, nativeGetDouble)(env, cls, h, 1);
    strs += static_cast<MString *>(J(Row, nativeGetString)(env, cls, h, 2))->s + ",";
    return J(Row, nativeGetDouble)(env, cls, h, 1) > 1.0;
  };
  CHECK(J(Table, nativeSelect)(env, cls, js("T"), probe, js("T2")) == 0);
  std::printf("buffers_nulls %d\nbuffers_dsum_x10 %lld\nbuffers_selected %lld\n", nulls, (long long)(dsum * 10),
              (long long)J(Table, nativeRowCount)(env, cls, js("T2")));
  CHECK(strs == "a,bb,ccc,dddd,");
  // an error surfaces as a code and a message (CylonContext.lastError)
  CHECK(J(Table, nativeJoin)(env, cls, js("A"), js("missing"), 0, 1, 0, 0, 0, js("X")) != 0);
  const std::string err = static_cast<MString *>(J(CylonContext, nativeLastError)(env, cls))->s;
  CHECK(err.find("missing") != std::string::npos);
  for (const char *t : {"A", "B", "J", "JO", "U", "S", "P", "M", "E", "T", "T2"})
    CHECK(J(Table, nativeRemove)(env, cls, js(t)) == 0);
  CHECK(J(CylonContext, nativeFinalize)(env, cls) == 0);
  std::printf("failures %d\n", g_fail);
  return g_fail == 0 ? 0 : 1;
}
