// JNI layer of the Java API (J2).  Reference: java/src/main/native/src/Table.cpp:26-141,
// ArrowTable.cpp:185-270, Row.cpp:12-81, TwisterXContext.cpp:20-48 (JNI over the string-ID
// table registry).  Here every call forwards to the C ABI in cylon_amd/include/cylon_capi.h.
// Build: java/build.sh (needs a JDK for jni.h; none ships in the development image).
#include <jni.h>

#include <string>
#include <vector>

#include "../../../../cylon_amd/include/cylon_capi.h"

namespace {
struct JStr {
  JNIEnv *env;
  jstring js;
  const char *c;
  JStr(JNIEnv *e, jstring s) : env(e), js(s), c(s ? e->GetStringUTFChars(s, nullptr) : nullptr) {}
  ~JStr() {
    if (c) env->ReleaseStringUTFChars(js, c);
  }
};

struct SelectCtx {
  JNIEnv *env;
  jobject pred;
  jclass row_cls;
  jmethodID row_ctor, test;
};

int select_trampoline(const cylon_row *row, void *user) {
  auto *s = static_cast<SelectCtx *>(user);
  jobject r = s->env->NewObject(s->row_cls, s->row_ctor, (jlong) reinterpret_cast<intptr_t>(row));
  const jboolean keep = s->env->CallBooleanMethod(s->pred, s->test, r);
  s->env->DeleteLocalRef(r);
  return keep ? 1 : 0;
}
}  // namespace

#define JFN(cls, name) JNICALL Java_org_cylonamd_##cls##_##name

extern "C" {

// ---- CylonContext
JNIEXPORT jint JFN(CylonContext, nativeInit)(JNIEnv *env, jclass, jstring dev) {
  JStr d(env, dev);
  return cylon_init(d.c);
}
JNIEXPORT jint JFN(CylonContext, nativeInitDistributed)(JNIEnv *env, jclass, jstring comm) {
  JStr c(env, comm);
  return cylon_init_distributed(c.c);
}
JNIEXPORT jint JFN(CylonContext, nativeRank)(JNIEnv *, jclass) { return cylon_get_rank(); }
JNIEXPORT jint JFN(CylonContext, nativeWorldSize)(JNIEnv *, jclass) { return cylon_get_world_size(); }
JNIEXPORT jint JFN(CylonContext, nativeBarrier)(JNIEnv *, jclass) { return cylon_barrier(); }
JNIEXPORT jint JFN(CylonContext, nativeFinalize)(JNIEnv *, jclass) { return cylon_finalize(); }
JNIEXPORT jstring JFN(CylonContext, nativeLastError)(JNIEnv *env, jclass) {
  return env->NewStringUTF(cylon_last_error());
}

// ---- Table
JNIEXPORT jint JFN(Table, nativeReadCSV)(JNIEnv *env, jclass, jstring path, jstring id) {
  JStr p(env, path), i(env, id);
  return cylon_read_csv(p.c, i.c);
}
JNIEXPORT jint JFN(Table, nativeWriteCSV)(JNIEnv *env, jclass, jstring id, jstring path) {
  JStr i(env, id), p(env, path);
  return cylon_write_csv(i.c, p.c);
}
JNIEXPORT jlong JFN(Table, nativeRowCount)(JNIEnv *env, jclass, jstring id) {
  JStr i(env, id);
  return cylon_row_count(i.c);
}
JNIEXPORT jint JFN(Table, nativeColumnCount)(JNIEnv *env, jclass, jstring id) {
  JStr i(env, id);
  return cylon_column_count(i.c);
}
JNIEXPORT jint JFN(Table, nativeJoin)(JNIEnv *env, jclass, jstring l, jstring r, jint type, jint alg, jint lc,
                                      jint rc, jboolean dist, jstring out) {
  JStr a(env, l), b(env, r), o(env, out);
  return dist ? cylon_distributed_join(a.c, b.c, type, alg, lc, rc, o.c) : cylon_join(a.c, b.c, type, alg, lc, rc, o.c);
}
JNIEXPORT jint JFN(Table, nativeSetOp)(JNIEnv *env, jclass, jstring a, jstring b, jint op, jboolean dist,
                                       jstring out) {
  JStr x(env, a), y(env, b), o(env, out);
  return cylon_set_op(x.c, y.c, op, dist ? 1 : 0, o.c);
}
JNIEXPORT jint JFN(Table, nativeSort)(JNIEnv *env, jclass, jstring id, jint col, jboolean asc, jstring out) {
  JStr i(env, id), o(env, out);
  return cylon_sort(i.c, col, asc ? 1 : 0, o.c);
}
JNIEXPORT jint JFN(Table, nativeProject)(JNIEnv *env, jclass, jstring id, jintArray cols, jstring out) {
  JStr i(env, id), o(env, out);
  const jsize n = env->GetArrayLength(cols);
  std::vector<int32_t> c(n);
  env->GetIntArrayRegion(cols, 0, n, reinterpret_cast<jint *>(c.data()));
  return cylon_project(i.c, c.data(), (int)n, o.c);
}
JNIEXPORT jint JFN(Table, nativeMerge)(JNIEnv *env, jclass, jobjectArray ids, jstring out) {
  const jsize n = env->GetArrayLength(ids);
  std::vector<std::string> s(n);
  std::vector<const char *> p(n);
  for (jsize k = 0; k < n; ++k) {
    JStr j(env, (jstring)env->GetObjectArrayElement(ids, k));
    s[k] = j.c;
    p[k] = s[k].c_str();
  }
  JStr o(env, out);
  return cylon_merge(p.data(), (int)n, o.c);
}
JNIEXPORT jint JFN(Table, nativeSelect)(JNIEnv *env, jclass, jstring id, jobject pred, jstring out) {
  JStr i(env, id), o(env, out);
  SelectCtx s{env, pred, env->FindClass("org/cylonamd/Row"), nullptr, nullptr};
  s.row_ctor = env->GetMethodID(s.row_cls, "<init>", "(J)V");
  s.test = env->GetMethodID(env->GetObjectClass(pred), "test", "(Ljava/lang/Object;)Z");
  return cylon_select(i.c, &select_trampoline, &s, o.c);
}
JNIEXPORT jint JFN(Table, nativePrint)(JNIEnv *env, jclass, jstring id, jlong from, jlong to) {
  JStr i(env, id);
  return cylon_print(i.c, from, to);
}
JNIEXPORT jint JFN(Table, nativeRemove)(JNIEnv *env, jclass, jstring id) {
  JStr i(env, id);
  return cylon_remove_table(i.c);
}

// ---- Row (handle valid during a select predicate)
static const cylon_row *R(jlong h) { return reinterpret_cast<const cylon_row *>((intptr_t)h); }
JNIEXPORT jlong JFN(Row, nativeIndex)(JNIEnv *, jclass, jlong h) { return cylon_row_index(R(h)); }
JNIEXPORT jboolean JFN(Row, nativeIsNull)(JNIEnv *, jclass, jlong h, jint c) { return cylon_row_is_null(R(h), c) != 0; }
JNIEXPORT jlong JFN(Row, nativeGetInt64)(JNIEnv *, jclass, jlong h, jint c) { return cylon_row_get_int64(R(h), c); }
JNIEXPORT jdouble JFN(Row, nativeGetDouble)(JNIEnv *, jclass, jlong h, jint c) {
  return cylon_row_get_double(R(h), c);
}
JNIEXPORT jstring JFN(Row, nativeGetString)(JNIEnv *env, jclass, jlong h, jint c) {
  const int64_t len = cylon_row_get_string(R(h), c, nullptr, 0);
  std::string s((size_t)len + 1, '\0');
  cylon_row_get_string(R(h), c, &s[0], len + 1);
  s.resize((size_t)len);
  return env->NewStringUTF(s.c_str());
}

// ---- ArrowTable
JNIEXPORT jint JFN(ArrowTable, nativeFromBuffers)(JNIEnv *env, jclass, jstring id, jobjectArray names,
                                                  jintArray types, jlong rows, jlongArray data, jlongArray validity,
                                                  jlongArray offsets) {
  JStr i(env, id);
  const jsize n = env->GetArrayLength(names);
  std::vector<std::string> ns(n);
  std::vector<const char *> np(n);
  for (jsize k = 0; k < n; ++k) {
    JStr j(env, (jstring)env->GetObjectArrayElement(names, k));
    ns[k] = j.c;
    np[k] = ns[k].c_str();
  }
  std::vector<int32_t> t(n);
  env->GetIntArrayRegion(types, 0, n, reinterpret_cast<jint *>(t.data()));
  std::vector<jlong> d(n), v(n), o(n);
  env->GetLongArrayRegion(data, 0, n, d.data());
  env->GetLongArrayRegion(validity, 0, n, v.data());
  env->GetLongArrayRegion(offsets, 0, n, o.data());
  std::vector<const void *> dp(n);
  std::vector<const uint8_t *> vp(n);
  std::vector<const int32_t *> op(n);
  for (jsize k = 0; k < n; ++k) {
    dp[k] = reinterpret_cast<const void *>((intptr_t)d[k]);
    vp[k] = reinterpret_cast<const uint8_t *>((intptr_t)v[k]);
    op[k] = reinterpret_cast<const int32_t *>((intptr_t)o[k]);
  }
  return cylon_table_from_buffers(i.c, (int)n, np.data(), t.data(), rows, dp.data(), vp.data(), op.data());
}

}  // extern "C"
