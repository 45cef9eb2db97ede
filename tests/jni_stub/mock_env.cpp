// Test-only mock JVM for the JNI shim (tests/test_jni_shim.py): Java arrays are std::vectors,
// region copies are bounds-checked like the JVM's (an out-of-range copy raises a pending
// exception instead of touching memory), critical regions are counted so the test can assert
// the shim never holds one across a library call.
//   mock_env validate            -- argument checks only (no GPU): every bad call -> MSG_EINVAL
//   mock_env run <in> <out>      -- one watershedColorize through the shim on GPU 0
//   mock_env batch <mode> <in> <out> [d0,d1,..] -- watershedColorizeBatch of the frames in <in> (batch
//                                    floods mode), optionally spread over a device list (setBatchDevices)
#include <jni.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "msegment.h"

extern "C" {
jint Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_watershedColorize(
    JNIEnv*, jclass, jlong, jbyteArray, jintArray, jint, jint, jint, jbyteArray, jbyteArray);
jint Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_ncMarkers(JNIEnv*, jclass, jlong, jbyteArray,
                                                                          jint, jint, jint, jint, jintArray,
                                                                          jintArray);
jint Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_shapeMarkers(JNIEnv*, jclass, jlong,
                                                                             jbyteArray, jint, jint, jintArray);
jint Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_colorMarkers(JNIEnv*, jclass, jlong, jbyteArray,
                                                                             jint, jint, jbyteArray, jintArray);
jint Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_setBatchFloods(JNIEnv*, jclass, jlong, jint);
jint Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_setBatchDevices(JNIEnv*, jclass, jlong, jintArray);
jint Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_watershedColorizeBatch(
    JNIEnv*, jclass, jlong, jobjectArray, jobjectArray, jintArray, jintArray, jint, jbyteArray, jobjectArray);
}

struct Bytes : _jbyteArray {
  std::vector<jbyte> v;
  explicit Bytes(size_t n) : v(n) {}
};
struct Ints : _jintArray {
  std::vector<jint> v;
  explicit Ints(size_t n) : v(n) {}
};
struct Objs : _jobjectArray {
  std::vector<jobject> v;
};

static bool g_exc = false;
static int g_critical = 0;
// arrays carry their kind in a side table (the stub classes are not polymorphic)
static std::vector<std::pair<const void*, size_t>> g_len;
static void reg(const void* a, size_t n) { g_len.push_back({a, n}); }
jsize JNIEnv_::GetArrayLength(jarray a) {
  for (auto& e : g_len)
    if (e.first == a) return (jsize)e.second;
  return 0;
}
template <class A, class T>
static void get_region(A* a, jsize start, jsize len, T* buf) {
  if (start < 0 || len < 0 || (size_t)start + len > a->v.size()) {
    g_exc = true;
    return;
  }
  std::memcpy(buf, a->v.data() + start, sizeof(T) * len);
}
template <class A, class T>
static void set_region(A* a, jsize start, jsize len, const T* buf) {
  if (start < 0 || len < 0 || (size_t)start + len > a->v.size()) {
    g_exc = true;
    return;
  }
  std::memcpy(a->v.data() + start, buf, sizeof(T) * len);
}
void JNIEnv_::GetByteArrayRegion(jbyteArray a, jsize s, jsize n, jbyte* b) { get_region(static_cast<Bytes*>(a), s, n, b); }
void JNIEnv_::SetByteArrayRegion(jbyteArray a, jsize s, jsize n, const jbyte* b) { set_region(static_cast<Bytes*>(a), s, n, b); }
void JNIEnv_::GetIntArrayRegion(jintArray a, jsize s, jsize n, jint* b) { get_region(static_cast<Ints*>(a), s, n, b); }
void JNIEnv_::SetIntArrayRegion(jintArray a, jsize s, jsize n, const jint* b) { set_region(static_cast<Ints*>(a), s, n, b); }
jstring JNIEnv_::NewStringUTF(const char*) { return nullptr; }
jboolean JNIEnv_::ExceptionCheck() { return g_exc ? 1 : 0; }
void* JNIEnv_::GetPrimitiveArrayCritical(jarray, jboolean*) {
  ++g_critical;
  return nullptr;
}
void JNIEnv_::ReleasePrimitiveArrayCritical(jarray, void*, jint) {}
static int g_refs = 0;  // local references handed out and not deleted
jobject JNIEnv_::GetObjectArrayElement(jobjectArray a, jsize i) {
  Objs* o = static_cast<Objs*>(a);
  if (i < 0 || (size_t)i >= o->v.size()) {
    g_exc = true;
    return nullptr;
  }
  if (o->v[i]) ++g_refs;
  return o->v[i];
}
void JNIEnv_::DeleteLocalRef(jobject r) {
  if (r) --g_refs;
}

static Bytes* bytes(size_t n) {
  Bytes* b = new Bytes(n);
  reg(static_cast<jarray>(b), n);
  return b;
}
static Ints* ints(size_t n) {
  Ints* a = new Ints(n);
  reg(static_cast<jarray>(a), n);
  return a;
}
static Objs* objs(std::vector<jobject> v) {
  Objs* o = new Objs;
  o->v = std::move(v);
  reg(static_cast<jarray>(o), o->v.size());
  return o;
}
static Ints* ints_of(std::vector<jint> v) {
  Ints* a = ints(v.size());
  a->v = std::move(v);
  return a;
}

static int validate() {
  JNIEnv env;
  jlong fake = 0x1000;  // never dereferenced: every call below must fail its argument checks first
  const int R = 6, C = 5, N = R * C;
  int bad = 0;
  auto expect = [&](int got, const char* what) {
    if (got != MSG_EINVAL) {
      std::printf("FAIL %s: %d\n", what, got);
      ++bad;
    }
  };
  expect(Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_watershedColorize(
             &env, nullptr, 0, bytes(3 * N), ints(N), R, C, 2, nullptr, bytes(3 * N)), "null ctx");
  expect(Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_watershedColorize(
             &env, nullptr, fake, bytes(3 * N - 1), ints(N), R, C, 2, nullptr, bytes(3 * N)), "short bgr");
  expect(Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_watershedColorize(
             &env, nullptr, fake, bytes(3 * N), ints(N - 1), R, C, 2, nullptr, bytes(3 * N)), "short markers");
  expect(Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_watershedColorize(
             &env, nullptr, fake, bytes(3 * N), ints(N), R, C, 2, nullptr, bytes(3 * N - 3)), "short dst");
  expect(Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_watershedColorize(
             &env, nullptr, fake, bytes(3 * N), ints(N), R, C, 4, bytes(11), bytes(3 * N)), "short palette");
  expect(Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_watershedColorize(
             &env, nullptr, fake, bytes(3 * N), ints(N), -R, C, 2, nullptr, bytes(3 * N)), "negative rows");
  expect(Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_watershedColorize(
             &env, nullptr, fake, bytes(3 * N), ints(N), R, C, -1, nullptr, bytes(3 * N)), "negative depth");
  expect(Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_watershedColorize(
             &env, nullptr, fake, bytes(3 * N), ints(N), 1 << 20, 1 << 20, 2, nullptr, bytes(3 * N)), "huge frame");
  expect(Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_ncMarkers(
             &env, nullptr, fake, bytes(3 * N), R, C, 4, 0, ints(N), ints(3 * 256 - 1)), "nc short levels");
  expect(Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_ncMarkers(
             &env, nullptr, fake, bytes(3 * N), R, C, 4, 0, ints(N - 1), ints(3 * 256)), "nc short markers");
  expect(Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_shapeMarkers(
             &env, nullptr, fake, bytes(3 * N - 2), R, C, ints(N)), "shape short bgr");
  expect(Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_shapeMarkers(
             &env, nullptr, fake, bytes(3 * N), R, C, nullptr), "shape null markers");
  expect(Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_colorMarkers(
             &env, nullptr, fake, bytes(3 * N), R, C, bytes(3 * N - 1), ints(N)), "color short sharp");
  expect(Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_colorMarkers(
             &env, nullptr, fake, bytes(3 * N), R, C, bytes(3 * N), ints(N - 1)), "color short markers");
  // the batch entry: mismatched array counts, a short frame array, a negative depth
  auto batch = [&](jlong cx, Objs* b, Objs* m, Ints* r, Ints* c, jint depth, Bytes* pal, Objs* d) {
    return Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_watershedColorizeBatch(&env, nullptr, cx, b, m, r,
                                                                                             c, depth, pal, d);
  };
  auto frames = [&](int n, size_t nb, size_t nm, size_t nd) {
    std::vector<jobject> b, m, d;
    for (int k = 0; k < n; ++k) {
      b.push_back(bytes(nb));
      m.push_back(ints(nm));
      d.push_back(bytes(nd));
    }
    return std::vector<Objs*>{objs(b), objs(m), objs(d)};
  };
  {
    auto f = frames(2, 3 * N, N, 3 * N);
    expect(batch(0, f[0], f[1], ints_of({R, R}), ints_of({C, C}), 2, nullptr, f[2]), "batch null ctx");
    expect(batch(fake, f[0], f[1], ints_of({R}), ints_of({C, C}), 2, nullptr, f[2]), "batch short rows");
    expect(batch(fake, f[0], f[1], ints_of({R, R}), ints_of({C, C}), -1, nullptr, f[2]), "batch negative depth");
    expect(batch(fake, f[0], f[1], ints_of({R, R}), ints_of({C, C}), 4, bytes(11), f[2]), "batch short palette");
    auto g = frames(3, 3 * N, N, 3 * N);
    expect(batch(fake, f[0], g[1], ints_of({R, R}), ints_of({C, C}), 2, nullptr, f[2]), "batch count mismatch");
    auto h = frames(2, 3 * N, N - 1, 3 * N);
    expect(batch(fake, h[0], h[1], ints_of({R, R}), ints_of({C, C}), 2, nullptr, h[2]), "batch short markers");
    auto e = frames(2, 3 * N, N, 3 * N - 1);
    expect(batch(fake, e[0], e[1], ints_of({R, R}), ints_of({C, C}), 2, nullptr, e[2]), "batch short dst");
    Objs* holes = objs({bytes(3 * N), nullptr});
    expect(batch(fake, holes, f[1], ints_of({R, R}), ints_of({C, C}), 2, nullptr, f[2]), "batch null frame");
  }
  expect(Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_setBatchFloods(&env, nullptr, 0, 1),
         "batch floods null ctx");
  expect(Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_setBatchDevices(&env, nullptr, 0, ints_of({0})),
         "batch devices null ctx");
  expect(Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_setBatchDevices(&env, nullptr, fake, nullptr),
         "batch devices null list");
  expect(Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_setBatchDevices(&env, nullptr, fake,
                                                                                     ints_of(std::vector<jint>(65, 0))),
         "batch devices 65 entries");
  if (g_critical) {
    std::printf("FAIL critical regions taken: %d\n", g_critical);
    ++bad;
  }
  if (g_refs) {
    std::printf("FAIL local references leaked: %d\n", g_refs);
    ++bad;
  }
  std::printf("%s (%d bad)\n", bad ? "validate FAILED" : "validate ok", bad);
  return bad ? 1 : 0;
}

// in: int32 rows, cols, depth, has_palette; rows*cols*3 BGR bytes; rows*cols int32 markers;
// [depth*3 palette bytes].  out: rc, then the markers and the dst bytes.
static int run(const char* in, const char* out) {
  FILE* f = std::fopen(in, "rb");
  if (!f) return 2;
  int32_t hdr[4];
  if (std::fread(hdr, 4, 4, f) != 4) return 2;
  const int R = hdr[0], C = hdr[1], depth = hdr[2];
  const size_t N = (size_t)R * C;
  Bytes* bgr = bytes(3 * N);
  Ints* mk = ints(N);
  Bytes* dst = bytes(3 * N);
  Bytes* pal = hdr[3] ? bytes(3 * (size_t)depth) : nullptr;
  if (std::fread(bgr->v.data(), 1, 3 * N, f) != 3 * N || std::fread(mk->v.data(), 4, N, f) != N) return 2;
  if (pal && std::fread(pal->v.data(), 1, 3 * (size_t)depth, f) != 3 * (size_t)depth) return 2;
  std::fclose(f);
  msg_ctx* c = nullptr;
  if (msg_create(&c, 0, 0) != MSG_OK) return 3;
  JNIEnv env;
  const jint rc = Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_watershedColorize(
      &env, nullptr, reinterpret_cast<jlong>(c), bgr, mk, R, C, depth, pal, dst);
  msg_destroy(c);
  FILE* g = std::fopen(out, "wb");
  std::fwrite(&rc, 4, 1, g);
  std::fwrite(mk->v.data(), 4, N, g);
  std::fwrite(dst->v.data(), 1, 3 * N, g);
  std::fclose(g);
  std::printf("run rc=%d critical=%d exc=%d\n", rc, g_critical, (int)g_exc);
  return (g_critical || g_exc) ? 4 : 0;
}

// in: int32 n, depth, has_palette; [depth*3 palette bytes]; n x {int32 rows, cols; BGR bytes;
// int32 markers}.  out: rc, then per frame the markers and the dst bytes.
static int run_batch(int mode, const char* in, const char* out, const char* devs) {
  FILE* f = std::fopen(in, "rb");
  if (!f) return 2;
  int32_t hdr[3];
  if (std::fread(hdr, 4, 3, f) != 3) return 2;
  const int n = hdr[0], depth = hdr[1];
  Bytes* pal = hdr[2] ? bytes(3 * (size_t)depth) : nullptr;
  if (pal && std::fread(pal->v.data(), 1, 3 * (size_t)depth, f) != 3 * (size_t)depth) return 2;
  std::vector<jobject> b, m, d;
  std::vector<jint> rv, cv;
  for (int k = 0; k < n; ++k) {
    int32_t rc2[2];
    if (std::fread(rc2, 4, 2, f) != 2) return 2;
    const size_t N = (size_t)rc2[0] * rc2[1];
    Bytes* bk = bytes(3 * N);
    Ints* mk = ints(N);
    if (std::fread(bk->v.data(), 1, 3 * N, f) != 3 * N || std::fread(mk->v.data(), 4, N, f) != N) return 2;
    b.push_back(bk);
    m.push_back(mk);
    d.push_back(bytes(3 * N));
    rv.push_back(rc2[0]);
    cv.push_back(rc2[1]);
  }
  std::fclose(f);
  msg_ctx* c = nullptr;
  if (msg_create(&c, 0, 0) != MSG_OK) return 3;
  JNIEnv env;
  const jlong cx = reinterpret_cast<jlong>(c);
  jint rc = Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_setBatchFloods(&env, nullptr, cx, mode);
  if (rc == MSG_OK && devs) {  // "0,0": MSegmentNative.watershedBatch(..., new int[]{0, 0})
    std::vector<jint> dv;
    for (const char* p = devs; *p;) {
      char* e = nullptr;
      const long v = std::strtol(p, &e, 10);
      if (e == p) break;
      dv.push_back((jint)v);
      p = (*e == ',') ? e + 1 : e;
    }
    rc = Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_setBatchDevices(&env, nullptr, cx, ints_of(dv));
  }
  Objs* ob = objs(b);
  Objs* om = objs(m);
  Objs* od = objs(d);
  if (rc == MSG_OK)
    rc = Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_watershedColorizeBatch(
        &env, nullptr, cx, ob, om, ints_of(rv), ints_of(cv), depth, pal, od);
  msg_destroy(c);
  FILE* g = std::fopen(out, "wb");
  std::fwrite(&rc, 4, 1, g);
  for (int k = 0; k < n; ++k) {
    std::fwrite(static_cast<Ints*>(m[k])->v.data(), 4, static_cast<Ints*>(m[k])->v.size(), g);
    std::fwrite(static_cast<Bytes*>(d[k])->v.data(), 1, static_cast<Bytes*>(d[k])->v.size(), g);
  }
  std::fclose(g);
  std::printf("batch rc=%d critical=%d exc=%d refs=%d\n", rc, g_critical, (int)g_exc, g_refs);
  return (g_critical || g_exc || g_refs) ? 4 : 0;
}

int main(int argc, char** argv) {
  if (argc >= 2 && std::string(argv[1]) == "validate") return validate();
  if (argc >= 4 && std::string(argv[1]) == "run") return run(argv[2], argv[3]);
  if (argc >= 5 && std::string(argv[1]) == "batch")
    return run_batch(std::atoi(argv[2]), argv[3], argv[4], argc >= 6 ? argv[5] : nullptr);
  std::fprintf(stderr, "usage: mock_env validate | run <in> <out> | batch <mode> <in> <out> [devices]\n");
  return 2;
}
