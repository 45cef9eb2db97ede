// msegment_jni.cpp -- JNI shim over the C ABI of include/msegment.h.
// Build (where a JDK exists), one command:
//   g++ -O2 -fPIC -shared -I"$JAVA_HOME/include" -I"$JAVA_HOME/include/linux" -I../../include
//       msegment_jni.cpp -L../msegment -lmsegment -Wl,-rpath,'$ORIGIN' -o libmsegment_jni.so
// Replaces the OpenCV 3.4.2 JNI entry Java_org_opencv_imgproc_Imgproc_watershed_10 reached from
// PictureService.java:909, plus the per-pixel colorByIndexes loop (PictureService.java:913-936),
// and the marker stages of notConnectedMarkers (PictureService.java:476-828) and
// shapeAutoMarkerWatershed (PictureService.java:402-452) and colorAutoMarkerWatershed (:301-366).
//
// Every Java array is checked against the sizes rows/cols/depth imply before anything is read
// (a short array returns MSG_EINVAL instead of letting libmsegment run past it), and the arrays
// are copied with Get/Set<Type>ArrayRegion into native buffers: no critical region is held while
// the GPU works (the flood can take seconds on interrupt-dense frames, and a critical region
// blocks the garbage collector for that long).  tests/test_jni_shim.py compiles this file against
// a JNI type stub and drives it through a mock JNIEnv.
#include <jni.h>

#include <cstdint>
#include <new>
#include <vector>

#include "msegment.h"

namespace {

// rows * cols * k fits the Java array of length `len` (and is representable)
bool fits(JNIEnv* env, jarray a, jint rows, jint cols, long long k) {
  if (!a || rows < 0 || cols < 0) return false;
  return (long long)env->GetArrayLength(a) >= (long long)rows * cols * k;
}

template <class T>
bool alloc(std::vector<T>& v, long long n) {
  try {
    v.resize((size_t)n);
  } catch (const std::bad_alloc&) {
    return false;
  }
  return true;
}

}  // namespace

extern "C" {

JNIEXPORT jlong JNICALL Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_create(JNIEnv*, jclass,
                                                                                          jint device) {
  msg_ctx* c = nullptr;
  return msg_create(&c, device, 0) == MSG_OK ? reinterpret_cast<jlong>(c) : 0;
}

JNIEXPORT void JNICALL Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_destroy(JNIEnv*, jclass,
                                                                                          jlong ctx) {
  msg_destroy(reinterpret_cast<msg_ctx*>(ctx));
}

JNIEXPORT jstring JNICALL Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_lastError(JNIEnv* env,
                                                                                               jclass, jlong ctx) {
  return env->NewStringUTF(msg_last_error(reinterpret_cast<msg_ctx*>(ctx)));
}

// PictureService.watershed (PictureService.java:908-911): markers rewritten in place (labels),
// dst = colorByIndexes(markers, depth, palette != null).
JNIEXPORT jint JNICALL Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_watershedColorize(
    JNIEnv* env, jclass, jlong ctx, jbyteArray bgr, jintArray markers, jint rows, jint cols, jint depth,
    jbyteArray palette, jbyteArray dst) {
  msg_ctx* c = reinterpret_cast<msg_ctx*>(ctx);
  if (!c || depth < 0 || !fits(env, bgr, rows, cols, 3) || !fits(env, markers, rows, cols, 1) ||
      !fits(env, dst, rows, cols, 3) || (palette && env->GetArrayLength(palette) < 3ll * depth))
    return MSG_EINVAL;
  const long long n = (long long)rows * cols;
  std::vector<jbyte> b, d, p;
  std::vector<jint> m;
  if (!alloc(b, 3 * n) || !alloc(m, n) || !alloc(d, 3 * n) || (palette && !alloc(p, 3ll * depth)))
    return MSG_ENOMEM;
  env->GetByteArrayRegion(bgr, 0, (jsize)(3 * n), b.data());
  env->GetIntArrayRegion(markers, 0, (jsize)n, m.data());
  if (palette) env->GetByteArrayRegion(palette, 0, 3 * depth, p.data());
  if (env->ExceptionCheck()) return MSG_EINVAL;
  const int rc = msg_watershed_colorize(c, reinterpret_cast<const uint8_t*>(b.data()), (size_t)cols * 3,
                                        reinterpret_cast<int32_t*>(m.data()), (size_t)cols * 4, rows, cols,
                                        depth, palette ? reinterpret_cast<const uint8_t*>(p.data()) : nullptr,
                                        reinterpret_cast<uint8_t*>(d.data()), (size_t)cols * 3, nullptr, 0);
  if (rc) return rc;
  env->SetIntArrayRegion(markers, 0, (jsize)n, m.data());
  env->SetByteArrayRegion(dst, 0, (jsize)(3 * n), d.data());
  return MSG_OK;
}

// msg_set_batch_floods (msegment.h): 0 = the full engine per flood, 1 / 2 = many floods per launch.
JNIEXPORT jint JNICALL Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_setBatchFloods(JNIEnv*, jclass,
                                                                                                jlong ctx, jint mode) {
  msg_ctx* c = reinterpret_cast<msg_ctx*>(ctx);
  return c ? msg_set_batch_floods(c, mode) : MSG_EINVAL;
}

// msg_set_batch_devices (msegment.h): the batch calls' frames split over a GPU list, block j on
// devices[j] (config 5: one frame stream per GPU); an empty array = the context's own device.
JNIEXPORT jint JNICALL Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_setBatchDevices(
    JNIEnv* env, jclass, jlong ctx, jintArray devices) {
  msg_ctx* c = reinterpret_cast<msg_ctx*>(ctx);
  if (!c || !devices) return MSG_EINVAL;
  const jsize n = env->GetArrayLength(devices);
  if (n > 64) return MSG_EINVAL;
  jint d[64];
  env->GetIntArrayRegion(devices, 0, n, d);
  if (env->ExceptionCheck()) return MSG_EINVAL;
  int v[64];
  for (jsize k = 0; k < n; ++k) v[k] = d[k];
  return msg_set_batch_devices(c, n, n ? v : nullptr);
}

// PictureService.watershed over a batch of frames in one call (the reference's evaluation loop:
// CorrelationTestService.java:84-86, 116, 128, 141 -> PictureService.java:852, 92 floods per
// image): bgrs[k] (byte[]), markers[k] (int[], rewritten in place), dsts[k] (byte[]) of
// rows[k] x cols[k]; one palette (or null = white) and depth for every frame.
JNIEXPORT jint JNICALL Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_watershedColorizeBatch(
    JNIEnv* env, jclass, jlong ctx, jobjectArray bgrs, jobjectArray markers, jintArray rows, jintArray cols,
    jint depth, jbyteArray palette, jobjectArray dsts) {
  msg_ctx* c = reinterpret_cast<msg_ctx*>(ctx);
  if (!c || !bgrs || !markers || !rows || !cols || !dsts || depth < 0) return MSG_EINVAL;
  const jsize n = env->GetArrayLength(bgrs);
  if (env->GetArrayLength(markers) != n || env->GetArrayLength(dsts) != n || env->GetArrayLength(rows) < n ||
      env->GetArrayLength(cols) < n || (palette && env->GetArrayLength(palette) < 3ll * depth))
    return MSG_EINVAL;
  std::vector<jint> R, C;
  if (!alloc(R, n) || !alloc(C, n)) return MSG_ENOMEM;
  env->GetIntArrayRegion(rows, 0, n, R.data());
  env->GetIntArrayRegion(cols, 0, n, C.data());
  if (env->ExceptionCheck()) return MSG_EINVAL;
  std::vector<std::vector<jbyte>> b(n), d(n);
  std::vector<std::vector<jint>> m(n);
  std::vector<jbyte> p;
  if (palette && (!alloc(p, 3ll * depth))) return MSG_ENOMEM;
  if (palette) env->GetByteArrayRegion(palette, 0, 3 * depth, p.data());
  for (jsize k = 0; k < n; ++k) {
    jbyteArray bk = static_cast<jbyteArray>(env->GetObjectArrayElement(bgrs, k));
    jintArray mk = static_cast<jintArray>(env->GetObjectArrayElement(markers, k));
    jbyteArray dk = static_cast<jbyteArray>(env->GetObjectArrayElement(dsts, k));
    const bool ok = fits(env, bk, R[k], C[k], 3) && fits(env, mk, R[k], C[k], 1) && fits(env, dk, R[k], C[k], 3);
    const long long nk = ok ? (long long)R[k] * C[k] : 0;
    const bool mem = ok && alloc(b[k], 3 * nk) && alloc(m[k], nk) && alloc(d[k], 3 * nk);
    if (mem) {
      env->GetByteArrayRegion(bk, 0, (jsize)(3 * nk), b[k].data());
      env->GetIntArrayRegion(mk, 0, (jsize)nk, m[k].data());
    }
    if (bk) env->DeleteLocalRef(bk);
    if (mk) env->DeleteLocalRef(mk);
    if (dk) env->DeleteLocalRef(dk);
    if (!ok) return MSG_EINVAL;
    if (!mem) return MSG_ENOMEM;
  }
  if (env->ExceptionCheck()) return MSG_EINVAL;
  std::vector<const uint8_t*> bp(n);
  std::vector<int32_t*> mp(n);
  std::vector<uint8_t*> dp(n);
  std::vector<size_t> bs(n), ms(n), ds(n);
  for (jsize k = 0; k < n; ++k) {
    bp[k] = reinterpret_cast<const uint8_t*>(b[k].data());
    mp[k] = reinterpret_cast<int32_t*>(m[k].data());
    dp[k] = reinterpret_cast<uint8_t*>(d[k].data());
    bs[k] = ds[k] = (size_t)C[k] * 3;
    ms[k] = (size_t)C[k] * 4;
  }
  const int rc = msg_watershed_colorize_batch(c, n, bp.data(), bs.data(), mp.data(), ms.data(), R.data(), C.data(),
                                              depth, palette ? reinterpret_cast<const uint8_t*>(p.data()) : nullptr,
                                              dp.data(), ds.data());
  if (rc) return rc;
  for (jsize k = 0; k < n; ++k) {
    const long long nk = (long long)R[k] * C[k];
    jintArray mk = static_cast<jintArray>(env->GetObjectArrayElement(markers, k));
    jbyteArray dk = static_cast<jbyteArray>(env->GetObjectArrayElement(dsts, k));
    env->SetIntArrayRegion(mk, 0, (jsize)nk, m[k].data());
    env->SetByteArrayRegion(dk, 0, (jsize)(3 * nk), d[k].data());
    env->DeleteLocalRef(mk);
    env->DeleteLocalRef(dk);
  }
  return env->ExceptionCheck() ? MSG_EINVAL : MSG_OK;
}

// notConnectedMarkers' marker stage (PictureService.java:476-828): markers out, levels as
// {start, end, count} triples into levelsOut (3 * 256 ints).  Returns the level count or a
// negative MSG_E* code.
JNIEXPORT jint JNICALL Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_ncMarkers(
    JNIEnv* env, jclass, jlong ctx, jbyteArray bgr, jint rows, jint cols, jint depth, jint options,
    jintArray markers, jintArray levelsOut) {
  msg_ctx* c = reinterpret_cast<msg_ctx*>(ctx);
  if (!c || !levelsOut || env->GetArrayLength(levelsOut) < 3 * 256 || !fits(env, bgr, rows, cols, 3) ||
      !fits(env, markers, rows, cols, 1))
    return MSG_EINVAL;
  const long long n = (long long)rows * cols;
  std::vector<jbyte> b;
  std::vector<jint> m;
  if (!alloc(b, 3 * n) || !alloc(m, n)) return MSG_ENOMEM;
  env->GetByteArrayRegion(bgr, 0, (jsize)(3 * n), b.data());
  if (env->ExceptionCheck()) return MSG_EINVAL;
  msg_bright_level lv[256];
  int nl = 0;
  const int rc = msg_nc_marker_stage(c, reinterpret_cast<const uint8_t*>(b.data()), (size_t)cols * 3, rows,
                                     cols, depth, (unsigned)options, reinterpret_cast<int32_t*>(m.data()),
                                     (size_t)cols * 4, lv, 256, &nl);
  if (rc) return rc;
  jint tri[3 * 256];
  for (int i = 0; i < nl; ++i) {
    tri[3 * i] = lv[i].start;
    tri[3 * i + 1] = lv[i].end;
    tri[3 * i + 2] = lv[i].count;
  }
  env->SetIntArrayRegion(markers, 0, (jsize)n, m.data());
  env->SetIntArrayRegion(levelsOut, 0, 3 * nl, tri);
  return nl;
}

// shapeAutoMarkerWatershed's marker stage (PictureService.java:402-452): markers out (the
// connectedComponents labels), returns the RETR_CCOMP contour count (the watershed depth; 0 =
// no contour, where the reference returns null) or a negative MSG_E* code.
JNIEXPORT jint JNICALL Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_shapeMarkers(
    JNIEnv* env, jclass, jlong ctx, jbyteArray bgr, jint rows, jint cols, jintArray markers) {
  msg_ctx* c = reinterpret_cast<msg_ctx*>(ctx);
  if (!c || !fits(env, bgr, rows, cols, 3) || !fits(env, markers, rows, cols, 1)) return MSG_EINVAL;
  const long long n = (long long)rows * cols;
  std::vector<jbyte> b;
  std::vector<jint> m;
  if (!alloc(b, 3 * n) || !alloc(m, n)) return MSG_ENOMEM;
  env->GetByteArrayRegion(bgr, 0, (jsize)(3 * n), b.data());
  if (env->ExceptionCheck()) return MSG_EINVAL;
  int depth = 0, ncomp = 0;
  const int rc = msg_shape_markers(c, reinterpret_cast<const uint8_t*>(b.data()), (size_t)cols * 3, rows, cols,
                                   0, reinterpret_cast<int32_t*>(m.data()), (size_t)cols * 4, &depth, &ncomp);
  if (rc) return rc;
  env->SetIntArrayRegion(markers, 0, (jsize)n, m.data());
  return depth;
}

// colorAutoMarkerWatershed's marker stage (PictureService.java:301-366): the sharpened image (the
// src the reference then floods, :333) and the markers out, returns the contour count (the
// watershed depth) or a negative MSG_E* code.
JNIEXPORT jint JNICALL Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_colorMarkers(
    JNIEnv* env, jclass, jlong ctx, jbyteArray bgr, jint rows, jint cols, jbyteArray sharp, jintArray markers) {
  msg_ctx* c = reinterpret_cast<msg_ctx*>(ctx);
  if (!c || !fits(env, bgr, rows, cols, 3) || !fits(env, sharp, rows, cols, 3) || !fits(env, markers, rows, cols, 1))
    return MSG_EINVAL;
  const long long n = (long long)rows * cols;
  std::vector<jbyte> b, sh;
  std::vector<jint> m;
  if (!alloc(b, 3 * n) || !alloc(sh, 3 * n) || !alloc(m, n)) return MSG_ENOMEM;
  env->GetByteArrayRegion(bgr, 0, (jsize)(3 * n), b.data());
  if (env->ExceptionCheck()) return MSG_EINVAL;
  int depth = 0;
  const int rc = msg_color_markers(c, reinterpret_cast<const uint8_t*>(b.data()), (size_t)cols * 3, rows, cols,
                                   reinterpret_cast<uint8_t*>(sh.data()), (size_t)cols * 3,
                                   reinterpret_cast<int32_t*>(m.data()), (size_t)cols * 4, &depth);
  if (rc) return rc;
  env->SetByteArrayRegion(sharp, 0, (jsize)(3 * n), sh.data());
  env->SetIntArrayRegion(markers, 0, (jsize)n, m.data());
  return depth;
}

}  // extern "C"
