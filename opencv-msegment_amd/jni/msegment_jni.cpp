// msegment_jni.cpp -- JNI shim over the C ABI of include/msegment.h.
// Build (where a JDK exists):
//   g++ -O2 -fPIC -shared -I"$JAVA_HOME/include" -I"$JAVA_HOME/include/linux" -I../../include \
//       msegment_jni.cpp -L../msegment -lmsegment -Wl,-rpath,'$ORIGIN' -o libmsegment_jni.so
// Replaces the OpenCV 3.4.2 JNI entry Java_org_opencv_imgproc_Imgproc_watershed_10 reached from
// PictureService.java:909, plus the per-pixel colorByIndexes loop (PictureService.java:913-936),
// and the marker stage of notConnectedMarkers (PictureService.java:476-828).
#include <jni.h>

#include "msegment.h"

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

JNIEXPORT jint JNICALL Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_watershedColorize(
    JNIEnv* env, jclass, jlong ctx, jbyteArray bgr, jintArray markers, jint rows, jint cols, jint depth,
    jbyteArray palette, jbyteArray dst) {
  msg_ctx* c = reinterpret_cast<msg_ctx*>(ctx);
  if (!c) return MSG_EINVAL;
  // pinned (critical) views: no per-pixel JNI traffic, one H2D/D2H per buffer inside libmsegment
  jbyte* pb = static_cast<jbyte*>(env->GetPrimitiveArrayCritical(bgr, nullptr));
  jint* pm = static_cast<jint*>(env->GetPrimitiveArrayCritical(markers, nullptr));
  jbyte* pd = static_cast<jbyte*>(env->GetPrimitiveArrayCritical(dst, nullptr));
  jbyte* pp = palette ? static_cast<jbyte*>(env->GetPrimitiveArrayCritical(palette, nullptr)) : nullptr;
  int rc = MSG_EINVAL;
  if (pb && pm && pd)
    rc = msg_watershed_colorize(c, reinterpret_cast<const uint8_t*>(pb), (size_t)cols * 3,
                                reinterpret_cast<int32_t*>(pm), (size_t)cols * 4, rows, cols, depth,
                                reinterpret_cast<const uint8_t*>(pp), reinterpret_cast<uint8_t*>(pd),
                                (size_t)cols * 3, nullptr, 0);
  if (pp) env->ReleasePrimitiveArrayCritical(palette, pp, JNI_ABORT);
  if (pd) env->ReleasePrimitiveArrayCritical(dst, pd, 0);
  if (pm) env->ReleasePrimitiveArrayCritical(markers, pm, 0);
  if (pb) env->ReleasePrimitiveArrayCritical(bgr, pb, JNI_ABORT);
  return rc;
}

// notConnectedMarkers' marker stage (PictureService.java:476-828): markers out, levels as
// {start, end, count} triples into levelsOut (3 * 256 ints).  Returns the level count or a
// negative MSG_E* code.
JNIEXPORT jint JNICALL Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_ncMarkers(
    JNIEnv* env, jclass, jlong ctx, jbyteArray bgr, jint rows, jint cols, jint depth, jint options,
    jintArray markers, jintArray levelsOut) {
  msg_ctx* c = reinterpret_cast<msg_ctx*>(ctx);
  if (!c || env->GetArrayLength(levelsOut) < 3 * 256) return MSG_EINVAL;
  msg_bright_level lv[256];
  int n = 0;
  jbyte* pb = static_cast<jbyte*>(env->GetPrimitiveArrayCritical(bgr, nullptr));
  jint* pm = static_cast<jint*>(env->GetPrimitiveArrayCritical(markers, nullptr));
  int rc = MSG_EINVAL;
  if (pb && pm)
    rc = msg_nc_marker_stage(c, reinterpret_cast<const uint8_t*>(pb), (size_t)cols * 3, rows, cols,
                             depth, (unsigned)options, reinterpret_cast<int32_t*>(pm),
                             (size_t)cols * 4, lv, 256, &n);
  if (pm) env->ReleasePrimitiveArrayCritical(markers, pm, 0);
  if (pb) env->ReleasePrimitiveArrayCritical(bgr, pb, JNI_ABORT);
  if (rc) return rc;
  jint tri[3 * 256];
  for (int i = 0; i < n; ++i) {
    tri[3 * i] = lv[i].start;
    tri[3 * i + 1] = lv[i].end;
    tri[3 * i + 2] = lv[i].count;
  }
  env->SetIntArrayRegion(levelsOut, 0, 3 * n, tri);
  return n;
}

// shapeAutoMarkerWatershed's marker stage (PictureService.java:402-452): markers out (the
// connectedComponents labels), returns the RETR_CCOMP contour count (the watershed depth; 0 =
// no contour, where the reference returns null) or a negative MSG_E* code.
JNIEXPORT jint JNICALL Java_ru_shayhulud_opencvcmsegment_nativeseg_MSegmentNative_shapeMarkers(
    JNIEnv* env, jclass, jlong ctx, jbyteArray bgr, jint rows, jint cols, jintArray markers) {
  msg_ctx* c = reinterpret_cast<msg_ctx*>(ctx);
  if (!c) return MSG_EINVAL;
  int depth = 0, ncomp = 0;
  jbyte* pb = static_cast<jbyte*>(env->GetPrimitiveArrayCritical(bgr, nullptr));
  jint* pm = static_cast<jint*>(env->GetPrimitiveArrayCritical(markers, nullptr));
  int rc = MSG_EINVAL;
  if (pb && pm)
    rc = msg_shape_markers(c, reinterpret_cast<const uint8_t*>(pb), (size_t)cols * 3, rows, cols, 0,
                           reinterpret_cast<int32_t*>(pm), (size_t)cols * 4, &depth, &ncomp);
  if (pm) env->ReleasePrimitiveArrayCritical(markers, pm, 0);
  if (pb) env->ReleasePrimitiveArrayCritical(bgr, pb, JNI_ABORT);
  return rc ? rc : depth;
}

}  // extern "C"
