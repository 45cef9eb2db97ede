package ru.shayhulud.opencvcmsegment.nativeseg;

import org.opencv.core.CvException;
import org.opencv.core.CvType;
import org.opencv.core.Mat;

/**
 * Java side of the libmsegment drop-in (see INTEGRATION.md).  Replaces the body of
 * PictureService.watershed (PictureService.java:908-911):
 * Imgproc.watershed (PictureService.java:909) + colorByIndexes (PictureService.java:913-936).
 * Bulk copies (one Mat.get / Mat.put per buffer) replace the reference's 2*H*W per-pixel JNI calls.
 * Not compiled in this repository's CI (no JDK in the build image).
 */
public final class MSegmentNative {
    static {
        System.loadLibrary("msegment_jni");   // links libmsegment.so
    }

    private static final ThreadLocal<Long> CTX = ThreadLocal.withInitial(() -> create(0));

    private MSegmentNative() {
    }

    private static native long create(int device);

    private static native void destroy(long ctx);

    /** Returns 0 or a negative MSG_E* code; markers rewritten in place, dst filled. */
    private static native int watershedColorize(long ctx, byte[] bgr, int[] markers, int rows, int cols,
                                                int depth, byte[] paletteOrNull, byte[] dst);

    private static native String lastError(long ctx);

    /** Drop-in for PictureService.watershed(src, markers, depth, colored) given its palette. */
    public static Mat watershed(Mat src, Mat markers, int depth, byte[] paletteOrNull) {
        if (src.type() != CvType.CV_8UC3 || markers.type() != CvType.CV_32SC1
                || !src.size().equals(markers.size())) {
            throw new CvException("watershed: src must be CV_8UC3 and markers CV_32SC1 of the same size");
        }
        int rows = src.rows();
        int cols = src.cols();
        byte[] bgr = new byte[rows * cols * 3];
        int[] lab = new int[rows * cols];
        byte[] out = new byte[rows * cols * 3];
        src.get(0, 0, bgr);
        markers.get(0, 0, lab);
        long ctx = CTX.get();
        int rc = watershedColorize(ctx, bgr, lab, rows, cols, depth, paletteOrNull, out);
        if (rc != 0) {
            throw new CvException("libmsegment error " + rc + ": " + lastError(ctx));
        }
        markers.put(0, 0, lab);
        Mat dst = new Mat(markers.size(), CvType.CV_8UC3);
        dst.put(0, 0, out);
        return dst;
    }
}
