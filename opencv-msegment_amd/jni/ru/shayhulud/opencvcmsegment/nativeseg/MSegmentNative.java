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

    /** The GPU new thread contexts open on: -Dmsegment.device=N, or useDevice(N); 0 by default. */
    private static volatile int defaultDevice = Integer.getInteger("msegment.device", 0);

    private static final ThreadLocal<Long> CTX = ThreadLocal.withInitial(() -> open(defaultDevice));

    private MSegmentNative() {
    }

    private static native long create(int device);

    private static native void destroy(long ctx);

    private static long open(int device) {
        long ctx = create(device);
        if (ctx == 0) {
            throw new CvException("libmsegment: no context on device " + device);
        }
        return ctx;
    }

    /**
     * Moves the calling thread's context to GPU {@code device} (its old context and workspace are
     * released) and makes it the device later threads start on.  Replaces the fixed device 0.
     */
    public static void useDevice(int device) {
        long fresh = open(device);
        long old = CTX.get();
        CTX.set(fresh);
        BATCH_MODE.get()[0] = BATCH_AUTO;  // a fresh context starts in the library's default mode
        BATCH_DEVICES.set(new int[0]);
        defaultDevice = device;
        destroy(old);
    }

    /** msg_set_batch_devices: the host batches' device list (empty = the context's own device). */
    private static native int setBatchDevices(long ctx, int[] devices);

    private static final ThreadLocal<int[]> BATCH_DEVICES = ThreadLocal.withInitial(() -> new int[0]);

    /** Returns 0 or a negative MSG_E* code; markers rewritten in place, dst filled. */
    private static native int watershedColorize(long ctx, byte[] bgr, int[] markers, int rows, int cols,
                                                int depth, byte[] paletteOrNull, byte[] dst);

    private static native String lastError(long ctx);

    /** Returns the level count or a negative MSG_E* code; markers and levels (3 ints each) filled. */
    private static native int ncMarkers(long ctx, byte[] bgr, int rows, int cols, int depth, int options,
                                        int[] markers, int[] levelsOut);

    /** AlgorithmOptions.GISTO_DIAP / MULTI_OTSU / MEDIAN_BLUR / BILATERIAL bits of
     *  msg_nc_marker_stage (msegment.h); the pre-filters take filterMaskSize in bits 8-15. */
    public static final int NC_GISTO_DIAP = 0x1;
    public static final int NC_MULTI_OTSU = 0x2;
    public static final int NC_MEDIAN_BLUR = 0x4;
    public static final int NC_BILATERAL = 0x8;

    /**
     * The pre-filter and mask-size bits for notConnectedMarkers' options (PictureService.java:481-495),
     * MEDIAN_BLUR winning over BILATERIAL as the reference's if / else-if.  MEDIAN_BLUR: medianBlur
     * asserts ksize % 2 == 1 (negative and even sizes throw there), and sizes above 255 do not fit
     * the option bits -- both throw instead of wrapping through the & 0xff packing.  BILATERIAL:
     * sizes <= 0 act as 0 in bilateralFilter (sigma <= 0 -> 1), sizes above 255 throw.
     */
    public static int ncFilterBits(boolean medianBlur, boolean bilateral, int filterMaskSize) {
        if (medianBlur) {
            if (filterMaskSize < 1 || filterMaskSize % 2 != 1 || filterMaskSize > 255) {
                throw new CvException("MEDIAN_BLUR mask size " + filterMaskSize + ": odd, 1..255");
            }
            return NC_MEDIAN_BLUR | (filterMaskSize << 8);
        }
        if (bilateral) {
            if (filterMaskSize > 255) {
                throw new CvException("BILATERIAL mask size " + filterMaskSize + ": at most 255");
            }
            return NC_BILATERAL | (Math.max(filterMaskSize, 0) << 8);
        }
        return 0;
    }

    /**
     * Drop-in for the marker stage of PictureService.notConnectedMarkers (PictureService.java:476-828):
     * returns wshedMarkSumm (CV_32SC1) and fills levelsOut with the BrightLevel list (the caller's
     * fThresholds; its size is the depth passed on to watershed / colorByIndexes).
     */
    public static Mat notConnectedMarkers(Mat src, int depth, int options, java.util.List<int[]> levelsOut) {
        if (src.type() != CvType.CV_8UC3) {
            throw new CvException("notConnectedMarkers: src must be CV_8UC3");
        }
        int rows = src.rows();
        int cols = src.cols();
        byte[] bgr = new byte[rows * cols * 3];
        int[] mk = new int[rows * cols];
        int[] lv = new int[3 * 256];
        src.get(0, 0, bgr);
        long ctx = CTX.get();
        int n = ncMarkers(ctx, bgr, rows, cols, depth, options, mk, lv);
        if (n < 0) {
            throw new CvException("libmsegment error " + n + ": " + lastError(ctx));
        }
        for (int i = 0; i < n; i++) {
            levelsOut.add(new int[]{lv[3 * i], lv[3 * i + 1], lv[3 * i + 2]});
        }
        Mat markers = new Mat(src.size(), CvType.CV_32SC1);
        markers.put(0, 0, mk);
        return markers;
    }

    /** Returns the contour count (>= 0) or a negative MSG_E* code; markers filled. */
    private static native int shapeMarkers(long ctx, byte[] bgr, int rows, int cols, int[] markers);

    /**
     * Drop-in for the marker stage of PictureService.shapeAutoMarkerWatershed
     * (PictureService.java:402-452): returns the connectedComponents markers (CV_32SC1) and puts
     * the RETR_CCOMP contour count (the depth passed to watershed) in depthOut[0]; 0 contours is
     * where the reference returns null.
     */
    public static Mat shapeMarkers(Mat src, int[] depthOut) {
        if (src.type() != CvType.CV_8UC3) {
            throw new CvException("shapeMarkers: src must be CV_8UC3");
        }
        int rows = src.rows();
        int cols = src.cols();
        byte[] bgr = new byte[rows * cols * 3];
        int[] mk = new int[rows * cols];
        src.get(0, 0, bgr);
        long ctx = CTX.get();
        int d = shapeMarkers(ctx, bgr, rows, cols, mk);
        if (d < 0) {
            throw new CvException("libmsegment error " + d + ": " + lastError(ctx));
        }
        depthOut[0] = d;
        Mat markers = new Mat(src.size(), CvType.CV_32SC1);
        markers.put(0, 0, mk);
        return markers;
    }

    /** Returns the contour count (>= 0) or a negative MSG_E* code; sharp and markers filled. */
    private static native int colorMarkers(long ctx, byte[] bgr, int rows, int cols, byte[] sharp, int[] markers);

    /**
     * Drop-in for the marker stage of PictureService.colorAutoMarkerWatershed
     * (PictureService.java:301-366): returns the markers (CV_32SC1), writes the sharpened image
     * the reference then floods (:333) into sharpOut (CV_8UC3, allocated here) and the contour
     * count (the depth passed to watershed) into depthOut[0].
     */
    public static Mat colorMarkers(Mat src, Mat sharpOut, int[] depthOut) {
        if (src.type() != CvType.CV_8UC3) {
            throw new CvException("colorMarkers: src must be CV_8UC3");
        }
        int rows = src.rows();
        int cols = src.cols();
        byte[] bgr = new byte[rows * cols * 3];
        byte[] sh = new byte[rows * cols * 3];
        int[] mk = new int[rows * cols];
        src.get(0, 0, bgr);
        long ctx = CTX.get();
        int d = colorMarkers(ctx, bgr, rows, cols, sh, mk);
        if (d < 0) {
            throw new CvException("libmsegment error " + d + ": " + lastError(ctx));
        }
        depthOut[0] = d;
        sharpOut.create(src.size(), CvType.CV_8UC3);
        sharpOut.put(0, 0, sh);
        Mat markers = new Mat(src.size(), CvType.CV_32SC1);
        markers.put(0, 0, mk);
        return markers;
    }

    /** msg_set_batch_floods: 0 the full engine per flood, 1 / 2 many floods per launch, 3 automatic. */
    private static native int setBatchFloods(long ctx, int mode);

    /** Batch modes of msg_set_batch_floods (msegment.h). */
    public static final int BATCH_FULL_ENGINE = 0;
    public static final int BATCH_MANY_FLOODS = 1;
    public static final int BATCH_AUTO = 3;

    /** Returns 0 or a negative MSG_E* code; every markers[k] rewritten in place, every dsts[k] filled. */
    private static native int watershedColorizeBatch(long ctx, byte[][] bgrs, int[][] markers, int[] rows,
                                                     int[] cols, int depth, byte[] paletteOrNull, byte[][] dsts);

    private static final ThreadLocal<int[]> BATCH_MODE = ThreadLocal.withInitial(() -> new int[]{BATCH_AUTO});

    /**
     * PictureService.watershed over many frames in one native call: the reference's evaluation
     * loop floods 92 frames per image (CorrelationTestService.java:84-86, 116, 128, 141, each through
     * PictureService.watershed at :852).  manyFloods = true selects msg_set_batch_floods mode 1
     * (every flood popped serially to its end, one wave per flood, all in one kernel: the mode for
     * notConnectedMarkers' scattered seeds); false, the library's automatic mode 3 (a probe flood per
     * frame size picks the full engine or the many-floods kernel).  Labels are written
     * back into each markers Mat, and the colourised frames are returned in order.  One palette
     * (or null: colored = false) serves every frame, as one generateBGRColor draw per call would.
     */
    public static java.util.List<Mat> watershedBatch(java.util.List<Mat> srcs, java.util.List<Mat> markers,
                                                     int depth, byte[] paletteOrNull, boolean manyFloods) {
        return watershedBatch(srcs, markers, depth, paletteOrNull, manyFloods ? BATCH_MANY_FLOODS : BATCH_AUTO,
                new int[0]);
    }

    /**
     * watershedBatch over several GPUs (BASELINE config 5: one frame stream per GPU, no collectives):
     * the frames are split into devices.length contiguous blocks, block j flooded on GPU devices[j]
     * (msg_set_batch_devices); an empty array keeps the thread's own device.  E.g. 64 frames on
     * {0..7}: GPU r floods frames 8r..8r+7.
     */
    public static java.util.List<Mat> watershedBatch(java.util.List<Mat> srcs, java.util.List<Mat> markers,
                                                     int depth, byte[] paletteOrNull, int batchMode,
                                                     int[] devices) {
        int n = srcs.size();
        if (devices == null) {
            throw new CvException("watershedBatch: null device list");
        }
        if (markers.size() != n) {
            throw new CvException("watershedBatch: " + n + " images but " + markers.size() + " marker maps");
        }
        byte[][] bgr = new byte[n][];
        int[][] lab = new int[n][];
        byte[][] out = new byte[n][];
        int[] rows = new int[n];
        int[] cols = new int[n];
        for (int k = 0; k < n; k++) {
            Mat src = srcs.get(k);
            Mat mk = markers.get(k);
            if (src.type() != CvType.CV_8UC3 || mk.type() != CvType.CV_32SC1 || !src.size().equals(mk.size())) {
                throw new CvException("watershedBatch: frame " + k + ": src must be CV_8UC3 and markers CV_32SC1 "
                        + "of the same size");
            }
            rows[k] = src.rows();
            cols[k] = src.cols();
            bgr[k] = new byte[rows[k] * cols[k] * 3];
            lab[k] = new int[rows[k] * cols[k]];
            out[k] = new byte[rows[k] * cols[k] * 3];
            src.get(0, 0, bgr[k]);
            mk.get(0, 0, lab[k]);
        }
        long ctx = CTX.get();
        int mode = batchMode;
        int[] cur = BATCH_MODE.get();
        if (cur[0] != mode) {  // switching back to 0 releases the mode's per-frame workspaces
            // switching to 0 releases the many-floods workspaces; 3 (automatic) keeps them for reuse
            int rc = setBatchFloods(ctx, mode);
            if (rc != 0) {
                throw new CvException("libmsegment error " + rc + ": " + lastError(ctx));
            }
            cur[0] = mode;
        }
        if (!java.util.Arrays.equals(BATCH_DEVICES.get(), devices)) {
            int rc = setBatchDevices(ctx, devices);
            if (rc != 0) {
                throw new CvException("libmsegment error " + rc + ": " + lastError(ctx));
            }
            BATCH_DEVICES.set(devices.clone());
        }
        int rc = watershedColorizeBatch(ctx, bgr, lab, rows, cols, depth, paletteOrNull, out);
        if (rc != 0) {
            throw new CvException("libmsegment error " + rc + ": " + lastError(ctx));
        }
        java.util.List<Mat> dsts = new java.util.ArrayList<>(n);
        for (int k = 0; k < n; k++) {
            markers.get(k).put(0, 0, lab[k]);
            Mat dst = new Mat(markers.get(k).size(), CvType.CV_8UC3);
            dst.put(0, 0, out[k]);
            dsts.add(dst);
        }
        return dsts;
    }

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
