/*
 * msegment.h -- C ABI of libmsegment, the MI355X (gfx950) drop-in for the reference's
 * watershed hot path.  Plain pointers and sizes only; no exceptions cross this boundary.
 *
 * Reference interface each entry point replaces (paths relative to the reference repo):
 *   PictureService.watershed(Mat src, Mat markers, Integer depth, boolean colored)
 *       src/main/java/ru/shayhulud/opencvcmsegment/service/PictureService.java:908-911
 *     = Imgproc.watershed(src, markers)                          PictureService.java:909
 *       -> static native void watershed_0(long image, long markers)   [ext, OpenCV 3.4.2 Java]
 *       -> Java_org_opencv_imgproc_Imgproc_watershed_10(JNIEnv*, jclass, jlong, jlong)
 *       -> cv::watershed(InputArray, InputOutputArray)  modules/imgproc/src/segmentation.cpp
 *     + colorByIndexes(markers, depth, colored)                   PictureService.java:913-936
 *       with the palette from generateBGRColor()                  PictureService.java:236-241
 *     + the callers' cvtColor(dst, COLOR_BGR2GRAY)                PictureService.java:376-379
 *
 * Semantics are OpenCV's, bit for bit: markers (int32, rows x cols) are overwritten in place
 * with the label map (input labels > 0, -1 on watershed lines and on the one-pixel frame, 0 for
 * interior pixels no seed reaches).  The image is 8-bit 3-channel BGR.
 *
 * Return codes: MSG_OK (0) or a negative MSG_E* code; msg_last_error() has the text.
 * MSG_EINVAL mirrors cv::watershed's CV_Assert (type/size/stride checks); the JNI shim
 *  turns any nonzero code into a Java exception like CvException.
 *
 * Frame sizes: the flood entry points (watershed, colorize, edge weights) take frames up to
 * about 2^29 pixels (4 rows*cols + 16 and the frame's 4x4-tile padded size below 2^31 - 512:
 * e.g. 23168 x 23168 or 16387 x 32749); the marker stages (msg_nc_*, msg_shape_*,
 * msg_color_*) take up to 2^28.  Larger frames are MSG_EINVAL.
 *
 * Threading: a context is used by one thread at a time; contexts are independent.
 */
#ifndef MSEGMENT_H
#define MSEGMENT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MSG_OK        0
#define MSG_EINVAL   (-1)  /* bad argument: null pointer, negative size, short stride      */
#define MSG_EHIP     (-2)  /* a HIP runtime call failed                                    */
#define MSG_ENOMEM   (-3)  /* device allocation failed                                     */
#define MSG_ETIMEOUT (-4)  /* a bounded in-kernel wait expired (result invalid)            */
#define MSG_ESTATE   (-5)  /* internal consistency check failed on the device, or a state
                              the reference itself fails in (documented per entry point)   */
#define MSG_ERANGE   (-6)  /* output array too small / search space beyond what the
                              reference could finish (documented per entry point)          */

#define MSG_ABI_VERSION 7

typedef struct msg_ctx msg_ctx;

typedef struct msg_stats {
    int64_t batches;        /* flood generations (bucket batches) in the last watershed call */
    int64_t pops;           /* pixels popped (labelled or WSHED) in the last call            */
    int64_t host_syncs;     /* host<->device control round trips in the last call            */
    int64_t rows, cols;     /* size of the last frame                                        */
    int64_t items;          /* batch items resolved, committed or not (>= pops)               */
    int64_t pushes;         /* queue appends after phase 1                                    */
    int64_t diag[8];        /* msg_set_diag counters (0 when off): k_resolve gather cycles,
                               dependency-loop cycles, loop rounds, max loop cycles, wave-rounds;
                               small-batch loop rounds, small-batch loop entries; reserved.
                               When speculative generations ran (10 ns ticks): sums over the
                               rounds of the round's longest wave's wave-cooperative cascades
                               and of its log copy + change marks; wave time in the round kernel;
                               longest wave; sums over the rounds of the longest wave's top-pop
                               waits, of its whole time, of its top-pop writes + cascades; waves.
                               Single floods only: 0 after a batch call (the frames' banks differ) */
    /* speculative generations (the interrupt-dense regime; msg_set_speculative) */
    int64_t spec_generations;   /* generations committed                                        */
    int64_t spec_rounds;        /* rounds run (every generation needs >= 2: run + confirm)      */
    int64_t spec_executions;    /* item executions over all rounds                              */
    int64_t spec_cascade_pops;  /* committed pops inside cascades (below the generation level)  */
    int64_t spec_fallbacks;     /* overflowing executions handed to serial pops                 */
    int64_t spec_replays;       /* executions whose cascade was replayed from the previous
                                   round's log (no input changed): spec_executions - spec_replays
                                   cascades were run pop by pop                                 */
    int64_t spec_cooldowns;     /* times the regime was judged slower than serial pops (each
                                   followed by a stretch of serial pops)                          */
    int64_t spec_gen_pops;      /* pops committed by generations (the rest were popped serially
                                   or in batches)                                               */
    int64_t spec_gen_us;        /* device time from generation starts to their flattening, us  */
    /* where the committed items went (the per-kernel algorithmic bytes of bench.py's roofline) */
    int64_t fast_pops, fast_pushes;        /* committed / appended by k_commit_fast             */
    int64_t scatter_pops, scatter_pushes;  /* committed / appended through k_scan + k_scatter
                                              (batches above 4096 items, phase 1, generations) */
    /* the other priced kernels' units, counted where the work happens */
    int64_t resolve_items;      /* items of the batches k_resolve decided (its re-runs included) */
    int64_t spec_exec_pops;     /* pops k_spec_round ran pop by pop: the top pops and cascade pops
                                   of every execution that was not replayed, over all rounds     */
    int64_t spec_longest_pops;  /* sum over the rounds of each round's longest such execution    */
    /* batch calls (ABI 7) */
    int64_t batch_mode;         /* the path the last batch call's frames took: 0 the full engine per
                                   flood, 1 / 2 the many-floods kernel (msg_set_batch_floods)     */
    int64_t batch_probe;        /* 1: mode 3 flooded frame 0 alone first to choose that path     */
} msg_stats;

#define MSG_NKERNELS 24
typedef struct msg_kernel_profile {
    char    name[32];       /* kernel name, e.g. "k_resolve"                                   */
    int64_t launches;       /* launches timed since the last reset                              */
    double  total_ms;       /* sum of HIP-event durations of those launches                     */
} msg_kernel_profile;

/* One context per thread: owns a HIP stream and the device workspace on `device_ordinal`.
 * Workspace, kept between calls and grown to the largest frame seen: ~44 B per pixel for the
 * flood, plus ~88 B per tiled pixel and ~200 MB for the speculative-generation engine
 * (DESIGN.md section 3a): allocated up front for frames of 2^20 tiled pixels or more when memory
 * allows (otherwise on the first flood that enters the interrupt-dense regime), and on that first
 * entry below that size.
 * flags: 0, or MSG_CREATE_HIGH_PRIORITY for a high-priority stream (the batch entry points'
 * internal sub-contexts use it: the HIP runtime keeps streams of different priorities on
 * different hardware queues, so concurrent floods overlap even at GPU_MAX_HW_QUEUES=4).
 * Replaces: OpenCV.loadLocally()  App.java:15 (library bring-up). */
#define MSG_CREATE_HIGH_PRIORITY 0x1u
int  msg_create(msg_ctx** out, int device_ordinal, unsigned flags);
void msg_destroy(msg_ctx* ctx);
const char* msg_last_error(const msg_ctx* ctx);
int  msg_abi_version(void);
/* Identity of the sources the library was built from: the first 16 hex digits of the SHA-256 of
 * csrc's sources and this header (opencv-msegment_amd/csrc/Makefile).  The Python binding refuses
 * a library whose id differs from the sources next to it (a stale build would test old kernels). */
const char* msg_build_id(void);
int  msg_get_stats(const msg_ctx* ctx, msg_stats* out);

/* Per-kernel timing with HIP events recorded on the launch stream around every kernel launch
 * (measurement aid for bench.py's roofline; off by default).  msg_get_kernel_profile fills up
 * to max_entries records and returns how many; reset != 0 zeroes the totals. */
int  msg_set_profiling(msg_ctx* ctx, int enable);
int  msg_get_kernel_profile(msg_ctx* ctx, msg_kernel_profile* out, int max_entries, int reset);
/* In-kernel cycle counters (s_memtime) for the flood kernels, reported in msg_stats.diag.
 * Diagnostics only: they add atomics to the kernels; never enabled in timed runs.
 * enable == 2 also injects faults for tests: the decision kernel's odd blocks give up their
 * first chunk of every batch once, which exercises the give-up / re-run path.
 * enable == 3 reports the regime split instead: tiny batches, their pops, their time
 * (s_memrealtime, 10 ns ticks); serial pops, their time; two reserved counters; pops of small
 * batches (65..4096 items).
 * enable == 4 (the -DMSEG_SPEC_PROF diagnostic build) reports the wave-cooperative cascade
 * pop's phases instead (s_memtime cycles summed over pops): loads issued + queue fix, the wait
 * for the loads, writes + decision, pushes, select; counters 5..7 are 0.  In the -DMSEG_SER_PROF
 * diagnostic build it reports the serial pops' phases (s_memtime cycles summed over pops): load,
 * fold, push, between pops, pushes, pops, ring-refill cycles, empty-bucket-scan cycles. */
int  msg_set_diag(msg_ctx* ctx, int enable);
/* Speculative generations for the interrupt-dense regime (textured frames, scattered seeds):
 * on by default.  enable = 0 keeps the batch engine's serial pops there instead (A/B runs and
 * tests of that path).  Results are identical either way (both are the exact serial order). */
int  msg_set_speculative(msg_ctx* ctx, int enable);
/* Two-launch flood iterations for large batches (decide, then one commit grid that also forms
 * the next batch) instead of three (decide, one-block scan, scatter): on by default; 0 keeps
 * the three-launch iterations (A/B runs and tests).  Results are identical either way. */
int  msg_set_fast_commit(msg_ctx* ctx, int enable);

/* ---- host-buffer entry points (synchronous; strides in BYTES) ---------------------------- */

/* cv::watershed(src, markers) in place.  Replaces Imgproc.watershed  PictureService.java:909. */
int msg_watershed(msg_ctx* ctx, const uint8_t* bgr, size_t bgr_stride, int32_t* markers,
                  size_t marker_stride, int rows, int cols);

/* colorByIndexes(labels, depth, colored)  PictureService.java:913-936.
 * palette_bgr: depth*3 bytes (B,G,R per label 1..depth) = the colored=true palette drawn by
 * generateBGRColor (PictureService.java:236-241); NULL = colored=false (all white). */
int msg_colorize(msg_ctx* ctx, const int32_t* labels, size_t label_stride, int rows, int cols,
                 int depth, const uint8_t* palette_bgr, uint8_t* dst_bgr, size_t dst_stride);

/* PictureService.watershed (PictureService.java:908-911) fused: watershed in place on
 * `markers`, then colorByIndexes into dst_bgr; if gray != NULL also the callers'
 * cvtColor(dst, COLOR_BGR2GRAY) (PictureService.java:376-379).  One H2D/D2H per buffer. */
int msg_watershed_colorize(msg_ctx* ctx, const uint8_t* bgr, size_t bgr_stride,
                           int32_t* markers, size_t marker_stride, int rows, int cols,
                           int depth, const uint8_t* palette_bgr, uint8_t* dst_bgr,
                           size_t dst_stride, uint8_t* gray, size_t gray_stride);

/* Batch of independent frames (BASELINE config 5), no collectives: up to msg_set_batch_inflight
 * floods run concurrently on this context's device (each on its own internal sub-context,
 * stream and host thread; the floods are latency-bound, so they overlap).  Arrays have n
 * entries.  Replaces: a loop of PictureService.watershed calls over frames. */
int msg_watershed_batch(msg_ctx* ctx, int n, const uint8_t* const* bgr, const size_t* bgr_stride,
                        int32_t* const* markers, const size_t* marker_stride, const int* rows,
                        const int* cols);
/* The same batch with each frame's colorByIndexes (one palette for every frame, NULL = white;
 * dst_bgr[k] rows*cols*3 bytes at dst_stride[k]): the reference's evaluation loop floods 92
 * frames per image through PictureService.watershed (CorrelationTestService.java:84-86, 116, 128,
 * 141 -> PictureService.java:852), which the JNI shim hands over in one call
 * (MSegmentNative.watershedBatch). */
int msg_watershed_colorize_batch(msg_ctx* ctx, int n, const uint8_t* const* bgr, const size_t* bgr_stride,
                                 int32_t* const* markers, const size_t* marker_stride, const int* rows,
                                 const int* cols, int depth, const uint8_t* palette_bgr,
                                 uint8_t* const* dst_bgr, const size_t* dst_stride);

/* Floods kept in flight by the batch entry points (1..8, default 4; 1 = back to back). */
int msg_set_batch_inflight(msg_ctx* ctx, int k);

/* Host-buffer batches over several devices (BASELINE config 5: 64 frames, one frame stream per GPU,
 * no collectives).  After this call msg_watershed_batch and msg_watershed_colorize_batch split
 * their n frames into ndev contiguous blocks -- block j = frames [n*j/ndev, n*(j+1)/ndev) -- and run
 * block j on an internal sub-context on devices[j] (one host thread per entry; each sub-context
 * keeps this context's msg_set_batch_inflight / msg_set_batch_floods / speculative / fast-commit
 * settings).  With 8 entries 0..7 and 64 frames, device r floods frames 8r..8r+7 -- the frames
 * bench.py's rank r takes.  A device may repeat (e.g. {0, 0}: two sub-contexts on one GPU).
 * ndev = 0 restores this context's own device.  Device-pointer batches (the _dev entry) are not
 * affected: their buffers live on one device.  Each entry costs a context and its workspace
 * (~44 B/px of the largest frame it flooded) on its device, released by ndev = 0 or msg_destroy.
 * The reference's JVM reaches it through MSegmentNative.watershedBatch(..., devices) (INTEGRATION.md
 * section 5); it replaces a loop of PictureService.watershed calls (PictureService.java:908) that
 * can only use the JVM's one context device.  MSG_EINVAL for ndev < 0 or > 64, a null list, or a
 * device ordinal outside [0, hipGetDeviceCount()). */
int msg_set_batch_devices(msg_ctx* ctx, int ndev, const int* devices);

/* Many floods per launch in the batch entry points (msg_watershed_batch,
 * msg_watershed_colorize_batch, msg_watershed_colorize_batch_dev), for frames whose exact flood is serial-bound -- photographs,
 * the scattered seeds of notConnectedMarkers (PictureService.java:852, called 90 times per image by
 * CorrelationTestService.java:84-86, 141): every frame of the call gets a workspace of its own
 * (~44 B/px of HBM each), and ONE kernel pops all of them, one wave per flood, so the call keeps
 * as many floods in flight as it has frames instead of msg_set_batch_inflight's streams.
 *   mode 0: off (the full engine per flood, msg_set_batch_inflight of them at a time);
 *   mode 1: every flood popped serially to its end in that kernel;
 *   mode 2: a flood that pops 4096 times in a row without pushing below its level (a plateau,
 *           where batches pay) is finished by the full engine instead;
 *   mode 3: automatic (the default).  The first batch call of a frame size floods frame 0 alone
 *           with the full engine (part of the call: its result is final) and prices the rest of
 *           the batch both ways -- the full engine at that flood's wall time per flood,
 *           msg_set_batch_inflight at a time, against the many-floods kernel at ~1 us per pop of
 *           one wave with every flood in flight -- then runs the cheaper path (mode 0 or 1); later
 *           calls of that frame size reuse the choice.  Plateaus and textures the speculative
 *           engine serves (mosaic, noise) stay on the full engine; chains of dependent pops
 *           (notConnectedMarkers' seeds, photographs) in batches larger than the floods in flight
 *           go to the many-floods kernel.  If that kernel's workspaces do not fit the device, the
 *           call falls back to mode 0.  msg_stats.batch_mode / batch_probe report what ran.
 * Results are identical in every mode (each is cv::watershed's exact serial order).
 * Memory: the per-frame workspaces stay allocated on the context between calls (the next call of
 * the same size reuses them) until mode 0 is set again, which releases them, or msg_destroy. */
int msg_set_batch_floods(msg_ctx* ctx, int mode);

/* Blocks per launch of the flood's decision kernel (0 = default: one wave of the device's
 * occupancy, halved for each flood of a batch call with two or more floods in flight).  A
 * performance knob only: its rank chunks are dealt in dispatch order, so any grid size -- and
 * any number of concurrent floods -- makes progress. */
int msg_set_resolve_grid(msg_ctx* ctx, int blocks);

/* ---- device-resident entry points (dense layouts; pointers are device memory of the
 * context's device; stream = hipStream_t, or NULL: the work then runs on the context's own
 * stream, ordered after what the legacy null stream had queued and before what it queues
 * next, i.e. as if on the null stream).  They return when the flood has finished; the
 * colourise kernel may still be in flight on `stream`. ---- */

/* d_markers_in (int32) is read, d_labels (int32) written; they may alias (in place). */
int msg_watershed_dev(msg_ctx* ctx, const void* d_bgr, const void* d_markers_in, void* d_labels,
                      int rows, int cols, void* stream);

int msg_colorize_dev(msg_ctx* ctx, const void* d_labels, int rows, int cols, int depth,
                     const void* d_palette_bgr, void* d_dst_bgr, void* d_gray, void* stream);

int msg_watershed_colorize_dev(msg_ctx* ctx, const void* d_bgr, const void* d_markers_in,
                               void* d_labels, int rows, int cols, int depth,
                               const void* d_palette_bgr, void* d_dst_bgr, void* d_gray,
                               void* stream);

/* Device-resident batch of the fused call above (BASELINE config 5 on one GPU): frame k reads
 * d_bgr[k], d_markers_in[k] and writes d_labels[k], d_dst_bgr[k] (rows[k] x cols[k]); one
 * palette and depth for all.  The inputs must be complete on `stream` (it is synchronised
 * first); returns when every frame's labels and colours are written. */
int msg_watershed_colorize_batch_dev(msg_ctx* ctx, int n, const void* const* d_bgr,
                                     const void* const* d_markers_in, void* const* d_labels,
                                     const int* rows, const int* cols, int depth,
                                     const void* d_palette_bgr, void* const* d_dst_bgr, void* stream);

/* Stencil only: L-inf BGR distance to the right and lower neighbour (uint8 each, 0 past the
 * edge) -- the colour-distance kernel of the flood, exposed for parity tests and the roofline. */
int msg_edge_weights_dev(msg_ctx* ctx, const void* d_bgr, void* d_wright, void* d_wdown,
                         int rows, int cols, void* stream);

/* ---- NOT_CONNECTED_MARKERS marker stage: the caller that builds the flood's seeds in
 * PictureService.notConnectedMarkers (PictureService.java:468-842).  Dense device layouts;
 * d_bgr and d_gray need 4-byte alignment, d_markers 16-byte alignment. ------------------- */

#define MSG_NC_GISTO_DIAP 0x1u  /* AlgorithmOptions.GISTO_DIAP: mark the +-3 band around a
                                   level's mean instead of the mean alone (:799-808)        */
#define MSG_NC_MULTI_OTSU 0x2u  /* AlgorithmOptions.MULTI_OTSU: replace the levels by the
                                   multi-Otsu split of the 128-bin histogram (:650-722)     */
#define MSG_NC_MEDIAN_BLUR 0x4u /* AlgorithmOptions.MEDIAN_BLUR: medianBlur(srcGray, k) before
                                   the histogram (:481-483); k = filterMaskSize in option
                                   bits 8-15 (MSG_NC_MASK(k)), odd, else MSG_EINVAL.         */
#define MSG_NC_BILATERAL 0x8u   /* AlgorithmOptions.BILATERIAL (ignored with MEDIAN_BLUR: the
                                   reference's else-if): bilateralFilter(srcGray, dst, d, 2d, 2d)
                                   before the histogram (:488-495), d = MSG_NC_MASK's bits,
                                   BORDER_REFLECT_101, fp32 as OpenCV 3.4.2's non-IPP 8-bit
                                   path sums it (an IPP build may round pixels differently). */
#define MSG_NC_MASK(k) (((unsigned)(k) & 0xffu) << 8)

typedef struct msg_bright_level {  /* model/BrightLevel.java */
    int32_t start, end, count;
} msg_bright_level;

/* srcGray = cvtColor(src, COLOR_BGR2GRAY) (:476-478) into d_gray (rows*cols bytes) and its
 * 256-bin histogram calcHist(srcGray, [0,256)) (:565) into hist256 (HOST, exact counts).
 * Returns when hist256 is filled. */
int msg_gray_hist_dev(msg_ctx* ctx, const void* d_bgr, int rows, int cols, void* d_gray,
                      int32_t* hist256, void* stream);

/* Host only (no context, no GPU): the brightness levels of notConnectedMarkers from the
 * histogram -- the flex thresholds (:574-640), or with MSG_NC_MULTI_OTSU the multi-Otsu
 * override (:650-722; the reference's recursion enumerates ~C(128,k) splits for k flex levels:
 * MSG_ERANGE when that exceeds 2e9 iterations, which it could not finish either).  depth is
 * the user's depth (block size limit 256/depth).  Writes min(n, max_levels) levels and n;
 * MSG_ERANGE if n > max_levels; MSG_ESTATE where the reference throws (no level at all);
 * MSG_EINVAL for depth <= 0 (ArithmeticException). */
int msg_nc_levels(const int32_t* hist256, int rows, int cols, int depth, unsigned options,
                  msg_bright_level* levels, int max_levels, int* n_levels);

/* Host only: brightness -> marker table of "ALLOCATE TO LAYERS" (:781-828): lut256[b] = 1 + the
 * index of the first level whose mean (GISTO_DIAP: mean band) holds b, else 0. */
int msg_nc_marker_lut(const msg_bright_level* levels, int n_levels, unsigned options,
                      int32_t* lut256);

/* markers(i,j) = lut256[gray(i,j)] into d_markers (int32, rows*cols): the summed marker maps
 * wshedMarkSumm (:823-828) that PictureService.watershed then floods (:834). */
int msg_nc_markers_dev(msg_ctx* ctx, const void* d_gray, int rows, int cols,
                       const int32_t* lut256, void* d_markers, void* stream);

/* The whole marker stage: gray (MSG_NC_MEDIAN_BLUR: then its k x k median; MSG_NC_BILATERAL:
 * then its bilateral filter) + histogram ->
 * levels -> markers.  d_gray (the final srcGray) may be NULL (context scratch).  The level count is the watershed depth the reference then uses (:834): draw the
 * palettes for it and call msg_watershed_colorize_dev(d_bgr, d_markers, ...). */
int msg_nc_marker_stage_dev(msg_ctx* ctx, const void* d_bgr, int rows, int cols, int depth,
                            unsigned options, void* d_gray, void* d_markers,
                            msg_bright_level* levels, int max_levels, int* n_levels,
                            void* stream);

/* Host-buffer form of the marker stage (synchronous; strides in bytes): bgr in, the int32
 * marker map out.  For callers without device memory (the JNI shim). */
int msg_nc_marker_stage(msg_ctx* ctx, const uint8_t* bgr, size_t bgr_stride, int rows, int cols,
                        int depth, unsigned options, int32_t* markers, size_t marker_stride,
                        msg_bright_level* levels, int max_levels, int* n_levels);

/* ---- SHAPE_METHOD marker stage: the caller that builds the flood's seeds in
 * PictureService.shapeAutoMarkerWatershed (PictureService.java:395-466):
 *   gray (:404-405) -> medianBlur k (:407-408) -> Canny(5, 50) (:415-416)
 *   -> dilate 3x3, dilate 5x5, subtract (:426-429) -> medianBlur 3 (:435)
 *   -> connectedComponents(8, CV_32S) = the markers (:441)
 *   -> depth = findContours(RETR_CCOMP).size() (:447-451; 0 = no contour: the reference
 *      returns null and never floods).
 * Then msg_watershed_colorize*(src, markers, depth, ...) is the reference's this.watershed (:455).
 * ----------------------------------------------------------------------------------------- */

/* Host only: calculateSizeOfSquareBlurMask (:877-899), the median size the stage uses. */
int msg_blur_mask_size(int rows, int cols);

/* The whole stage on device buffers: d_bgr (rows*cols*3, BGR) in, d_markers (int32 rows*cols)
 * out; ksize <= 0 picks msg_blur_mask_size (the reference's choice), else the k x k median
 * (odd, <= 255).  depth / ncomp (host ints): contour count and component count.  d_blur,
 * d_edges, d_mask (rows*cols bytes each) may be NULL; when given they receive the blurred gray,
 * the Canny edges and the marker mask (the reference's saved steps :410, :420, :437).  Returns
 * when depth and ncomp are known (the markers are complete on `stream`). */
int msg_shape_markers_dev(msg_ctx* ctx, const void* d_bgr, int rows, int cols, int ksize,
                          void* d_markers, int* depth, int* ncomp, void* d_blur, void* d_edges,
                          void* d_mask, void* stream);

/* Host-buffer form (synchronous; strides in bytes). */
int msg_shape_markers(msg_ctx* ctx, const uint8_t* bgr, size_t bgr_stride, int rows, int cols,
                      int ksize, int32_t* markers, size_t marker_stride, int* depth, int* ncomp);

/* ---- COLOR_METHOD marker stage: the caller that builds the flood's seeds in
 * PictureService.colorAutoMarkerWatershed (PictureService.java:301-392):
 *   src - filter2D(9x1 Laplacian column) saturated = the flood's src (:323-333; the white -> black
 *   loop :309-318 never fires in Java: PixelUtil.java:19 compares a signed byte with 255)
 *   -> bw = threshold(BGR2GRAY, OTSU) (:338, :938-943)
 *   -> distanceTransform(bw, DIST_L2, 5), normalize(NORM_MINMAX) (:343, :1018-1023)
 *   -> threshold(0.4), dilate 3x3 (:348-350)
 *   -> findContours(RETR_CCOMP) + drawContours(i, i + 1, FILLED, hierarchy) + circle((5,5), 3,
 *      255) = the markers, depth = the contour count (:355-365)
 * Then msg_watershed_colorize*(sharp, markers, depth, ...) is the reference's this.watershed
 * (:378).  The contour numbering is restated through connected components:
 * unpinned against a real OpenCV build, like the rest of the stage.
 * ----------------------------------------------------------------------------------------- */

/* The whole stage on device buffers: d_bgr (rows*cols*3, BGR) in; d_sharp (rows*cols*3, the
 * sharpened BGR image the watershed floods) and d_markers (int32 rows*cols) out; *depth (host)
 * = the contour count.  d_bgr and d_sharp must not alias.  Returns when depth is known (the
 * outputs are complete on `stream`). */
int msg_color_markers_dev(msg_ctx* ctx, const void* d_bgr, int rows, int cols, void* d_sharp,
                          void* d_markers, int* depth, void* stream);

/* Host-buffer form (synchronous; strides in bytes). */
int msg_color_markers(msg_ctx* ctx, const uint8_t* bgr, size_t bgr_stride, int rows, int cols,
                      uint8_t* sharp, size_t sharp_stride, int32_t* markers, size_t marker_stride,
                      int* depth);

#ifdef __cplusplus
}
#endif
#endif /* MSEGMENT_H */
