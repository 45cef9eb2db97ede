/*
 * ws_oracle.c -- CPU ORACLE for the msegment hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / the timed CPU baseline.  The product path
 * (libmsegment.so, opencv-msegment_amd/) never links or calls it.
 *
 * What it restates (behavioural specification, written from scratch):
 *   (1) OpenCV 3.4.2 cv::watershed(InputArray image CV_8UC3, InputOutputArray markers CV_32SC1)
 *       [ext] modules/imgproc/src/segmentation.cpp, reached from the reference at
 *       src/main/java/ru/shayhulud/opencvcmsegment/service/PictureService.java:909
 *       (Imgproc.watershed(src, markers)).  OpenCV is a Maven dependency
 *       (pom.xml:38-43, org.openpnp:opencv:3.4.2-1) and is NOT in /root/reference,
 *       so the algorithm is restated from its published behaviour:
 *         - phase 0: rows 0 and H-1, and cols 0 and W-1 become WSHED (-1);
 *         - phase 1: raster scan of the interior; negatives -> 0; a 0 pixel with a
 *           4-neighbour > 0 is pushed with level = min L-inf BGR distance to those
 *           neighbours and marked IN_QUEUE (-2);
 *         - phase 2: 256 FIFO buckets, always pop the lowest non-empty bucket; the
 *           popped pixel takes the label of its positive 4-neighbours (scan order
 *           L,R,T,B; two different labels -> WSHED); a non-WSHED pixel pushes every
 *           0 neighbour (order L,R,T,B) at level = L-inf distance to it.
 *   (2) PictureService.colorByIndexes  PictureService.java:913-936
 *       label in 1..depth -> palette[label-1] (white when !colored), anything else black.
 *   (3) cvtColor(dst, COLOR_BGR2GRAY) on the colourised result  PictureService.java:376-379
 *       (OpenCV fixed point: (1868*B + 9617*G + 4899*R + 8192) >> 14).
 *
 * Parity status: OpenCV cannot be built or run in this container (no sources, no jar);
 * the reference has no tests or fixtures for this path.  This oracle is
 * pinned by the hand-derived known-answer tests KAT-1..4 of SURVEY.md 5.A and by an
 * independent pure-Python restatement (oracle/ws_pyref.py) -- otherwise "parity unpinned"
 * against real OpenCV.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define WS_WSHED (-1)
#define WS_INQ   (-2)
#define WS_NQ    256

typedef struct {
    int32_t* v;      /* pixel linear indices (row*cols + col) in FIFO order */
    size_t   head;   /* next element to pop */
    size_t   len;    /* one past the last pushed element */
    size_t   cap;
} ws_fifo;

static int fifo_push(ws_fifo* q, int32_t x)
{
    if (q->len == q->cap) {
        size_t nc = q->cap ? q->cap * 2 : 1024;
        int32_t* nv = (int32_t*)realloc(q->v, nc * sizeof(int32_t));
        if (!nv) return -1;
        q->v = nv;
        q->cap = nc;
    }
    q->v[q->len++] = x;
    return 0;
}

static inline int cdiff(const uint8_t* a, const uint8_t* b)
{
    int d0 = abs((int)a[0] - (int)b[0]);
    int d1 = abs((int)a[1] - (int)b[1]);
    int d2 = abs((int)a[2] - (int)b[2]);
    int m = d0 > d1 ? d0 : d1;
    return m > d2 ? m : d2;
}

/* Returns 0 on success, -1 on bad arguments (CV_Assert analogue), -3 on allocation failure.
 * bgr_stride / marker_stride are in BYTES.  markers are rewritten in place. */
int oracle_watershed(const uint8_t* bgr, size_t bgr_stride, int32_t* markers,
                     size_t marker_stride, int rows, int cols)
{
    if (rows < 0 || cols < 0) return -1;
    if (rows == 0 || cols == 0) return 0;          /* empty Mat: nothing to do */
    if (!bgr || !markers) return -1;
    if (bgr_stride < (size_t)cols * 3 || marker_stride < (size_t)cols * 4 ||
        (marker_stride & 3))
        return -1;

#define M(r, c) (((int32_t*)((uint8_t*)markers + (size_t)(r) * marker_stride))[c])
#define P(r, c) (bgr + (size_t)(r) * bgr_stride + (size_t)(c) * 3)

    /* phase 0: one-pixel frame of WSHED */
    for (int c = 0; c < cols; c++) {
        M(0, c) = WS_WSHED;
        M(rows - 1, c) = WS_WSHED;
    }
    ws_fifo q[WS_NQ];
    memset(q, 0, sizeof(q));
    int rc = 0;

    /* phase 1: raster order over the interior */
    for (int r = 1; r < rows - 1; r++) {
        M(r, 0) = WS_WSHED;
        M(r, cols - 1) = WS_WSHED;
        for (int c = 1; c < cols - 1; c++) {
            int32_t m = M(r, c);
            if (m < 0) { m = 0; M(r, c) = 0; }
            if (m != 0) continue;
            /* left/top neighbours were already visited: positives are untouched, so '>0'
             * still reads the raw input; the frame is already WSHED. */
            int lvl = 256;
            const uint8_t* p = P(r, c);
            if (M(r, c - 1) > 0) { int t = cdiff(p, P(r, c - 1)); if (t < lvl) lvl = t; }
            if (M(r, c + 1) > 0) { int t = cdiff(p, P(r, c + 1)); if (t < lvl) lvl = t; }
            if (M(r - 1, c) > 0) { int t = cdiff(p, P(r - 1, c)); if (t < lvl) lvl = t; }
            if (M(r + 1, c) > 0) { int t = cdiff(p, P(r + 1, c)); if (t < lvl) lvl = t; }
            if (lvl < 256) {
                if (fifo_push(&q[lvl], (int32_t)(r * cols + c))) { rc = -3; goto done; }
                M(r, c) = WS_INQ;
            }
        }
    }

    int active = 0;
    while (active < WS_NQ && q[active].head == q[active].len) active++;

    /* phase 2: priority flood, FIFO within a level */
    while (active < WS_NQ) {
        if (q[active].head == q[active].len) {
            active++;
            while (active < WS_NQ && q[active].head == q[active].len) active++;
            if (active == WS_NQ) break;
        }
        int32_t idx = q[active].v[q[active].head++];
        int r = idx / cols, c = idx - r * cols;
        int32_t nb[4];
        nb[0] = M(r, c - 1);
        nb[1] = M(r, c + 1);
        nb[2] = M(r - 1, c);
        nb[3] = M(r + 1, c);
        int32_t lab = 0;
        for (int k = 0; k < 4; k++) {
            int32_t t = nb[k];
            if (t > 0) {
                if (lab == 0) lab = t;
                else if (t != lab) lab = WS_WSHED;
            }
        }
        M(r, c) = lab;
        if (lab == WS_WSHED) continue;
        static const int dr[4] = {0, 0, -1, 1};
        static const int dc[4] = {-1, 1, 0, 0};
        const uint8_t* p = P(r, c);
        for (int k = 0; k < 4; k++) {
            int rr = r + dr[k], cc = c + dc[k];
            if (M(rr, cc) != 0) continue;
            int t = cdiff(p, P(rr, cc));
            if (fifo_push(&q[t], (int32_t)(rr * cols + cc))) { rc = -3; goto done; }
            if (t < active) active = t;
            M(rr, cc) = WS_INQ;
        }
    }
done:
    for (int i = 0; i < WS_NQ; i++) free(q[i].v);
    return rc;
#undef M
#undef P
}

/* colorByIndexes (PictureService.java:913-936).  palette: depth*3 BGR bytes, or NULL for
 * the colored=false case (every label in 1..depth painted white). */
int oracle_colorize(const int32_t* labels, size_t label_stride, int rows, int cols, int depth,
                    const uint8_t* palette, uint8_t* dst, size_t dst_stride)
{
    if (rows < 0 || cols < 0 || depth < 0) return -1;
    for (int r = 0; r < rows; r++) {
        const int32_t* L = (const int32_t*)((const uint8_t*)labels + (size_t)r * label_stride);
        uint8_t* D = dst + (size_t)r * dst_stride;
        for (int c = 0; c < cols; c++) {
            int32_t l = L[c];
            uint8_t b = 0, g = 0, rr = 0;
            if (l > 0 && l <= depth) {
                if (palette) {
                    b = palette[(size_t)(l - 1) * 3 + 0];
                    g = palette[(size_t)(l - 1) * 3 + 1];
                    rr = palette[(size_t)(l - 1) * 3 + 2];
                } else {
                    b = g = rr = 255;
                }
            }
            D[3 * c + 0] = b;
            D[3 * c + 1] = g;
            D[3 * c + 2] = rr;
        }
    }
    return 0;
}

/* cvtColor(BGR2GRAY) for CV_8UC3 (PictureService.java:376-379, 461-464, 858-862). */
int oracle_bgr2gray(const uint8_t* bgr, size_t bgr_stride, int rows, int cols, uint8_t* gray,
                    size_t gray_stride)
{
    for (int r = 0; r < rows; r++) {
        const uint8_t* S = bgr + (size_t)r * bgr_stride;
        uint8_t* G = gray + (size_t)r * gray_stride;
        for (int c = 0; c < cols; c++) {
            uint32_t v = 1868u * S[3 * c] + 9617u * S[3 * c + 1] + 4899u * S[3 * c + 2] + 8192u;
            G[c] = (uint8_t)(v >> 14);
        }
    }
    return 0;
}

/* distanceTransform(bw, dist, DIST_L2, 5) of OpenCV 3.4.2 (imgproc/src/distransform.cpp,
 * distanceTransform_5x5), restated for the colour-method marker stage (PictureService.java:1018-
 * 1023, reached from :346): a two-pass raster scan of the 5x5 chamfer mask with the DIST_L2
 * weights {1, 1.4, 2.1969} in 16-bit fixed point (65536, 91750, 143976), a border of
 * INIT_DIST0 = INT_MAX >> 2 around the image, distances of pixels with bw == 0 are 0.
 * Writes the raw fixed-point distances (the float image is t0 * (1.f / 65536)). */
int oracle_chamfer5(const uint8_t* bw, int rows, int cols, uint32_t* out)
{
    enum { B = 2 };
    const uint32_t HV = 65536u, DG = 91750u, LG = 143976u, INIT = 0x7fffffffu >> 2;
    const int st = cols + 2 * B;
    uint32_t* t = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)st * (size_t)(rows + 2 * B));
    if (!t) return -3;
    for (int i = 0; i < B; i++)
        for (int j = 0; j < st; j++) {
            t[(size_t)i * st + j] = INIT;
            t[(size_t)(rows + 2 * B - 1 - i) * st + j] = INIT;
        }
    for (int i = 0; i < rows; i++) {
        uint32_t* r = t + (size_t)(i + B) * st + B;
        const uint8_t* s = bw + (size_t)i * cols;
        for (int j = 0; j < B; j++) r[-j - 1] = r[cols + j] = INIT;
        for (int j = 0; j < cols; j++) {
            if (!s[j]) { r[j] = 0; continue; }
            uint32_t t0 = r[j - 2 * st - 1] + LG, v;
            v = r[j - 2 * st + 1] + LG; if (t0 > v) t0 = v;
            v = r[j - st - 2] + LG; if (t0 > v) t0 = v;
            v = r[j - st - 1] + DG; if (t0 > v) t0 = v;
            v = r[j - st] + HV; if (t0 > v) t0 = v;
            v = r[j - st + 1] + DG; if (t0 > v) t0 = v;
            v = r[j - st + 2] + LG; if (t0 > v) t0 = v;
            v = r[j - 1] + HV; if (t0 > v) t0 = v;
            r[j] = t0;
        }
    }
    for (int i = rows - 1; i >= 0; i--) {
        uint32_t* r = t + (size_t)(i + B) * st + B;
        for (int j = cols - 1; j >= 0; j--) {
            uint32_t t0 = r[j], v;
            if (t0 > HV) {
                v = r[j + 2 * st + 1] + LG; if (t0 > v) t0 = v;
                v = r[j + 2 * st - 1] + LG; if (t0 > v) t0 = v;
                v = r[j + st + 2] + LG; if (t0 > v) t0 = v;
                v = r[j + st + 1] + DG; if (t0 > v) t0 = v;
                v = r[j + st] + HV; if (t0 > v) t0 = v;
                v = r[j + st - 1] + DG; if (t0 > v) t0 = v;
                v = r[j + st - 2] + LG; if (t0 > v) t0 = v;
                v = r[j + 1] + HV; if (t0 > v) t0 = v;
                r[j] = t0;
            }
            out[(size_t)i * cols + j] = t0;
        }
    }
    free(t);
    return 0;
}
