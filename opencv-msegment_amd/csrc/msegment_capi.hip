// msegment_capi.hip -- host engine + C ABI of libmsegment (see include/msegment.h).
//
// One translation unit with the kernels (no relocatable device code needed).  The flood is
// driven from the host as a stream of fixed 3-kernel iterations (resolve -> scan -> scatter);
// every kernel reads the current batch from the device control block, so the host never needs
// the batch size: it only polls a pinned "done" word once per group of iterations, with one
// group always queued ahead so the GPU never idles on the poll.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/msegment.h"
#include "ws_kernels.hip"
#include "spec_kernels.hip"
#include "nc_kernels.hip"
#include "shape_kernels.hip"
#include "color_kernels.hip"

#include <hipcub/hipcub.hpp>

using namespace msg;

struct msg_ctx {
  int dev = 0;
  hipStream_t own = nullptr;
  std::string err;
  Ctl* d_ctl = nullptr;
  // flood workspace (sized for cap_n pixels, cap_np tiled pixel words, cap_rc raster chunks)
  long long cap_n = 0, cap_np = 0, cap_rc = 0;
  // tiled states [0, cap_np) then tiled weights [cap_np, 2 cap_np), each with a one-tile-row
  // margin either side of the frame's tiles
  int32_t* d_px_base = nullptr;
  int32_t* d_px = nullptr;       // states of the frame's tiles = d_px_base + margin
  int32_t *d_qbuf = nullptr, *d_ilist = nullptr;
  int32_t *d_cnt = nullptr, *d_coff = nullptr, *d_tot = nullptr, *d_choff = nullptr;
  unsigned* d_capp = nullptr;  // CAP_SLOTS x NQ
  bool capp_clean = false;     // d_capp is zero (k_init_scan clears it after reading it)
  unsigned long long *d_tl = nullptr, *d_desc = nullptr, *d_cflag = nullptr;
  long long qcap = 0;
  // speculative generations (spec_kernels.hip): allocated on the first flood that may use them
  bool fast = true;             // msg_set_fast_commit: two-launch iterations for large batches
  bool spec = true;             // msg_set_speculative
  long long spec_np = 0, spec_logcap = 0;
  SpecPx* d_spx = nullptr;       // per tiled pixel: both parities' claims and labels, final claim
  unsigned long long *d_stl = nullptr, *d_slog = nullptr;
  unsigned long long *d_ssig = nullptr, *d_stmp = nullptr, *d_sflag = nullptr, *d_sxp = nullptr;
  long long spec_xcap = 0;       // d_sxp entries (k_spec_round's per-round chunk pool)
  int4* d_srec = nullptr;
  int2* d_sfrec = nullptr;
  unsigned* d_sdirt = nullptr;
  unsigned stag = 0;            // last round tag used (claims carry it; never reused)
  int spec_grid = 0;            // k_spec_round blocks
  // staging for the host-buffer entry points
  long long stage_n = 0;
  uint8_t* d_img = nullptr;
  int32_t* d_mk = nullptr;
  uint8_t* d_dst = nullptr;
  uint8_t* d_gray = nullptr;
  uint8_t* d_pal = nullptr;
  size_t pal_cap = 0;
  // host-mapped progress mirror {iteration, done, error, remaining}, written by k_scatter
  int* h_mir = nullptr;
  int* d_mir = nullptr;  // its device address
  Ctl* h_tail = nullptr;  // pinned copy of the control block read back at the end of a flood
  Ctl* d_tail = nullptr;  // its device address (k_tail writes it)
  int tail_seq = 0;       // k_tail's last release into h_mir[7]
  // ordering with the legacy null stream for device calls given stream = NULL (StreamScope)
  hipEvent_t ev_in = nullptr, ev_out = nullptr;
  unsigned epoch = 1;
  int group = 8;
  int res_grid = 0;   // k_resolve blocks per launch (occupancy x CUs by default; a perf knob)
  bool res_grid_set = false;  // msg_set_resolve_grid chose it (batches then keep it as it is)
  int commit_subs = FAST_SUBS;  // k_commit_fast sub-round blocks: the whole chip, or a share of it
                                // per flood when a batch keeps several in flight (run_batch)
  msg_stats stats{};
  // optional per-kernel HIP-event profiling (msg_set_profiling)
  bool prof = false;
  unsigned long long* d_diag = nullptr;  // 8 counters when diagnostics are on
  bool diag = false;
  int diag_bank = 0;  // msg_set_diag(ctx, 3): report bank 2 (the small-batch loop's regime split)
  int inject = 0;  // msg_set_diag(ctx, 2): k_resolve give-up injection (tests)
  std::vector<hipEvent_t> evpool;
  size_t evused = 0;
  std::vector<std::pair<int, size_t>> recs;  // (kernel id, index of the start event)
  double prof_ms[MSG_NKERNELS] = {};
  long long prof_n[MSG_NKERNELS] = {};
  // batches: floods in flight (msg_set_batch_inflight) and the sub-contexts that run them, each
  // with its own stream and workspace on this device (independent floods overlap: each is
  // latency-bound), created on first use
  int inflight = 4;
  std::vector<msg_ctx*> subs;
  // many-floods batches (msg_set_batch_floods): one workspace per frame of the call, the Ws array
  // k_serial_multi reads, and the per-flood "still running" flags it leaves
  int many = 3;                  // 0 off, 1 every flood serial to the end, 2 hand back to batches,
                                 // 3 automatic (the default: choose_mode)
  long long auto_key = -1;       // mode 3: frame size (rows << 32 | cols) the last probe was taken on
  int auto_mode = -1;            //         and the mode it chose (0 or 1)
  std::vector<msg_ctx*> msubs;
  Ws* d_wss = nullptr;
  int wss_cap = 0;
  uint8_t* d_mstage = nullptr;   // host-buffer many-floods batches: every frame's image + markers
  long long mstage_cap = 0;
  // host-buffer batches over several devices (msg_set_batch_devices): the device list and one
  // sub-context per entry (created on first use), each running its contiguous block of frames
  std::vector<int> bdevs;
  std::vector<msg_ctx*> dsubs;
  // the eager speculative workspace failed with ENOMEM for frames of this many tiled pixels: frames
  // at least this large go straight to the lazy path (cleared by msg_set_speculative)
  long long spec_eager_failed_np = 0;
  // marker stage: device histogram + its pinned host mirror, gray scratch
  int cus = 0;
  unsigned* d_hist = nullptr;  // 256 bins
  unsigned* h_hist = nullptr;
  uint8_t* d_gscr = nullptr;
  long long gscr_n = 0;
  uint8_t* d_gscr2 = nullptr;  // unblurred gray of the NC MEDIAN_BLUR branch
  long long gscr2_n = 0;
  // NC BILATERIAL branch: the disc of taps (device copy and the host table it is uploaded from,
  // kept until the stage's histogram read-back has synchronised the stream)
  BilTap* d_btaps = nullptr;
  long long btaps_n = 0;
  std::vector<BilTap> h_btaps;
  // shape marker stage: 6 byte planes, 2 int planes (parents, block keys), 2 block-key arrays,
  // scan scratch, 4 counters
  long long sh_n = 0, sh_nb = 0;
  uint8_t* d_sh8 = nullptr;
  int* d_sh32 = nullptr;
  int *d_shF = nullptr, *d_shP = nullptr, *d_shcnt = nullptr;
  void* d_scan_tmp = nullptr;
  size_t scan_tmp_bytes = 0;
  // colour marker stage: 5 int planes (distances, fg / bg components, region labels x 2), the
  // region lists, sweep flags and counters
  long long cm_n = 0;
  int* d_cm32 = nullptr;
  int2* d_cmreg = nullptr;
  int* d_cmcnt = nullptr;
};

namespace {

enum KernelId { KID_PREP, KID_INIT_SCAN, KID_COMPACT, KID_RESOLVE, KID_SCAN, KID_SCATTER,
                KID_COLORIZE, KID_EDGE, KID_UNTILE, KID_GRAY_HIST, KID_NC_MARKERS, KID_SPEC_ROUND,
                KID_GRAY, KID_MEDIAN, KID_CANNY, KID_CCL, KID_RING, KID_NUMBER, KID_HOLES, KID_SPEC_FLATTEN,
                KID_COLOR, KID_BILATERAL, KID_COMMIT_FAST, KID_SERIAL_MULTI };
const char* const kKernelNames[MSG_NKERNELS] = {"k_prep", "k_init_scan", "k_compact", "k_resolve",
                                                "k_scan", "k_scatter", "k_colorize",
                                                "k_edge_weights", "k_untile", "k_gray_hist",
                                                "k_nc_markers", "k_spec_round", "k_gray",
                                                "k_median", "k_canny_nms", "k_ccl", "k_ring_median3",
                                                "k_cc_number", "k_holes", "k_spec_flatten",
                                                "k_color_stage", "k_bilateral", "k_commit_fast",
                                                "k_serial_multi"};

hipEvent_t pool_event(msg_ctx* c) {
  if (c->evused == c->evpool.size()) {
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    c->evpool.push_back(e);
  }
  return c->evpool[c->evused++];
}

// Launch with optional start/stop events on the launch stream.
#define LAUNCH(c, kid, st, kern, grid, block, shm, ...)                                     \
  do {                                                                                   \
    size_t i0_ = 0;                                                                      \
    if ((c)->prof) {                                                                     \
      i0_ = (c)->evused;                                                                 \
      hipEvent_t a_ = pool_event(c), b_ = pool_event(c);                                 \
      if (a_ && b_) (void)hipEventRecord(a_, st);                                        \
      else (c)->prof = false;                                                            \
    }                                                                                    \
    hipLaunchKernelGGL(kern, grid, block, shm, st, __VA_ARGS__);                         \
    if ((c)->prof) {                                                                     \
      (void)hipEventRecord((c)->evpool[i0_ + 1], st);                                    \
      (c)->recs.emplace_back((int)(kid), i0_);                                           \
    }                                                                                    \
  } while (0)

// Fold recorded event pairs into the per-kernel totals (stream must be synchronised).
void collect_profile(msg_ctx* c) {
  for (auto& r : c->recs) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, c->evpool[r.second], c->evpool[r.second + 1]) == hipSuccess) {
      c->prof_ms[r.first] += ms;
      c->prof_n[r.first] += 1;
    }
  }
  c->recs.clear();
  c->evused = 0;
}

int fail(msg_ctx* c, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  return code;
}

#define HIPCHK(c, call)                                                                      \
  do {                                                                                       \
    hipError_t e_ = (call);                                                                  \
    if (e_ != hipSuccess)                                                                    \
      return fail((c), e_ == hipErrorOutOfMemory ? MSG_ENOMEM : MSG_EHIP, "%s: %s (%s:%d)", \
                  #call, hipGetErrorString(e_), __FILE__, __LINE__);                         \
  } while (0)

// Device entry points with stream == NULL run on the context's own non-blocking stream, which
// does not order with the legacy null stream that e.g. torch's default stream is.  The scope
// makes the own stream wait for the null stream's work on entry, and the null stream wait for
// the own stream's work on exit, so stream = NULL behaves like the caller's default stream.
struct StreamScope {
  msg_ctx* c;
  hipStream_t st;
  int rc = MSG_OK;
  bool joined = false;
  StreamScope(msg_ctx* c_, void* stream) : c(c_), st(stream ? (hipStream_t)stream : c_->own) {
    if (stream) return;
    if (hipEventRecord(c->ev_in, nullptr) != hipSuccess || hipStreamWaitEvent(c->own, c->ev_in, 0) != hipSuccess)
      rc = fail(c, MSG_EHIP, "cannot order the context stream after the null stream");
    else
      joined = true;
  }
  ~StreamScope() {
    if (!joined) return;
    if (hipEventRecord(c->ev_out, c->own) == hipSuccess) (void)hipStreamWaitEvent(nullptr, c->ev_out, 0);
  }
};

template <class T>
void dfree(T*& p) {
  if (p) (void)hipFree((void*)p);
  p = nullptr;
}

void free_flood(msg_ctx* c) {
  dfree(c->d_px_base);
  c->d_px = nullptr;
  dfree(c->d_qbuf); dfree(c->d_ilist);
  dfree(c->d_cnt); dfree(c->d_coff); dfree(c->d_tot); dfree(c->d_choff); dfree(c->d_capp);
  dfree(c->d_tl); dfree(c->d_desc); dfree(c->d_cflag);
  c->cap_n = c->cap_np = c->cap_rc = 0;
  c->qcap = 0;
}

void free_spec(msg_ctx* c) {
  dfree(c->d_spx); dfree(c->d_stl); dfree(c->d_slog); dfree(c->d_ssig);
  dfree(c->d_stmp); dfree(c->d_sflag); dfree(c->d_srec); dfree(c->d_sfrec); dfree(c->d_sdirt);
  dfree(c->d_sxp);
  c->spec_np = c->spec_logcap = c->spec_xcap = 0;
  c->stag = 0;
}

// Speculative-generation workspace for np tiled pixels (n frame pixels): the SpecPx record (round
// claims and labels of both parities, final claim: 32 B), change marks (2 x 4 B) and the
// generation log (32 B) per pixel, per-rank arrays for
// SPEC_WIN items, SPEC_RL records of scratch per k_spec_round thread.  Tags start at 1 on a
// zeroed claim space and are never reused; near 2^31 the space is zeroed again.
int ensure_spec(msg_ctx* c, long long np, long long n, hipStream_t st) {
  const long long logcap = 4 * n + (1 << 20);
  if (np <= c->spec_np && logcap <= c->spec_logcap && c->stag < 0x70000000u) return MSG_OK;
  if (np > c->spec_np || logcap > c->spec_logcap) {
    free_spec(c);
    const long long slots = (long long)c->spec_grid * SPEC_BS;
    HIPCHK(c, hipMalloc((void**)&c->d_spx, np * sizeof(SpecPx)));
    HIPCHK(c, hipMalloc((void**)&c->d_sdirt, 2 * np * sizeof(unsigned)));
    HIPCHK(c, hipMalloc((void**)&c->d_stl, (size_t)SPEC_WIN * 8));
    HIPCHK(c, hipMalloc((void**)&c->d_slog, logcap * 8));
    HIPCHK(c, hipMalloc((void**)&c->d_srec, (size_t)2 * SPEC_WIN * sizeof(int4)));
    HIPCHK(c, hipMalloc((void**)&c->d_ssig, (size_t)2 * SPEC_WIN * 8));
    HIPCHK(c, hipMalloc((void**)&c->d_sfrec, (size_t)SPEC_WIN * sizeof(int2)));
    HIPCHK(c, hipMalloc((void**)&c->d_stmp, slots * SPEC_RL * 8));
    HIPCHK(c, hipMalloc((void**)&c->d_sflag, (size_t)(SPEC_WIN / SPEC_FT + 2) * 8));
    // a round's cold cascade queues and long executions' records (8 B each): a pool of 2 per
    // tiled pixel, at least 2^24 (an exhausted pool is a capacity overflow: serial pops, exact)
    c->spec_xcap = std::max<long long>(1ll << 24, 2 * np);
    HIPCHK(c, hipMalloc((void**)&c->d_sxp, c->spec_xcap * 8));
    c->spec_np = np;
    c->spec_logcap = logcap;
  }
  HIPCHK(c, hipMemsetAsync(c->d_spx, 0, c->spec_np * sizeof(SpecPx), st));
  HIPCHK(c, hipMemsetAsync(c->d_sdirt, 0, 2 * c->spec_np * sizeof(unsigned), st));
  HIPCHK(c, hipMemsetAsync(c->d_stl, 0, (size_t)SPEC_WIN * 8, st));
  HIPCHK(c, hipMemsetAsync(c->d_sflag, 0, (size_t)(SPEC_WIN / SPEC_FT + 2) * 8, st));
  c->stag = 0;
  return MSG_OK;
}

void free_stage(msg_ctx* c) {
  dfree(c->d_img); dfree(c->d_mk); dfree(c->d_dst); dfree(c->d_gray);
  c->stage_n = 0;
}

long long tile_margin(int W) { return 16ll * ((W + 3) / 4 + 1); }  // tiled entries

int ensure_flood(msg_ctx* c, int H, int W, hipStream_t st) {
  const long long N = (long long)H * W;
  // + a margin of one tile row (+ one tile) before and after: k_resolve's speculative
  // radius-2 loads around frame-adjacent pixels may land there (values discarded)
  const long long Np = (long long)((H + 3) / 4) * ((W + 3) / 4) * 16 + 2 * tile_margin(W);
  const long long nrc = (long long)H * ((W + RSEG - 1) / RSEG);
  if (N <= c->cap_n && Np <= c->cap_np && nrc <= c->cap_rc) return MSG_OK;
  const long long n = std::max(N, c->cap_n), np = std::max(Np, c->cap_np), rc = std::max(nrc, c->cap_rc);
  free_flood(c);
  const long long nch = (n + CH - 1) / CH;
  const long long qcap = 4 * n + 16;
  HIPCHK(c, hipMalloc((void**)&c->d_px_base, np * 8));  // np states + np weights
  // stream-ordered: a null-stream hipMemset does not order with the non-blocking flood stream
  // and could land after k_prep's first writes (seen as an all-zero label map / ERR_STATE on
  // the first flood of a fresh batch sub-context)
  HIPCHK(c, hipMemsetAsync(c->d_px_base, 0, np * 8, st));
  HIPCHK(c, hipMalloc((void**)&c->d_ilist, n * 4));
  HIPCHK(c, hipMalloc((void**)&c->d_qbuf, qcap * 4));
  HIPCHK(c, hipMalloc((void**)&c->d_tl, n * 8));
  HIPCHK(c, hipMalloc((void**)&c->d_desc, n * 8));
  HIPCHK(c, hipMalloc((void**)&c->d_cnt, nch * NQ * 4));
  HIPCHK(c, hipMalloc((void**)&c->d_coff, nch * NQ * 4));
  HIPCHK(c, hipMalloc((void**)&c->d_tot, rc * 4));
  HIPCHK(c, hipMalloc((void**)&c->d_choff, rc * 4));
  HIPCHK(c, hipMalloc((void**)&c->d_capp, (size_t)CAP_SLOTS * NQ * 4));
  c->capp_clean = false;
  HIPCHK(c, hipMemsetAsync(c->d_tl, 0, n * 8, st));
  HIPCHK(c, hipMalloc((void**)&c->d_cflag, (size_t)(n / RBS + 2) * 16));
  HIPCHK(c, hipMemsetAsync(c->d_cflag, 0, (size_t)(n / RBS + 2) * 16, st));
  c->epoch = 1;
  c->cap_n = n;
  c->cap_np = np;
  c->cap_rc = rc;
  c->qcap = qcap;
  return MSG_OK;
}

int ensure_stage(msg_ctx* c, long long N) {
  if (N <= c->stage_n) return MSG_OK;
  free_stage(c);
  HIPCHK(c, hipMalloc((void**)&c->d_img, N * 3 + 16));
  HIPCHK(c, hipMalloc((void**)&c->d_mk, N * 4 + 16));
  HIPCHK(c, hipMalloc((void**)&c->d_dst, N * 3 + 16));
  HIPCHK(c, hipMalloc((void**)&c->d_gray, N + 16));
  c->stage_n = N;
  return MSG_OK;
}

// Frame-size limits.  The flood indexes its tiled state (4x4 tiles plus a tile row of margin
// either side) and its bucket FIFOs (up to 4 slots per pixel; slot s is stored as the state
// -3 - s, which must stay clear of the phase-1 states 0x80000000 | level) with 32-bit ints, so
// 4N + 16 and the padded tiled count stay below 2^31 - 512: frames up to ~2^29 pixels
// (23168^2, 16384 x 32767).  Byte offsets of the BGR frame (3N < 1.61e9) fit signed 32 bits
// there too.  The marker stages are audited for 2^28 pixels only and keep that bound.
constexpr long long kStageMaxPixels = 1ll << 28;
constexpr long long kFloodIndexLimit = (1ll << 31) - 512;

int check_size(msg_ctx* c, int rows, int cols, bool flood = false) {
  if (rows < 0 || cols < 0) return fail(c, MSG_EINVAL, "negative size %d x %d", rows, cols);
  const long long N = (long long)rows * cols;
  if (!flood) {
    if (N > kStageMaxPixels)
      return fail(c, MSG_EINVAL, "frame too large for the marker stage: %d x %d (2^28 pixels at most)", rows, cols);
    return MSG_OK;
  }
  const long long Np = (long long)((rows + 3) / 4) * ((cols + 3) / 4) * 16 + 2 * tile_margin(cols);
  if (4 * N + 16 >= kFloodIndexLimit || Np >= kFloodIndexLimit)
    return fail(c, MSG_EINVAL, "frame too large for the flood's 32-bit indices: %d x %d (about 2^29 pixels at most)",
                rows, cols);
  return MSG_OK;
}

// Spin on the host-mapped progress mirror until iteration `target` has reported.  A stream that
// drains (or fails) without the report ends the wait with an error instead of spinning forever.
int wait_mirror(msg_ctx* c, hipStream_t st, int word, int target) {
  for (unsigned spins = 1;; ++spins) {
    if (__atomic_load_n(&c->h_mir[word], __ATOMIC_ACQUIRE) >= target) return MSG_OK;
    if ((spins & 4095) == 0) {
      const hipError_t q = hipStreamQuery(st);
      if (q == hipSuccess) {
        if (__atomic_load_n(&c->h_mir[word], __ATOMIC_ACQUIRE) >= target) return MSG_OK;
        return fail(c, MSG_ESTATE, "stream drained before mirror word %d reached %d", word, target);
      }
      if (q != hipErrorNotReady) return fail(c, MSG_EHIP, "flood stream: %s", hipGetErrorString(q));
    }
    __builtin_ia32_pause();
  }
}
int wait_progress(msg_ctx* c, hipStream_t st, int target) { return wait_mirror(c, st, 0, target); }

// A flood in progress on a context: its kernel arguments and the host loop's regime flags.
struct FloodRun {
  Ws ws;
  int H = 0, W = 0;
  long long N = 0, ntiled = 0;
  bool spec = false, spec_bound = false;
  hipStream_t st = nullptr;
};

void bind_spec(msg_ctx* c, FloodRun& fr, bool on) {
  Ws& ws = fr.ws;
  ws.spx = on ? c->d_spx : nullptr; ws.stl = on ? c->d_stl : nullptr;
  ws.slog = on ? c->d_slog : nullptr; ws.srec = on ? c->d_srec : nullptr;
  ws.ssig = on ? c->d_ssig : nullptr; ws.sfrec = on ? c->d_sfrec : nullptr;
  ws.stmp = on ? c->d_stmp : nullptr; ws.sflag = on ? c->d_sflag : nullptr;
  ws.sdirt = on ? c->d_sdirt : nullptr;
  ws.sxp = on ? c->d_sxp : nullptr;
  ws.sxcap = on ? std::min<long long>(c->spec_xcap, 0x7fffffffll) : 0;
  ws.snp = on ? c->spec_np : 0;
  ws.slogcap = on ? c->spec_logcap : 0;
  ws.spec_lazy = (fr.spec && !on) ? 1 : 0;
}

// The exact flood on device buffers, in the context's tiled workspace: flood_begin sets it up and
// queues phase 1 (k_prep .. k_scatter), flood_loop runs the host loop of iterations until the
// flood is done, flood_end writes the row-major label map into d_labels (may alias d_mk_in) fused
// with the colourisation when d_dst is given, and reads the counters back.  run_flood = all three;
// the many-floods batch (batch_many) runs k_serial_multi between the first two.
int flood_begin(msg_ctx* c, const uint8_t* d_img, const int32_t* d_mk_in, int H, int W, hipStream_t st,
                FloodRun& fr, bool multi = false) {
  const long long N = (long long)H * W;
  c->stats = msg_stats{};
  c->stats.rows = H;
  c->stats.cols = W;
  fr.H = H;
  fr.W = W;
  fr.N = N;
  fr.st = st;
  fr.ws = Ws{};  // a zero-pixel flood keeps ctl == nullptr: k_serial_multi skips it
  if (N == 0) return MSG_OK;
  int rc = ensure_flood(c, H, W, st);
  if (rc) return rc;
  if (c->epoch > 0x70000000u) {  // granule bit 63 flags a provisional value
    HIPCHK(c, hipMemsetAsync(c->d_tl, 0, c->cap_n * 8, st));
    HIPCHK(c, hipMemsetAsync(c->d_cflag, 0, (size_t)(c->cap_n / RBS + 2) * 16, st));
    c->epoch = 1;
  }
  Ws& ws = fr.ws;
  ws = Ws{};
  ws.img = d_img;
  c->d_px = c->d_px_base + tile_margin(W);
  ws.mk = c->d_px;
  ws.w4 = c->d_px_base + c->cap_np + tile_margin(W);
  ws.marg = (int)tile_margin(W);
  ws.qbuf = c->d_qbuf;
  ws.ilist = c->d_ilist;
  ws.tl = c->d_tl;
  ws.desc = c->d_desc;
  ws.ipx = c->d_ilist;
  ws.cnt = c->d_cnt;
  ws.coff = c->d_coff;
  ws.tot = c->d_tot;
  ws.choff = c->d_choff;
  ws.capp = c->d_capp;
  ws.cflag = c->d_cflag;
  ws.ctl = c->d_ctl;
  ws.diag = c->diag ? c->d_diag : nullptr;

  ws.hmir = c->d_mir;
  ws.multi = multi ? 1 : 0;
  ws.H = H;
  ws.W = W;
  ws.Wt = (W + 3) / 4;
  ws.nseg = (W + RSEG - 1) / RSEG;
  ws.N = N;
  ws.qcap = c->qcap;

  // speculative generations: tiled indices must fit their 28-bit log field.  The engine's
  // workspace (~64 B/px) is allocated up front for frames of 2^20 tiled pixels or more, lazily
  // for smaller ones (once a flood of this context has entered the interrupt-dense regime, which
  // k_scan reports through the progress mirror).  Round 4: allocated in the middle of a flood,
  // the first flood of a context on uniform noise at 4096^2 took 16.2 s (the later ones 1.45 s;
  // scripts/first_flood.py).  From then on it is kept (msg_set_speculative(ctx, 0) frees it).
  fr.ntiled = (long long)((H + 3) / 4) * ws.Wt * 16;
  fr.spec = c->spec && !multi && fr.ntiled <= (1ll << 28) && H >= 3 && W >= 3;
  fr.spec_bound = false;
  const bool eager_failed = c->spec_eager_failed_np > 0 && fr.ntiled >= c->spec_eager_failed_np;
  if (fr.spec && (c->spec_np >= fr.ntiled || (!eager_failed && (c->spec_np > 0 || fr.ntiled >= (1ll << 20))))) {
    rc = ensure_spec(c, fr.ntiled, N, st);
    if (rc == MSG_ENOMEM) {  // out of memory up front: the lazy path (only a flood that enters
      free_spec(c);          // the regime needs the engine, and it fails there if memory is short)
      (void)hipGetLastError();
      c->err.clear();
      // remembered: later floods of this size or larger skip the failing eager allocation
      c->spec_eager_failed_np = fr.ntiled;
    } else if (rc) {
      return rc;
    } else {
      fr.spec_bound = true;
    }
  }
  bind_spec(c, fr, fr.spec_bound);
  const int npx = (int)((N + CH - 1) / CH);
  const int gsc = std::min(npx * (CH / 1024), 1024);
  // the control block and the level histograms are zeroed by the phase-0 kernel (prep_zero), the
  // capacity histograms by k_init_scan after reading them: a host memset only when a flood
  // stopped in between (or the buffer is new)
  if (!c->capp_clean) HIPCHK(c, hipMemsetAsync(c->d_capp, 0, (size_t)CAP_SLOTS * NQ * 4, st));
  c->capp_clean = false;
  if (c->diag) HIPCHK(c, hipMemsetAsync(c->d_diag, 0, 32 * sizeof(unsigned long long), st));
  (void)npx;
  const int nrc = H * ws.nseg;  // raster chunks
  // k_prep4 (one thread per tile) where widths and buffers allow 12-B / 16-B quad loads
  if (W % 4 == 0 && ((uintptr_t)d_img & 3) == 0 && ((uintptr_t)d_mk_in & 15) == 0)
    LAUNCH(c, KID_PREP, st, k_prep4, dim3((H + 3) / 4 * ws.nseg), dim3(PREP4_T), 0, ws, d_mk_in);
  else
    LAUNCH(c, KID_PREP, st, k_prep, dim3((H + 3) / 4 * ws.nseg), dim3(RSEG), 0, ws, d_mk_in);
  LAUNCH(c, KID_INIT_SCAN, st, k_init_scan, dim3(1), dim3(1024), 0, ws, nrc, c->epoch, c->stag);
  c->capp_clean = hipPeekAtLastError() == hipSuccess;
  LAUNCH(c, KID_COMPACT, st, k_compact, dim3((nrc + 4 * CPW - 1) / (4 * CPW)), dim3(256), 0, ws, nrc);
  LAUNCH(c, KID_SCAN, st, k_scan, dim3(1), dim3(1024), 0, ws, 0);
  LAUNCH(c, KID_SCATTER, st, k_scatter, dim3(gsc), dim3(1024), 0, ws, -1);
  HIPCHK(c, hipGetLastError());
  return MSG_OK;
}

int flood_loop(msg_ctx* c, FloodRun& fr) {
  if (fr.N == 0) return MSG_OK;
  Ws& ws = fr.ws;
  ws.multi = 0;  // from here on the full engine, small-batch loop included
  hipStream_t st = fr.st;
  const long long N = fr.N;
  const int npx = (int)((N + CH - 1) / CH);
  const int gres = std::max(1, std::min(c->res_grid, (int)((N + RBS - 1) / RBS)));
  const int gsc = std::min(npx * (CH / 1024), 1024);
  int rc = MSG_OK;
  // Host loop: groups of iterations, one group always queued ahead.  Progress comes from the
  // host-mapped mirror that each iteration's k_scatter writes (no copy kernel, no event wait):
  // after queueing a group the host spins until the previous group's last iteration reported.
  __atomic_store_n(&c->h_mir[0], -1, __ATOMIC_RELEASE);
  c->h_mir[4] = 0;
  c->h_mir[5] = 0;
  c->h_mir[8] = 0;
  // the first two groups are queued before any report: assume a large flood batch (two-launch
  // iterations), as phase 1's queue usually is -- a wrong guess costs a declined commit or a small
  // batch committed by the grid instead of k_scan's loop, never a wrong result (every kernel checks
  // the batch it serves).  The three-launch start cost the headline frame ~8 x 4 us (r05p trace).
  c->h_mir[6] = 1;
  int it = 0, prev_end = -1;
  c->group = 4;
  long long syncs = 0;
  // Two kinds of iteration, chosen per group from the regime the last poll reported (a stale
  // choice only costs no-op launches: every kernel checks the batch mode it serves, and k_scan
  // commits only decided batches): batches (k_resolve) or a speculative generation's rounds and
  // flattening (k_spec_round x SPEC_ITER_ROUNDS, k_spec_flatten), then the common commit.
  constexpr int SPEC_ITER_ROUNDS = 3;
  const int gflat = std::max(1, c->cus);
  for (;;) {
    const bool spec_it = fr.spec_bound && c->h_mir[4] != 0;
    // serial pops in a kernel of their own once the flood has reached that regime
    const bool ser_it = c->h_mir[8] != 0 && !ws.multi;
    // two-launch iterations while the last report was a large flood batch (k_commit_fast)
    const bool fast_it = !spec_it && c->fast && c->h_mir[6] != 0;
    for (int g = 0; g < c->group; ++g, ++it) {
      if (fast_it) {
        if (c->inject)  // test only: give-ups (msg_set_diag 2) -> k_commit_fast schedules re-runs
          LAUNCH(c, KID_RESOLVE, st, k_resolve<true>, dim3(gres), dim3(RBS), 0, ws);
        else
          LAUNCH(c, KID_RESOLVE, st, k_resolve<false>, dim3(gres), dim3(RBS), 0, ws);
        if (c->h_mir[6] == 2)  // the last report was a batch above FAST_CH chunks
          LAUNCH(c, KID_COMMIT_FAST, st, k_commit_fast_mp, dim3(FAST_SUBS + 1), dim3(1024), 0, ws, it);
        else if (c->commit_subs < FAST_SUBS)  // a share of the chip: FAST_PASS sub-rounds per block
          LAUNCH(c, KID_COMMIT_FAST, st, k_commit_fast_mp, dim3(c->commit_subs + 1), dim3(1024), 0, ws, it);
        else
          LAUNCH(c, KID_COMMIT_FAST, st, k_commit_fast, dim3(FAST_SUBS + 1), dim3(1024), 0, ws, it);
        continue;
      }
      if (spec_it) {
        for (int r = 0; r < SPEC_ITER_ROUNDS; ++r)
          LAUNCH(c, KID_SPEC_ROUND, st, k_spec_round, dim3(c->spec_grid), dim3(SPEC_BS), 0, ws);
        LAUNCH(c, KID_SPEC_FLATTEN, st, k_spec_flatten, dim3(gflat), dim3(SPEC_FT), 0, ws);
      } else if (c->inject) {  // test only: odd blocks give up their first chunk (msg_set_diag 2)
        LAUNCH(c, KID_RESOLVE, st, k_resolve<true>, dim3(gres), dim3(RBS), 0, ws);
      } else {
        LAUNCH(c, KID_RESOLVE, st, k_resolve<false>, dim3(gres), dim3(RBS), 0, ws);
      }
      // + small batches; in the serial regime k_serial_one pops what k_scan's loop hands it
      // (in a speculative iteration too: a cooldown's serial pops start in its k_scan)
      LAUNCH(c, KID_SCAN, st, k_scan, dim3(1), dim3(1024), 0, ws, ser_it ? 1 : 0);
      if (ser_it) LAUNCH(c, KID_SERIAL_MULTI, st, k_serial_one, dim3(1), dim3(64), 0, ws);
      LAUNCH(c, KID_SCATTER, st, k_scatter, dim3(gsc), dim3(1024), 0, ws, it);
    }
    HIPCHK(c, hipGetLastError());
    if (prev_end >= 0) {
      rc = wait_progress(c, st, prev_end);
      if (rc) {  // iterations are still queued: let them drain before the context is reused
        (void)hipStreamSynchronize(st);
        return rc;
      }
      ++syncs;
      if (c->h_mir[1] || c->h_mir[2]) break;
      if (fr.spec && !fr.spec_bound && c->h_mir[5]) {
        // first entry into the serial regime: allocate the engine; launches from here on carry it
        // (the zero fills are stream-ordered after the iterations already queued, which run
        // without it, and before the first launch that may use it)
        rc = ensure_spec(c, fr.ntiled, N, st);
        if (rc) {  // queued iterations still write the shared progress mirror: drain them first
          (void)hipStreamSynchronize(st);
          return rc;
        }
        fr.spec_bound = true;
        bind_spec(c, fr, true);
      }
      // fewer queued items -> fewer batches left: shrink the group so that the iterations
      // enqueued past the end of the flood (no-ops, but each still a launch) stay few
      const int rem = c->h_mir[3];
      c->group = rem > (1 << 21) ? 8 : rem > (1 << 19) ? 4 : rem > (1 << 17) ? 2 : 1;
    }
    prev_end = it - 1;
  }
  c->stats.host_syncs += syncs;
  return MSG_OK;
}

int flood_end(msg_ctx* c, FloodRun& fr, int32_t* d_labels, int depth = 0, const uint8_t* d_pal = nullptr,
              uint8_t* d_dst = nullptr, uint8_t* d_gray = nullptr) {
  if (fr.N == 0) return MSG_OK;
  Ws& ws = fr.ws;
  hipStream_t st = fr.st;
  const int H = fr.H, W = fr.W;
  {
    const long long nrows = (long long)((H + 3) / 4) * ws.Wt * 4;  // one tile row per lane
    const int grid = (int)std::min<long long>((nrows + 255) / 256, 1 << 20);
    const size_t shm = (d_dst && d_pal && depth <= PAL_LDS_MAX) ? (size_t)std::max(depth, 1) * 4 : 0;
    LAUNCH(c, KID_UNTILE, st, k_untile, dim3(grid), dim3(256), shm, c->d_px, H, W, ws.Wt, d_labels,
           depth, d_pal, d_dst, d_gray, &c->d_ctl->error);
    HIPCHK(c, hipGetLastError());
  }
  unsigned long long dgv[32] = {0};
  if (c->diag || c->prof) {  // (the counters' copy and the profile's events want the stream drained)
    // into pinned memory: a copy to pageable memory is staged and synchronous on its own
    HIPCHK(c, hipMemcpyAsync(c->h_tail, c->d_ctl, sizeof(Ctl), hipMemcpyDeviceToHost, st));
    if (c->diag) HIPCHK(c, hipMemcpyAsync(dgv, c->d_diag, sizeof(dgv), hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
  } else {
    const int seq = ++c->tail_seq;
    LAUNCH(c, KID_UNTILE, st, k_tail, dim3(1), dim3(256), 0, c->d_ctl, c->d_tail, c->d_mir, seq);
    HIPCHK(c, hipGetLastError());
    const int rc = wait_mirror(c, st, 7, seq);
    if (rc) {
      (void)hipStreamSynchronize(st);
      return rc;
    }
  }
  const Ctl& tail = *c->h_tail;
  c->stats.host_syncs += 1;
  if (c->prof) collect_profile(c);
  c->stats.batches = tail.batches;
  c->stats.pops = tail.pops;
  c->stats.items = tail.items;
  c->stats.pushes = tail.pushes;
  // k_commit_fast's share is what the other commit paths leave
  c->stats.fast_pops = std::max(0ll, tail.pops - tail.s0pops - tail.lpops);
  c->stats.fast_pushes = std::max(0ll, tail.pushes - tail.spushes - tail.lpushes);
  c->stats.scatter_pops = tail.spops;
  c->stats.scatter_pushes = tail.spushes;
  c->stats.resolve_items = tail.ritems;
  c->stats.spec_exec_pops = tail.spec.xpops;
  c->stats.spec_longest_pops = tail.spec.xlong;
  // when speculative generations ran, diag reports their round split instead (spec_kernels.hip)
  for (int k = 0; k < 8; ++k)
#ifdef MSEG_CF_PROF
    c->stats.diag[k] = (int64_t)dgv[8 + k];  // k_commit_fast's phase split (diagnostic build)
#else
    c->stats.diag[k] = (int64_t)dgv[c->diag_bank == 2 ? 16 + k : c->diag_bank == 3 ? 24 + k : tail.spec.gens ? 8 + k : k];
#endif
  c->stats.spec_generations = tail.spec.gens;
  c->stats.spec_rounds = tail.spec.rounds_total;
  c->stats.spec_executions = tail.spec.execs;
  c->stats.spec_replays = tail.spec.replays;
  c->stats.spec_cooldowns = tail.spec.cools;
  c->stats.spec_gen_pops = tail.spec.gpops_total;
  c->stats.spec_gen_us = tail.spec.gticks_total / 100;  // s_memrealtime: 100 MHz
  c->stats.spec_cascade_pops = tail.spec.cpops;
  c->stats.spec_fallbacks = tail.spec.fallbacks;
  if (fr.spec_bound) c->stag = tail.spec.T;
  c->epoch += (unsigned)std::min<long long>(tail.batches + 4, 0x7fffffff);
  if (tail.error & ERR_TIMEOUT)
    return fail(c, MSG_ETIMEOUT, "in-kernel wait timed out (grid not co-resident?)");
  if (tail.error & ERR_CAPACITY) return fail(c, MSG_ESTATE, "bucket capacity exceeded");
  if (tail.error & ERR_LEFTOVER) {
    unsigned long long lo[8] = {0};
    if (c->diag) {  // classify them (k_leftover_diag) for the message
      HIPCHK(c, hipMemsetAsync(c->d_diag, 0, 8 * sizeof(unsigned long long), st));
      const long long nt = (long long)((H + 3) / 4) * ws.Wt * 16;
      LAUNCH(c, KID_UNTILE, st, k_leftover_diag, dim3(1024), dim3(256), 0, ws, nt, c->d_diag);
      HIPCHK(c, hipMemcpyAsync(lo, c->d_diag, sizeof(lo), hipMemcpyDeviceToHost, st));
      HIPCHK(c, hipStreamSynchronize(st));
    }
    return fail(c, MSG_ESTATE, "queued pixels left at the end of the flood (%llu: phase-1 %llu, popped %llu, "
                "slot reused %llu; last tiled %llu slot %llu)", lo[3], lo[0], lo[1], lo[2], lo[4], lo[5]);
  }
  if (tail.error) return fail(c, MSG_ESTATE, "device consistency check failed (%d)", tail.error);
  if (!tail.done) return fail(c, MSG_ESTATE, "flood did not finish");
  return MSG_OK;
}

int run_flood(msg_ctx* c, const uint8_t* d_img, const int32_t* d_mk_in, int32_t* d_labels, int H,
              int W, hipStream_t st, int depth = 0, const uint8_t* d_pal = nullptr,
              uint8_t* d_dst = nullptr, uint8_t* d_gray = nullptr) {
  FloodRun fr;
  int rc = flood_begin(c, d_img, d_mk_in, H, W, st, fr);
  if (rc) return rc;
  rc = flood_loop(c, fr);
  if (rc) return rc;
  return flood_end(c, fr, d_labels, depth, d_pal, d_dst, d_gray);
}

int launch_colorize(msg_ctx* c, const int32_t* d_lab, long long N, int depth, const uint8_t* d_pal,
                    uint8_t* d_dst, uint8_t* d_gray, hipStream_t st) {
  if (N == 0) return MSG_OK;
  const long long th = (N + 3) / 4;
  const int grid = (int)std::min<long long>((th + 255) / 256, 2048);
  const size_t shm = (d_pal && depth <= PAL_LDS_MAX) ? (size_t)std::max(depth, 1) * 4 : 0;
  LAUNCH(c, KID_COLORIZE, st, k_colorize, dim3(grid), dim3(256), shm, d_lab, N, depth, d_pal, d_dst,
         d_gray);
  HIPCHK(c, hipGetLastError());
  return MSG_OK;
}

int upload_palette(msg_ctx* c, const uint8_t* pal, int depth, hipStream_t st) {
  const size_t need = (size_t)std::max(depth, 1) * 3;
  if (need > c->pal_cap) {
    dfree(c->d_pal);
    HIPCHK(c, hipMalloc((void**)&c->d_pal, need));
    c->pal_cap = need;
  }
  HIPCHK(c, hipMemcpyAsync(c->d_pal, pal, (size_t)depth * 3, hipMemcpyHostToDevice, st));
  return MSG_OK;
}

constexpr int MAX_INFLIGHT = 8;

// Batch totals: every counter of msg_stats summed over the frames, the frame size of the last one.
// diag is zeroed: a frame's diag is one of several banks (k_resolve cycles with a max-type slot, or
// the speculative round split), chosen per frame, so sums over frames would mix units and add
// maxima (msegment.h: diag is reported for single floods only).
// batch_mode / batch_probe are flags, not counts: the largest over the parts (e.g. the devices of a
// msg_set_batch_devices call).
void add_stats(msg_stats& tot, const msg_stats& s) {
  static_assert(sizeof(msg_stats) % sizeof(int64_t) == 0, "msg_stats is int64 fields only");
  const int64_t mode = std::max(tot.batch_mode, s.batch_mode), probe = std::max(tot.batch_probe, s.batch_probe);
  int64_t* t = reinterpret_cast<int64_t*>(&tot);
  const int64_t* a = reinterpret_cast<const int64_t*>(&s);
  for (size_t k = 0; k < sizeof(msg_stats) / sizeof(int64_t); ++k) t[k] += a[k];
  tot.rows = s.rows;
  tot.cols = s.cols;
  for (auto& d : tot.diag) d = 0;
  tot.batch_mode = mode;
  tot.batch_probe = probe;
}

int ensure_subs(msg_ctx* c, int k) {
  while ((int)c->subs.size() < k) {
    msg_ctx* sub = nullptr;
    const int rc = msg_create(&sub, c->dev, MSG_CREATE_HIGH_PRIORITY);
    if (rc) return fail(c, rc, "batch sub-context creation failed (%d)", rc);
    c->subs.push_back(sub);
  }
  return MSG_OK;
}

// fn(i, ctx) for frames i in [0, n): with inflight == 1 on c itself, else frame i on worker
// i % inflight (one host thread per sub-context, the API's one-context-per-thread model).
// Returns the first error, its text copied into c; stats = the sums over the frames.
template <class F>
int run_batch(msg_ctx* c, int n, F fn) {
  const int k = std::max(1, std::min({c->inflight, n, MAX_INFLIGHT}));
  msg_stats tot{};
  auto add = [&tot](const msg_stats& s) { add_stats(tot, s); };
  if (k == 1) {
    for (int i = 0; i < n; ++i) {
      const int rc = fn(i, c);
      if (rc) return rc;
      add(c->stats);
    }
    c->stats = tot;
    return MSG_OK;
  }
  int rc = ensure_subs(c, k);
  if (rc) return rc;
  // up to min(k, hardware queues) floods run kernels concurrently (streams beyond the HIP
  // runtime's hardware queues share them and serialise).  Concurrent k_resolve grids need not be
  // co-resident (a block waiting on an unclaimed chunk gives its own chunk up and the batch is
  // re-run, ws_kernels.hip), so each flood keeps the full grid.
  // k in flight: each flood's commit grid takes a 1/k share of the chip (its blocks then take up
  // to FAST_PASS sub-rounds each), so that concurrent floods' commits overlap instead of each
  // filling every wave slot; at least FAST_SUBS / FAST_PASS blocks (the batches reported as
  // fitting FAST_CH chunks still fit).
  const int csubs = std::max(FAST_SUBS / FAST_PASS, (FAST_SUBS / k) / (CH / 1024) * (CH / 1024));
  for (int w = 0; w < k; ++w) {
    c->subs[w]->commit_subs = csubs;
    // ... and, unless msg_set_resolve_grid chose one, half the default k_resolve grid (8 frames of
    // 4096^2, 4 in flight: 8833 -> 9230 Mpx/s, profiles/r04o_batch_grid_probe.log)
    c->subs[w]->res_grid = (c->res_grid_set || k < 2) ? c->res_grid : std::max(c->cus, c->res_grid / 2);
    c->subs[w]->spec = c->spec;
    c->subs[w]->fast = c->fast;
    if (c->subs[w]->diag != c->diag || c->subs[w]->inject != c->inject) {
      rc = msg_set_diag(c->subs[w], c->inject ? 2 : c->diag ? 1 : 0);
      if (rc) return rc;
    }
  }
  std::vector<int> rcs(k, MSG_OK);
  std::vector<msg_stats> st(k);
  std::vector<std::thread> th;
  for (int w = 0; w < k; ++w)
    th.emplace_back([&, w]() {
      msg_ctx* sub = c->subs[w];
      if (hipSetDevice(c->dev) != hipSuccess) {
        rcs[w] = MSG_EHIP;
        return;
      }
      msg_stats acc{};
      for (int i = w; i < n; i += k) {
        const int r = fn(i, sub);
        if (r) {
          rcs[w] = r;
          return;
        }
        add_stats(acc, sub->stats);
      }
      if (hipStreamSynchronize(sub->own) != hipSuccess) rcs[w] = MSG_EHIP;
      st[w] = acc;
    });
  for (auto& t : th) t.join();
  for (int w = 0; w < k; ++w) {
    if (rcs[w]) {
      c->err = c->subs[w]->err.empty() ? std::string("batch worker failed") : c->subs[w]->err;
      return rcs[w];
    }
    add(st[w]);
  }
  c->stats = tot;
  return MSG_OK;
}

// The many-floods mode's per-frame sub-contexts (~44 B/px each), Ws array and staging.
void release_many(msg_ctx* c) {
  for (msg_ctx* sub : c->msubs) msg_destroy(sub);
  c->msubs.clear();
  (void)hipSetDevice(c->dev);
  dfree(c->d_wss);
  c->wss_cap = 0;
  dfree(c->d_mstage);
  c->mstage_cap = 0;
}

// Many floods per launch (msg_set_batch_floods): every frame of the call gets a workspace of its
// own (a sub-context), phase 1 of each is queued on its stream with k_scan's small-batch loop off
// (FloodRun multi), then ONE k_serial_multi launch pops all of them, one wave per flood.  A flood
// that k_serial_multi leaves unfinished (mode 2: it handed back to batches after SERIAL_RUN clean
// pops) is finished by the full engine, up to `inflight` at a time, speculative generations off.
// frame(k, img, mk, H, W, lab, dst) describes frame k (device buffers; dst may be null).
template <class F>
int batch_many(msg_ctx* c, int n, int mode, int depth, const uint8_t* d_pal, F frame) {
  if (n == 0) {
    c->stats = msg_stats{};
    return MSG_OK;
  }
  while ((int)c->msubs.size() < n) {
    msg_ctx* sub = nullptr;
    const int rc = msg_create(&sub, c->dev, 0);
    if (rc) return fail(c, rc, "batch sub-context creation failed (%d)", rc);
    c->msubs.push_back(sub);
  }
  if (c->wss_cap < n) {
    dfree(c->d_wss);
    c->wss_cap = 0;
    HIPCHK(c, hipMalloc((void**)&c->d_wss, (size_t)n * sizeof(Ws)));
    c->wss_cap = n;
  }
  std::vector<FloodRun> frs(n);
  std::vector<Ws> h_ws(n);
  std::vector<hipEvent_t> ev(n + 1, nullptr);
  auto cleanup = [&]() {
    for (auto e : ev)
      if (e) (void)hipEventDestroy(e);
  };
  for (int k = 0; k <= n; ++k)
    if (hipEventCreateWithFlags(&ev[k], hipEventDisableTiming) != hipSuccess) {
      cleanup();
      return fail(c, MSG_EHIP, "hipEventCreate failed");
    }
  for (int k = 0; k < n; ++k) {
    msg_ctx* x = c->msubs[k];
    x->res_grid = c->res_grid;
    x->fast = c->fast;
    x->spec = false;  // the full engine finishes handed-back floods without the speculative engine
    const uint8_t* img;
    const int32_t* mk;
    int H, W;
    int32_t* lab;
    uint8_t* dst;
    frame(k, img, mk, H, W, lab, dst);
    int rc = check_size(x, H, W, true);
    if (!rc) rc = flood_begin(x, img, mk, H, W, x->own, frs[k], true);
    if (!rc && hipEventRecord(ev[k], x->own) != hipSuccess) rc = fail(x, MSG_EHIP, "hipEventRecord failed");
    if (rc) {
      c->err = x->err;
      for (int j = 0; j <= k; ++j) (void)hipStreamSynchronize(c->msubs[j]->own);
      cleanup();
      return rc;
    }
    h_ws[k] = frs[k].ws;
  }
  int rc = MSG_OK;
  const int run_limit = mode == 2 ? SERIAL_RUN : 0x7fffffff;
  // the Ws array (copied before any launch reads it: hipMemcpyAsync from pageable memory returns
  // once the source is consumed), then one wave per flood once every phase 1 is queued before it
  if (hipMemcpyAsync(c->d_wss, h_ws.data(), (size_t)n * sizeof(Ws), hipMemcpyHostToDevice, c->own) != hipSuccess)
    rc = fail(c, MSG_EHIP, "Ws upload failed");
  for (int k = 0; k < n && !rc; ++k)
    if (frs[k].N > 0 && hipStreamWaitEvent(c->own, ev[k], 0) != hipSuccess) rc = fail(c, MSG_EHIP, "stream wait failed");
  if (!rc) {
    LAUNCH(c, KID_SERIAL_MULTI, c->own, k_serial_multi, dim3(n), dim3(64), 0, c->d_wss, n, run_limit);
    if (hipGetLastError() != hipSuccess || hipEventRecord(ev[n], c->own) != hipSuccess)
      rc = fail(c, MSG_EHIP, "k_serial_multi launch failed");
  }
  for (int k = 0; k < n && !rc; ++k)
    if (hipStreamWaitEvent(c->msubs[k]->own, ev[n], 0) != hipSuccess) rc = fail(c, MSG_EHIP, "stream wait failed");
  if (rc) {
    (void)hipStreamSynchronize(c->own);
    for (int k = 0; k < n; ++k) (void)hipStreamSynchronize(c->msubs[k]->own);
    cleanup();
    return rc;
  }
  // every flood: the rest of its flood (a no-op loop of one group when k_serial_multi finished it)
  // and its label map + colours, `inflight` host threads
  const int K = std::max(1, std::min({c->inflight, n, MAX_INFLIGHT}));
  std::vector<int> rcs(K, MSG_OK);
  std::vector<msg_stats> st(K);
  std::vector<std::thread> th;
  for (int w = 0; w < K; ++w)
    th.emplace_back([&, w]() {
      if (hipSetDevice(c->dev) != hipSuccess) {
        rcs[w] = MSG_EHIP;
        return;
      }
      msg_stats acc{};
      for (int k = w; k < n; k += K) {
        msg_ctx* x = c->msubs[k];
        const uint8_t* img;
        const int32_t* mk;
        int H, W;
        int32_t* lab;
        uint8_t* dst;
        frame(k, img, mk, H, W, lab, dst);
        int r = flood_loop(x, frs[k]);
        if (!r) r = flood_end(x, frs[k], lab, depth, dst ? d_pal : nullptr, dst, nullptr);
        if (r) {
          rcs[w] = r;
          return;
        }
        add_stats(acc, x->stats);
      }
      st[w] = acc;
    });
  for (auto& t : th) t.join();
  cleanup();
  msg_stats tot{};
  for (int w = 0; w < K; ++w) {
    if (rcs[w]) {
      c->err = "a flood of the batch failed";
      for (int k = w; k < n; k += K)
        if (!c->msubs[k]->err.empty()) c->err = c->msubs[k]->err;
      return rcs[w];
    }
    add_stats(tot, st[w]);
  }
  c->stats = tot;
  return MSG_OK;
}

// Streaming-kernel grid: enough 256-thread blocks for ~4 waves of 4-pixel groups per SIMD.
int stream_grid(long long N) {
  const long long th = (N + 3) / 4;
  return (int)std::max<long long>(1, std::min<long long>((th + 255) / 256, 4096));
}

bool aligned(const void* p, uintptr_t a) { return ((uintptr_t)p & (a - 1)) == 0; }

// from_gray: d_bgr is a gray plane to histogram (no gray output)
int gray_hist(msg_ctx* c, const uint8_t* d_bgr, long long N, uint8_t* d_gray, int32_t* hist,
              hipStream_t st, bool from_gray = false) {
  if (!c->d_hist) {
    HIPCHK(c, hipMalloc((void**)&c->d_hist, 256 * sizeof(unsigned)));
    HIPCHK(c, hipHostMalloc((void**)&c->h_hist, 256 * sizeof(unsigned), hipHostMallocDefault));
  }
  if (N == 0) {
    for (int i = 0; i < 256; ++i) hist[i] = 0;
    return MSG_OK;
  }
  HIPCHK(c, hipMemsetAsync(c->d_hist, 0, 256 * sizeof(unsigned), st));
  // one block per CU (fewer when the frame is small)
  const long long per_block = (long long)GH_BS * GH_UNROLL;
  const int grid = (int)std::max<long long>(1, std::min<long long>(c->cus, ((N >> 2) + per_block - 1) / per_block));
  if (from_gray)
    LAUNCH(c, KID_GRAY_HIST, st, k_gray_hist<true>, dim3(grid), dim3(GH_BS), 0, d_bgr, N, d_gray, c->d_hist);
  else
    LAUNCH(c, KID_GRAY_HIST, st, k_gray_hist<false>, dim3(grid), dim3(GH_BS), 0, d_bgr, N, d_gray, c->d_hist);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(c->h_hist, c->d_hist, 256 * sizeof(unsigned), hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipStreamSynchronize(st));
  if (c->prof) collect_profile(c);
  for (int i = 0; i < 256; ++i) hist[i] = (int32_t)c->h_hist[i];
  return MSG_OK;
}

int nc_markers(msg_ctx* c, const uint8_t* d_gray, long long N, const int32_t* lut, int32_t* d_markers,
               hipStream_t st) {
  if (N == 0) return MSG_OK;
  NcLut L;
  std::memcpy(L.v, lut, sizeof(L.v));
  LAUNCH(c, KID_NC_MARKERS, st, k_nc_markers, dim3(stream_grid(N)), dim3(256), 0, d_gray, N,
         d_markers, L);
  HIPCHK(c, hipGetLastError());
  return MSG_OK;
}

int blur_mask_size(int rows, int cols) {  // PictureService.java:877-899
  const int m = cols <= rows ? cols : rows;
  if (m < 3) return 1;
  if (m <= 100) return 5;
  const double scale = m <= 360 ? 0.025 : m <= 480 ? 0.02 : m <= 720 ? 0.015 : m <= 1080 ? 0.01 : 0.005;
  const int r = (int)(m * scale);  // Double.intValue()
  return r % 2 == 0 ? r + 1 : r;
}

int ensure_shape(msg_ctx* c, long long N, long long nb) {
  if (c->sh_n >= N && c->sh_nb >= nb) return MSG_OK;
  dfree(c->d_sh8);
  dfree(c->d_sh32);
  dfree(c->d_shF);
  dfree(c->d_shP);
  dfree(c->d_scan_tmp);
  c->d_sh8 = nullptr;
  c->d_sh32 = nullptr;
  c->d_shF = c->d_shP = nullptr;
  c->d_scan_tmp = nullptr;
  c->sh_n = c->sh_nb = 0;
  HIPCHK(c, hipMalloc((void**)&c->d_sh8, 6 * N + 64));
  HIPCHK(c, hipMalloc((void**)&c->d_sh32, 2 * N * sizeof(int) + 64));
  HIPCHK(c, hipMalloc((void**)&c->d_shF, nb * sizeof(int) + 64));
  HIPCHK(c, hipMalloc((void**)&c->d_shP, nb * sizeof(int) + 64));
  if (!c->d_shcnt) HIPCHK(c, hipMalloc((void**)&c->d_shcnt, 4 * sizeof(int)));
  size_t tb = 0;
  HIPCHK(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tb, c->d_shF, c->d_shP, (int)nb));
  HIPCHK(c, hipMalloc(&c->d_scan_tmp, tb + 64));
  c->scan_tmp_bytes = tb + 64;
  c->sh_n = N;
  c->sh_nb = nb;
  return MSG_OK;
}

int ensure_color(msg_ctx* c, long long N) {
  if (c->cm_n >= N) return MSG_OK;
  dfree(c->d_cm32);
  dfree(c->d_cmreg);
  c->cm_n = 0;
  HIPCHK(c, hipMalloc((void**)&c->d_cm32, 5 * N * sizeof(int) + 64));
  HIPCHK(c, hipMalloc((void**)&c->d_cmreg, 2 * N * sizeof(int2) + 64));
  if (!c->d_cmcnt) HIPCHK(c, hipMalloc((void**)&c->d_cmcnt, 16 * sizeof(int)));
  c->cm_n = N;
  return MSG_OK;
}

// OpenCV's getThreshVal_Otsu_8u (threshold(..., THRESH_OTSU), PictureService.java:941): the first
// threshold of maximal between-class variance, in double arithmetic, operation for operation.
double otsu_threshold(const int32_t* h, long long n) {
  const double scale = 1.0 / (double)n;
  double mu = 0;
  for (int i = 0; i < 256; ++i) mu += i * (double)h[i];
  mu *= scale;
  double mu1 = 0, q1 = 0, max_sigma = 0, max_val = 0;
  const double eps = 1.1920928955078125e-07;  // FLT_EPSILON
  for (int i = 0; i < 256; ++i) {
    const double p_i = h[i] * scale;
    mu1 *= q1;
    q1 += p_i;
    const double q2 = 1. - q1;
    if (std::min(q1, q2) < eps || std::max(q1, q2) > 1. - eps) continue;
    mu1 = (mu1 + i * p_i) / q1;
    const double mu2 = (mu - q1 * mu1) / q2;
    const double sigma = q1 * q2 * (mu1 - mu2) * (mu1 - mu2);
    if (sigma > max_sigma) {
      max_sigma = sigma;
      max_val = i;
    }
  }
  return max_val;
}

// Union-find labelling of the pixels `mode` selects (k_ccl_*): L = root per pixel, -1 elsewhere.
int ccl(msg_ctx* c, const uint8_t* a, int* L, int H, int W, int mode, hipStream_t st) {
  const long long N = (long long)H * W;
  const int grid = stream_grid(N);
  LAUNCH(c, KID_CCL, st, k_ccl_local, dim3((W + CT - 1) / CT, (H + CT - 1) / CT), dim3(256), 0, a, L, H, W,
         mode);
  LAUNCH(c, KID_CCL, st, k_ccl_boundary, dim3((W + CT - 1) / CT, (H + CT - 1) / CT), dim3(128), 0, a, L, H, W,
         mode);
  LAUNCH(c, KID_CCL, st, k_ccl_compress, dim3(grid), dim3(256), 0, L, N);
  HIPCHK(c, hipGetLastError());
  return MSG_OK;
}

}  // namespace

extern "C" {

int msg_abi_version(void) { return MSG_ABI_VERSION; }

#ifndef MSEG_BUILD_ID
#define MSEG_BUILD_ID "unknown"
#endif
const char* msg_build_id(void) { return MSEG_BUILD_ID; }

int msg_create(msg_ctx** out, int device_ordinal, unsigned flags) {
  if (!out || (flags & ~MSG_CREATE_HIGH_PRIORITY)) return MSG_EINVAL;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return MSG_EHIP;
  if (device_ordinal < 0 || device_ordinal >= ndev) return MSG_EINVAL;
  msg_ctx* c = new (std::nothrow) msg_ctx();
  if (!c) return MSG_ENOMEM;
  c->dev = device_ordinal;
  // MSG_CREATE_HIGH_PRIORITY: the context's stream at the device's highest priority (the batch
  // entry points' sub-contexts: the HIP runtime keeps streams of different priorities on different
  // hardware queues)
  int prio = 0;
  if (hipSetDevice(c->dev) != hipSuccess) {  // the priority range below is the current device's
    msg_destroy(c);
    return MSG_EHIP;
  }
  {
    int lo = 0, hi = 0;
    if ((flags & MSG_CREATE_HIGH_PRIORITY) && hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess) prio = hi;
  }
  if (hipSetDevice(c->dev) != hipSuccess ||
      hipStreamCreateWithPriority(&c->own, hipStreamNonBlocking, prio) != hipSuccess ||
      hipMalloc((void**)&c->d_ctl, sizeof(Ctl)) != hipSuccess ||
      hipHostMalloc((void**)&c->h_mir, 16 * sizeof(int), hipHostMallocMapped | hipHostMallocCoherent) !=
          hipSuccess ||
      hipHostGetDevicePointer((void**)&c->d_mir, c->h_mir, 0) != hipSuccess ||
      hipHostMalloc((void**)&c->h_tail, sizeof(Ctl), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void**)&c->d_tail, c->h_tail, 0) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_in, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_out, hipEventDisableTiming) != hipSuccess) {
    msg_destroy(c);
    return MSG_EHIP;
  }
  for (int k = 0; k < 16; ++k) c->h_mir[k] = 0;  // (word 7: k_tail's releases start at 1)
  {
    int cus = 0, per = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_resolve<false>, RBS, 0) != hipSuccess || cus <= 0 ||
        per <= 0) {
      msg_destroy(c);
      return MSG_EHIP;
    }
    // one full wave of k_resolve blocks (3 x 512 threads per CU at its 80 VGPRs, capped at 4):
    // a performance choice only -- chunks are dealt in dispatch order, so progress does not
    // depend on how many of the blocks are resident (msg_set_resolve_grid overrides it)
    c->res_grid = cus * std::max(1, std::min(per, 4));
    c->cus = cus;
    // k_spec_round: one block per CU (two fit; ranks are dealt in dispatch order, so this is a
    // performance choice only).  Round 4 A/B (profiles/r04sg_ab_spec_grid.log, flood only):
    // 2 -> 1 block per CU took mosaic+noise 1024^2 47.4 -> 35.9 ms, 4096^2 186.6 -> 175.2 ms,
    // uniform noise 4096^2 1444 -> 1424 ms, album.jpg 1313 -> 1300 ms (fewer waves contending for
    // the dealing counter and the L2 at every round's start and end); half a block per CU was
    // better still on the 1024^2 frames and worse at 4096^2
    int sper = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&sper, k_spec_round, SPEC_BS, 0) != hipSuccess || sper <= 0)
      sper = 1;
    c->spec_grid = cus * std::min(sper, 1);
  }
  *out = c;
  return MSG_OK;
}

void msg_destroy(msg_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->dev);
  if (c->own) (void)hipStreamSynchronize(c->own);
  free_flood(c);
  free_spec(c);
  for (msg_ctx* sub : c->subs) msg_destroy(sub);
  c->subs.clear();
  for (msg_ctx* sub : c->msubs) msg_destroy(sub);
  c->msubs.clear();
  for (msg_ctx* sub : c->dsubs) msg_destroy(sub);  // other devices: each switches the thread's device
  c->dsubs.clear();
  (void)hipSetDevice(c->dev);
  dfree(c->d_wss);
  dfree(c->d_mstage);
  free_stage(c);
  dfree(c->d_pal);
  dfree(c->d_ctl);
  dfree(c->d_diag);
  dfree(c->d_hist);
  dfree(c->d_gscr);
  dfree(c->d_gscr2);
  dfree(c->d_btaps);
  dfree(c->d_sh8);
  dfree(c->d_sh32);
  dfree(c->d_shF);
  dfree(c->d_shP);
  dfree(c->d_shcnt);
  dfree(c->d_scan_tmp);
  dfree(c->d_cm32);
  dfree(c->d_cmreg);
  dfree(c->d_cmcnt);
  if (c->h_hist) (void)hipHostFree(c->h_hist);
  if (c->h_mir) (void)hipHostFree(c->h_mir);
  if (c->h_tail) (void)hipHostFree(c->h_tail);
  for (auto& e : c->evpool) (void)hipEventDestroy(e);
  if (c->ev_in) (void)hipEventDestroy(c->ev_in);
  if (c->ev_out) (void)hipEventDestroy(c->ev_out);
  if (c->own) (void)hipStreamDestroy(c->own);
  delete c;
}

const char* msg_last_error(const msg_ctx* c) { return c ? c->err.c_str() : "null context"; }

int msg_get_stats(const msg_ctx* c, msg_stats* out) {
  if (!c || !out) return MSG_EINVAL;
  *out = c->stats;
  return MSG_OK;
}

int msg_set_fast_commit(msg_ctx* c, int enable) {
  if (!c) return MSG_EINVAL;
  c->fast = enable != 0;
  for (msg_ctx* sub : c->subs) sub->fast = c->fast;
  return MSG_OK;
}

int msg_set_speculative(msg_ctx* c, int enable) {
  if (!c) return MSG_EINVAL;
  c->spec = enable != 0;
  c->spec_eager_failed_np = 0;
  if (!c->spec) free_spec(c);  // the engine's workspace comes back on its next first use
  for (msg_ctx* sub : c->subs) {
    sub->spec = c->spec;
    if (!sub->spec) free_spec(sub);
  }
  for (msg_ctx* sub : c->dsubs)
    if (sub) (void)msg_set_speculative(sub, enable);
  return MSG_OK;
}

int msg_set_profiling(msg_ctx* c, int enable) {
  if (!c) return MSG_EINVAL;
  c->prof = enable != 0;
  return MSG_OK;
}

int msg_set_diag(msg_ctx* c, int enable) {
  if (!c) return MSG_EINVAL;
  if (enable && !c->d_diag) {
    HIPCHK(c, hipSetDevice(c->dev));
    HIPCHK(c, hipMalloc((void**)&c->d_diag, 32 * sizeof(unsigned long long)));
  }
  c->diag = enable != 0;
  c->inject = enable == 2;
  c->diag_bank = enable == 3 ? 2 : enable == 4 ? 3 : 0;
  return MSG_OK;
}

int msg_get_kernel_profile(msg_ctx* c, msg_kernel_profile* out, int max_entries, int reset) {
  if (!c || (max_entries > 0 && !out)) return MSG_EINVAL;
  if (!c->recs.empty()) {
    (void)hipSetDevice(c->dev);
    (void)hipDeviceSynchronize();
    collect_profile(c);
  }
  int n = 0;
  for (int k = 0; k < MSG_NKERNELS && n < max_entries; ++k) {
    std::snprintf(out[n].name, sizeof(out[n].name), "%s", kKernelNames[k]);
    out[n].launches = c->prof_n[k];
    out[n].total_ms = c->prof_ms[k];
    ++n;
  }
  if (reset) {
    for (int k = 0; k < MSG_NKERNELS; ++k) {
      c->prof_ms[k] = 0;
      c->prof_n[k] = 0;
    }
  }
  return n;
}

int msg_watershed_dev(msg_ctx* c, const void* d_bgr, const void* d_markers_in, void* d_labels,
                      int rows, int cols, void* stream) {
  if (!c) return MSG_EINVAL;
  int rc = check_size(c, rows, cols, true);
  if (rc) return rc;
  if ((long long)rows * cols > 0 && (!d_bgr || !d_markers_in || !d_labels))
    return fail(c, MSG_EINVAL, "null device pointer");
  HIPCHK(c, hipSetDevice(c->dev));
  StreamScope scope(c, stream);
  if (scope.rc) return scope.rc;
  hipStream_t st = scope.st;
  return run_flood(c, (const uint8_t*)d_bgr, (const int32_t*)d_markers_in, (int32_t*)d_labels,
                   rows, cols, st);
}

int msg_colorize_dev(msg_ctx* c, const void* d_labels, int rows, int cols, int depth,
                     const void* d_palette_bgr, void* d_dst_bgr, void* d_gray, void* stream) {
  if (!c) return MSG_EINVAL;
  int rc = check_size(c, rows, cols, true);
  if (rc) return rc;
  if (depth < 0) return fail(c, MSG_EINVAL, "negative depth");
  if ((long long)rows * cols > 0 && (!d_labels || !d_dst_bgr))
    return fail(c, MSG_EINVAL, "null device pointer");
  HIPCHK(c, hipSetDevice(c->dev));
  StreamScope scope(c, stream);
  if (scope.rc) return scope.rc;
  hipStream_t st = scope.st;
  return launch_colorize(c, (const int32_t*)d_labels, (long long)rows * cols, depth,
                         (const uint8_t*)d_palette_bgr, (uint8_t*)d_dst_bgr, (uint8_t*)d_gray, st);
}

int msg_watershed_colorize_dev(msg_ctx* c, const void* d_bgr, const void* d_markers_in,
                               void* d_labels, int rows, int cols, int depth,
                               const void* d_palette_bgr, void* d_dst_bgr, void* d_gray,
                               void* stream) {
  if (!c) return MSG_EINVAL;
  int rc = check_size(c, rows, cols, true);
  if (rc) return rc;
  if (depth < 0) return fail(c, MSG_EINVAL, "negative depth");
  if ((long long)rows * cols > 0 && (!d_bgr || !d_markers_in || !d_labels || !d_dst_bgr))
    return fail(c, MSG_EINVAL, "null device pointer");
  HIPCHK(c, hipSetDevice(c->dev));
  StreamScope scope(c, stream);
  if (scope.rc) return scope.rc;
  hipStream_t st = scope.st;
  return run_flood(c, (const uint8_t*)d_bgr, (const int32_t*)d_markers_in, (int32_t*)d_labels, rows,
                   cols, st, depth, (const uint8_t*)d_palette_bgr, (uint8_t*)d_dst_bgr,
                   (uint8_t*)d_gray);
}

int msg_edge_weights_dev(msg_ctx* c, const void* d_bgr, void* d_wright, void* d_wdown, int rows,
                         int cols, void* stream) {
  if (!c) return MSG_EINVAL;
  int rc = check_size(c, rows, cols, true);
  if (rc) return rc;
  const long long N = (long long)rows * cols;
  if (N == 0) return MSG_OK;
  if (!d_bgr || !d_wright || !d_wdown) return fail(c, MSG_EINVAL, "null device pointer");
  HIPCHK(c, hipSetDevice(c->dev));
  StreamScope scope(c, stream);
  if (scope.rc) return scope.rc;
  hipStream_t st = scope.st;
  const bool vec = cols % 16 == 0 && (((uintptr_t)d_bgr | (uintptr_t)d_wright | (uintptr_t)d_wdown) & 15) == 0;
  if (vec) {
    // rows per thread measured per size (scripts/exp/stream_variants.hip): 1 up to 4096^2
    // (14.3 us vs 15.7 for 2), 2 above (8192^2: 61.4 us vs 63.0 for 4 and 64.9 for 1)
    if (N <= (1ll << 24)) {
      const long long th = (long long)rows * (cols / 16);
      LAUNCH(c, KID_EDGE, st, k_edge_weights16<1>, dim3((unsigned)((th + 255) / 256)), dim3(256), 0,
             (const uint8_t*)d_bgr, (uint8_t*)d_wright, (uint8_t*)d_wdown, rows, cols);
    } else {
      const long long th = (long long)((rows + 1) / 2) * (cols / 16);
      LAUNCH(c, KID_EDGE, st, k_edge_weights16<2>, dim3((unsigned)((th + 255) / 256)), dim3(256), 0,
             (const uint8_t*)d_bgr, (uint8_t*)d_wright, (uint8_t*)d_wdown, rows, cols);
    }
  } else {
    const long long th = (N + 3) / 4;
    LAUNCH(c, KID_EDGE, st, k_edge_weights, dim3((unsigned)((th + 255) / 256)), dim3(256), 0,
           (const uint8_t*)d_bgr, (uint8_t*)d_wright, (uint8_t*)d_wdown, rows, cols);
  }
  HIPCHK(c, hipGetLastError());
  return MSG_OK;
}

static int host_args(msg_ctx* c, const void* bgr, size_t bgr_stride, const void* markers,
                     size_t marker_stride, int rows, int cols, bool flood = false) {
  if (!c) return MSG_EINVAL;
  int rc = check_size(c, rows, cols, flood);
  if (rc) return rc;
  if ((long long)rows * cols == 0) return MSG_OK;
  if (!bgr || !markers) return fail(c, MSG_EINVAL, "null host pointer");
  if (bgr_stride < (size_t)cols * 3) return fail(c, MSG_EINVAL, "bgr stride too small");
  if (marker_stride < (size_t)cols * 4 || (marker_stride & 3))
    return fail(c, MSG_EINVAL, "marker stride invalid");
  return MSG_OK;
}

int msg_watershed_colorize(msg_ctx* c, const uint8_t* bgr, size_t bgr_stride, int32_t* markers,
                           size_t marker_stride, int rows, int cols, int depth,
                           const uint8_t* palette_bgr, uint8_t* dst_bgr, size_t dst_stride,
                           uint8_t* gray, size_t gray_stride) {
  int rc = host_args(c, bgr, bgr_stride, markers, marker_stride, rows, cols, true);
  if (rc) return rc;
  const long long N = (long long)rows * cols;
  if (N == 0) return MSG_OK;
  const bool want_color = dst_bgr != nullptr;
  if (want_color) {
    if (depth < 0) return fail(c, MSG_EINVAL, "negative depth");
    if (dst_stride < (size_t)cols * 3) return fail(c, MSG_EINVAL, "dst stride too small");
    if (gray && gray_stride < (size_t)cols) return fail(c, MSG_EINVAL, "gray stride too small");
  }
  HIPCHK(c, hipSetDevice(c->dev));
  rc = ensure_stage(c, N);
  if (rc) return rc;
  hipStream_t st = c->own;
  HIPCHK(c, hipMemcpy2DAsync(c->d_img, (size_t)cols * 3, bgr, bgr_stride, (size_t)cols * 3, rows,
                             hipMemcpyHostToDevice, st));
  HIPCHK(c, hipMemcpy2DAsync(c->d_mk, (size_t)cols * 4, markers, marker_stride, (size_t)cols * 4,
                             rows, hipMemcpyHostToDevice, st));
  const uint8_t* dp = nullptr;
  if (want_color && palette_bgr && depth > 0) {
    rc = upload_palette(c, palette_bgr, depth, st);
    if (rc) return rc;
    dp = c->d_pal;  // (depth 0: every pixel is background either way)
  }
  rc = run_flood(c, c->d_img, c->d_mk, c->d_mk, rows, cols, st, depth, dp,
                 want_color ? c->d_dst : nullptr, (want_color && gray) ? c->d_gray : nullptr);
  if (rc) return rc;
  HIPCHK(c, hipMemcpy2DAsync(markers, marker_stride, c->d_mk, (size_t)cols * 4, (size_t)cols * 4,
                             rows, hipMemcpyDeviceToHost, st));
  // consistency check, no retry: cv::watershed leaves the whole first row at WSHED, so anything
  // else means the flood or the read-back was misordered -- a hard error, never re-issued
  HIPCHK(c, hipStreamSynchronize(st));
  for (int j = 0; j < cols; ++j)
    if (markers[j] != WSHED) return fail(c, MSG_ESTATE, "label read-back failed the frame-border check");
  if (want_color) {
    HIPCHK(c, hipMemcpy2DAsync(dst_bgr, dst_stride, c->d_dst, (size_t)cols * 3, (size_t)cols * 3,
                               rows, hipMemcpyDeviceToHost, st));
    if (gray)
      HIPCHK(c, hipMemcpy2DAsync(gray, gray_stride, c->d_gray, (size_t)cols, (size_t)cols, rows,
                                 hipMemcpyDeviceToHost, st));
  }
  HIPCHK(c, hipStreamSynchronize(st));
  return MSG_OK;
}

int msg_watershed(msg_ctx* c, const uint8_t* bgr, size_t bgr_stride, int32_t* markers,
                  size_t marker_stride, int rows, int cols) {
  return msg_watershed_colorize(c, bgr, bgr_stride, markers, marker_stride, rows, cols, 0, nullptr,
                                nullptr, 0, nullptr, 0);
}

int msg_colorize(msg_ctx* c, const int32_t* labels, size_t label_stride, int rows, int cols,
                 int depth, const uint8_t* palette_bgr, uint8_t* dst_bgr, size_t dst_stride) {
  if (!c) return MSG_EINVAL;
  int rc = check_size(c, rows, cols, true);
  if (rc) return rc;
  const long long N = (long long)rows * cols;
  if (N == 0) return MSG_OK;
  if (depth < 0) return fail(c, MSG_EINVAL, "negative depth");
  if (!labels || !dst_bgr) return fail(c, MSG_EINVAL, "null host pointer");
  if (label_stride < (size_t)cols * 4 || (label_stride & 3) || dst_stride < (size_t)cols * 3)
    return fail(c, MSG_EINVAL, "stride invalid");
  HIPCHK(c, hipSetDevice(c->dev));
  rc = ensure_stage(c, N);
  if (rc) return rc;
  hipStream_t st = c->own;
  HIPCHK(c, hipMemcpy2DAsync(c->d_mk, (size_t)cols * 4, labels, label_stride, (size_t)cols * 4,
                             rows, hipMemcpyHostToDevice, st));
  const uint8_t* dp = nullptr;
  if (palette_bgr && depth > 0) {
    rc = upload_palette(c, palette_bgr, depth, st);
    if (rc) return rc;
    dp = c->d_pal;
  }
  rc = launch_colorize(c, c->d_mk, N, depth, dp, c->d_dst, nullptr, st);
  if (rc) return rc;
  HIPCHK(c, hipMemcpy2DAsync(dst_bgr, dst_stride, c->d_dst, (size_t)cols * 3, (size_t)cols * 3,
                             rows, hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipStreamSynchronize(st));
  return MSG_OK;
}

}  // extern "C"

namespace {

int host_batch(msg_ctx* c, int n, const uint8_t* const* bgr, const size_t* bgr_stride, int32_t* const* markers,
               const size_t* marker_stride, const int* rows, const int* cols, int depth, const uint8_t* palette,
               uint8_t* const* dst, const size_t* dst_stride);

// msg_set_batch_floods mode 3 (automatic): which path a batch's frames take.  The regime of a flood
// is only known by running it, so the first call for a frame size floods frame 0 alone with the full
// engine on this context (a probe: its result is final, it is part of the call) and prices both paths
// for the rest of the batch:
//   full engine: the probe's wall time per flood, `inflight` floods overlapped at a time;
//   many floods: every flood at once in one k_serial_multi launch, a serial pop per ~1 us of one
//                wave, so about the probe's pop count in microseconds.
// Interrupt-dense floods that the speculative engine serves well (noise) and plateaus (mosaic) price
// far below their pop count and stay on the full engine; chains of dependent pops (notConnectedMarkers'
// seeds, photographs) price at ~1 us per pop either way and go to the many-floods kernel once the batch
// has more floods than in flight.  The choice is kept for that frame size (later calls skip the probe);
// results are identical on either path.
constexpr double AUTO_SERIAL_POP_US = 1.0;
int auto_choice(const msg_ctx* c, int nrest, const msg_stats& probe, double probe_s) {
  if (nrest <= 0) return 0;
  const int k = std::max(1, std::min({c->inflight, nrest, MAX_INFLIGHT}));
  const double full = probe_s * (double)((nrest + k - 1) / k);
  const double many = 1e-6 * AUTO_SERIAL_POP_US * (double)probe.pops;
  return many < full ? 1 : 0;
}

// msg_set_batch_devices: frames [n*j/D, n*(j+1)/D) on the sub-context of device-list entry j, one
// host thread per entry, each a host_batch of its own (this context's batch settings copied over).
// No data crosses devices: every block's buffers are the caller's host memory.
int spread_batch(msg_ctx* c, int n, const uint8_t* const* bgr, const size_t* bgr_stride, int32_t* const* markers,
                 const size_t* marker_stride, const int* rows, const int* cols, int depth, const uint8_t* palette,
                 uint8_t* const* dst, const size_t* dst_stride) {
  const int D = (int)c->bdevs.size();
  c->dsubs.resize(D, nullptr);
  for (int j = 0; j < D; ++j) {
    msg_ctx*& x = c->dsubs[j];
    if (!x) {
      const int rc = msg_create(&x, c->bdevs[j], 0);
      if (rc) {
        x = nullptr;
        return fail(c, rc, "sub-context on device %d (entry %d) failed (%d)", c->bdevs[j], j, rc);
      }
    }
    x->inflight = c->inflight;
    x->fast = c->fast;
    if (c->res_grid_set) {
      x->res_grid = c->res_grid;
      x->res_grid_set = true;
    }
    if (x->spec != c->spec) {
      const int rc = msg_set_speculative(x, c->spec ? 1 : 0);
      if (rc) return fail(c, rc, "%s", x->err.c_str());
    }
    if (x->many != c->many) {
      const int rc = msg_set_batch_floods(x, c->many);
      if (rc) return fail(c, rc, "%s", x->err.c_str());
    }
    if (x->diag != c->diag || x->inject != c->inject) {
      const int rc = msg_set_diag(x, c->inject ? 2 : c->diag ? 1 : 0);
      if (rc) return fail(c, rc, "%s", x->err.c_str());
    }
  }
  std::vector<int> rcs(D, MSG_OK);
  std::vector<std::thread> th;
  for (int j = 0; j < D; ++j)
    th.emplace_back([&, j]() {
      msg_ctx* x = c->dsubs[j];
      const int lo = (int)((long long)n * j / D), hi = (int)((long long)n * (j + 1) / D);
      x->stats = msg_stats{};
      if (hi == lo) return;
      if (hipSetDevice(x->dev) != hipSuccess) {
        rcs[j] = fail(x, MSG_EHIP, "hipSetDevice(%d) failed", x->dev);
        return;
      }
      rcs[j] = host_batch(x, hi - lo, bgr + lo, bgr_stride + lo, markers + lo, marker_stride + lo, rows + lo,
                          cols + lo, depth, palette, dst ? dst + lo : nullptr, dst ? dst_stride + lo : nullptr);
    });
  for (auto& t : th) t.join();
  msg_stats tot{};
  for (int j = 0; j < D; ++j) {
    if (rcs[j]) {
      c->err = "device " + std::to_string(c->dsubs[j]->dev) + " (entry " + std::to_string(j) +
               "): " + c->dsubs[j]->err;
      return rcs[j];
    }
    if ((long long)n * (j + 1) / D > (long long)n * j / D) add_stats(tot, c->dsubs[j]->stats);
  }
  c->stats = tot;
  return MSG_OK;
}

int host_batch_mode(msg_ctx* c, int mode, int n, const uint8_t* const* bgr, const size_t* bgr_stride,
                    int32_t* const* markers, const size_t* marker_stride, const int* rows, const int* cols, int depth,
                    const uint8_t* palette, uint8_t* const* dst, const size_t* dst_stride);

// The host-buffer batch (msg_watershed_batch, msg_watershed_colorize_batch): labels in place, and
// the colourised frames when dst is given.  Many-floods mode: every frame staged (image, markers,
// colour output, each 16-B aligned), flooded together, read back; otherwise run_batch.
int host_batch(msg_ctx* c, int n, const uint8_t* const* bgr, const size_t* bgr_stride, int32_t* const* markers,
               const size_t* marker_stride, const int* rows, const int* cols, int depth, const uint8_t* palette,
               uint8_t* const* dst, const size_t* dst_stride) {
  if (!c || n < 0) return MSG_EINVAL;
  if (n > 0 && (!bgr || !bgr_stride || !markers || !marker_stride || !rows || !cols))
    return fail(c, MSG_EINVAL, "null batch array");
  if (n > 0 && dst && !dst_stride) return fail(c, MSG_EINVAL, "null batch array");
  if (dst && depth < 0) return fail(c, MSG_EINVAL, "negative depth");
  for (int k = 0; k < n; ++k) {
    const int rc = host_args(c, bgr[k], bgr_stride[k], markers[k], marker_stride[k], rows[k], cols[k], true);
    if (rc) return rc;
    if (dst && (long long)rows[k] * cols[k] > 0 && (!dst[k] || dst_stride[k] < (size_t)cols[k] * 3))
      return fail(c, MSG_EINVAL, "dst of frame %d: null or stride too small", k);
  }
  if (!c->bdevs.empty() && n > 0)
    return spread_batch(c, n, bgr, bgr_stride, markers, marker_stride, rows, cols, depth, palette, dst, dst_stride);
  int mode = c->many;
  msg_stats pst{};
  bool probed = false;
  if (mode == 3) {  // automatic: the frame size's known choice, or a probe on frame 0 (auto_choice)
    mode = 0;
    const long long key = n > 0 ? ((long long)rows[0] << 32 | (unsigned)cols[0]) : -1;
    if (n >= 2 && key == c->auto_key) {
      mode = c->auto_mode;
    } else if (n >= 2) {
      const auto t0 = std::chrono::steady_clock::now();
      const int rc = dst ? msg_watershed_colorize(c, bgr[0], bgr_stride[0], markers[0], marker_stride[0], rows[0],
                                                  cols[0], depth, palette, dst[0], dst_stride[0], nullptr, 0)
                         : msg_watershed(c, bgr[0], bgr_stride[0], markers[0], marker_stride[0], rows[0], cols[0]);
      if (rc) return rc;
      const double ps = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      pst = c->stats;
      probed = true;
      mode = auto_choice(c, n - 1, pst, ps);
      c->auto_key = key;
      c->auto_mode = mode;
      ++bgr, ++bgr_stride, ++markers, ++marker_stride, ++rows, ++cols;  // the rest of the batch
      if (dst) ++dst, ++dst_stride;
      --n;
    }
  }
  int rc = host_batch_mode(c, mode, n, bgr, bgr_stride, markers, marker_stride, rows, cols, depth, palette,
                           dst, dst_stride);
  if (rc == MSG_ENOMEM && c->many == 3 && mode != 0) {  // automatic choice without the memory: the full engine
    release_many(c);
    (void)hipGetLastError();
    c->auto_mode = mode = 0;
    rc = host_batch_mode(c, 0, n, bgr, bgr_stride, markers, marker_stride, rows, cols, depth, palette, dst,
                         dst_stride);
  }
  if (probed) {
    add_stats(c->stats, pst);
    c->stats.batch_probe = 1;
  }
  c->stats.batch_mode = mode;
  return rc;
}

// host_batch with the mode settled: 0 = run_batch (the full engine, `inflight` floods at a time),
// 1 / 2 = the many-floods kernel.
int host_batch_mode(msg_ctx* c, int mode, int n, const uint8_t* const* bgr, const size_t* bgr_stride,
                    int32_t* const* markers, const size_t* marker_stride, const int* rows, const int* cols, int depth,
                    const uint8_t* palette, uint8_t* const* dst, const size_t* dst_stride) {
  if (!(mode && n > 0))
    return run_batch(c, n, [&](int k, msg_ctx* x) {
      return dst ? msg_watershed_colorize(x, bgr[k], bgr_stride[k], markers[k], marker_stride[k], rows[k], cols[k],
                                          depth, palette, dst[k], dst_stride[k], nullptr, 0)
                 : msg_watershed(x, bgr[k], bgr_stride[k], markers[k], marker_stride[k], rows[k], cols[k]);
    });
  // every frame staged (image, then its markers, then its colour output, each 16-B aligned),
  // flooded in place together
  auto al = [](long long b) { return (b + 15) & ~15ll; };
  std::vector<long long> off(n + 1, 0);
  for (int k = 0; k < n; ++k) {
    const long long N = (long long)rows[k] * cols[k];
    off[k + 1] = off[k] + al(3 * N) + al(4 * N) + (dst ? al(3 * N) : 0);
  }
  HIPCHK(c, hipSetDevice(c->dev));
  if (off[n] > c->mstage_cap) {
    dfree(c->d_mstage);
    c->mstage_cap = 0;
    HIPCHK(c, hipMalloc((void**)&c->d_mstage, off[n] + 16));
    c->mstage_cap = off[n];
  }
  auto img_of = [&](int k) { return c->d_mstage + off[k]; };
  auto mk_of = [&](int k) { return (int32_t*)(c->d_mstage + off[k] + al(3ll * rows[k] * cols[k])); };
  auto dst_of = [&](int k) {
    const long long N = (long long)rows[k] * cols[k];
    return c->d_mstage + off[k] + al(3 * N) + al(4 * N);
  };
  hipStream_t st = c->own;
  const uint8_t* dp = nullptr;
  if (dst && palette && depth > 0) {
    const int rc = upload_palette(c, palette, depth, st);
    if (rc) return rc;
    dp = c->d_pal;
  }
  for (int k = 0; k < n; ++k) {
    if ((long long)rows[k] * cols[k] == 0) continue;
    HIPCHK(c, hipMemcpy2DAsync(img_of(k), (size_t)cols[k] * 3, bgr[k], bgr_stride[k], (size_t)cols[k] * 3,
                               rows[k], hipMemcpyHostToDevice, st));
    HIPCHK(c, hipMemcpy2DAsync(mk_of(k), (size_t)cols[k] * 4, markers[k], marker_stride[k],
                               (size_t)cols[k] * 4, rows[k], hipMemcpyHostToDevice, st));
  }
  HIPCHK(c, hipStreamSynchronize(st));  // the floods run on the sub-contexts' streams
  int rc = batch_many(c, n, mode, depth, dp,
                      [&](int k, const uint8_t*& img, const int32_t*& mk, int& H, int& W, int32_t*& lab, uint8_t*& d) {
                        img = img_of(k);
                        mk = mk_of(k);
                        H = rows[k];
                        W = cols[k];
                        lab = mk_of(k);
                        d = dst ? dst_of(k) : nullptr;
                      });
  if (rc) return rc;
  for (int k = 0; k < n; ++k) {
    if ((long long)rows[k] * cols[k] == 0) continue;
    HIPCHK(c, hipMemcpy2DAsync(markers[k], marker_stride[k], mk_of(k), (size_t)cols[k] * 4, (size_t)cols[k] * 4,
                               rows[k], hipMemcpyDeviceToHost, st));
    if (dst)
      HIPCHK(c, hipMemcpy2DAsync(dst[k], dst_stride[k], dst_of(k), (size_t)cols[k] * 3, (size_t)cols[k] * 3,
                                 rows[k], hipMemcpyDeviceToHost, st));
  }
  HIPCHK(c, hipStreamSynchronize(st));
  for (int k = 0; k < n; ++k)
    for (int j = 0; j < cols[k] && rows[k] > 0; ++j)
      if (markers[k][j] != WSHED) return fail(c, MSG_ESTATE, "label read-back of frame %d failed the frame-border check", k);
  return MSG_OK;
}

}  // namespace

extern "C" {

int msg_watershed_batch(msg_ctx* c, int n, const uint8_t* const* bgr, const size_t* bgr_stride,
                        int32_t* const* markers, const size_t* marker_stride, const int* rows,
                        const int* cols) {
  return host_batch(c, n, bgr, bgr_stride, markers, marker_stride, rows, cols, 0, nullptr, nullptr, nullptr);
}

int msg_watershed_colorize_batch(msg_ctx* c, int n, const uint8_t* const* bgr, const size_t* bgr_stride,
                                 int32_t* const* markers, const size_t* marker_stride, const int* rows,
                                 const int* cols, int depth, const uint8_t* palette_bgr, uint8_t* const* dst_bgr,
                                 const size_t* dst_stride) {
  if (c && n > 0 && !dst_bgr) return fail(c, MSG_EINVAL, "null batch array");
  return host_batch(c, n, bgr, bgr_stride, markers, marker_stride, rows, cols, depth, palette_bgr,
                    n > 0 ? dst_bgr : nullptr, dst_stride);
}

int msg_set_resolve_grid(msg_ctx* c, int blocks) {
  if (!c || blocks < 0) return MSG_EINVAL;
  c->res_grid_set = blocks > 0;
  if (blocks == 0) {
    int per = 0;
    HIPCHK(c, hipSetDevice(c->dev));
    HIPCHK(c, hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_resolve<false>, RBS, 0));
    blocks = c->cus * std::max(1, std::min(per, 4));
  }
  c->res_grid = blocks;
  for (msg_ctx* sub : c->subs) sub->res_grid = blocks;
  return MSG_OK;
}

int msg_set_batch_inflight(msg_ctx* c, int k) {
  if (!c || k < 1) return MSG_EINVAL;
  c->inflight = std::min(k, MAX_INFLIGHT);
  return MSG_OK;
}

int msg_watershed_colorize_batch_dev(msg_ctx* c, int n, const void* const* d_bgr,
                                     const void* const* d_markers_in, void* const* d_labels,
                                     const int* rows, const int* cols, int depth,
                                     const void* d_palette_bgr, void* const* d_dst_bgr, void* stream) {
  if (!c || n < 0) return MSG_EINVAL;
  if (n > 0 && (!d_bgr || !d_markers_in || !d_labels || !rows || !cols || !d_dst_bgr))
    return fail(c, MSG_EINVAL, "null batch array");
  HIPCHK(c, hipSetDevice(c->dev));
  // the inputs may still be in flight on the caller's stream: the floods run on other streams
  HIPCHK(c, stream ? hipStreamSynchronize((hipStream_t)stream) : hipDeviceSynchronize());
  for (int k = 0; k < n; ++k) {
    if (rows[k] < 0 || cols[k] < 0) return fail(c, MSG_EINVAL, "negative size of frame %d", k);
    if ((long long)rows[k] * cols[k] > 0 && (!d_bgr[k] || !d_markers_in[k] || !d_labels[k]))
      return fail(c, MSG_EINVAL, "null device pointer of frame %d", k);
  }
  int mode = c->many, first = 0;
  msg_stats pst{};
  if (mode == 3) {  // automatic (auto_choice): the frame size's known choice, or a probe on frame 0
    mode = 0;
    const long long key = n > 0 ? ((long long)rows[0] << 32 | (unsigned)cols[0]) : -1;
    if (n >= 2 && key == c->auto_key) {
      mode = c->auto_mode;
    } else if (n >= 2) {
      const auto t0 = std::chrono::steady_clock::now();
      int rc = msg_watershed_colorize_dev(c, d_bgr[0], d_markers_in[0], d_labels[0], rows[0], cols[0], depth,
                                          d_palette_bgr, d_dst_bgr[0], nullptr, nullptr);
      if (!rc && hipStreamSynchronize(c->own) != hipSuccess) rc = fail(c, MSG_EHIP, "probe flood stream failed");
      if (rc) return rc;
      const double ps = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      pst = c->stats;
      first = 1;
      mode = auto_choice(c, n - 1, pst, ps);
      c->auto_key = key;
      c->auto_mode = mode;
    }
  }
  auto run_mode = [&](int m) {
    const int nr = n - first;
    if (m)
      return batch_many(c, nr, m, depth, (const uint8_t*)d_palette_bgr,
                        [&](int k, const uint8_t*& img, const int32_t*& mk, int& H, int& W, int32_t*& lab, uint8_t*& dst) {
                          k += first;
                          img = (const uint8_t*)d_bgr[k];
                          mk = (const int32_t*)d_markers_in[k];
                          H = rows[k];
                          W = cols[k];
                          lab = (int32_t*)d_labels[k];
                          dst = (uint8_t*)d_dst_bgr[k];
                        });
    return run_batch(c, nr, [&](int k, msg_ctx* x) {
      k += first;
      return msg_watershed_colorize_dev(x, d_bgr[k], d_markers_in[k], d_labels[k], rows[k], cols[k],
                                        depth, d_palette_bgr, d_dst_bgr[k], nullptr, nullptr);
    });
  };
  int rc = run_mode(mode);
  if (rc == MSG_ENOMEM && c->many == 3 && mode != 0) {  // automatic choice without the memory: the full engine
    release_many(c);
    (void)hipGetLastError();
    c->auto_mode = mode = 0;
    rc = run_mode(0);
  }
  if (first) {
    add_stats(c->stats, pst);
    c->stats.batch_probe = 1;
  }
  c->stats.batch_mode = mode;
  return rc;
}

int msg_set_batch_devices(msg_ctx* c, int ndev, const int* devices) {
  if (!c) return MSG_EINVAL;
  if (ndev < 0 || ndev > 64 || (ndev > 0 && !devices))
    return fail(c, MSG_EINVAL, "device list: %d entries%s (0..64)", ndev, ndev > 0 && !devices ? ", null" : "");
  int count = 0;
  if (ndev > 0 && (hipGetDeviceCount(&count) != hipSuccess || count <= 0))
    return fail(c, MSG_EHIP, "hipGetDeviceCount failed");
  for (int j = 0; j < ndev; ++j)
    if (devices[j] < 0 || devices[j] >= count)
      return fail(c, MSG_EINVAL, "device list entry %d: ordinal %d outside [0, %d)", j, devices[j], count);
  // sub-contexts whose entry changed device (or was dropped) go; the others keep their workspaces
  for (size_t j = 0; j < c->dsubs.size(); ++j)
    if (c->dsubs[j] && ((int)j >= ndev || c->dsubs[j]->dev != devices[j])) {
      msg_destroy(c->dsubs[j]);
      c->dsubs[j] = nullptr;
    }
  c->dsubs.resize(ndev, nullptr);
  c->bdevs.assign(devices, devices + ndev);
  (void)hipSetDevice(c->dev);  // msg_destroy of a sub-context switched the thread's device
  return MSG_OK;
}

int msg_set_batch_floods(msg_ctx* c, int mode) {
  if (!c || mode < 0 || mode > 3) return MSG_EINVAL;
  for (msg_ctx* sub : c->dsubs)
    if (sub) {
      const int rc = msg_set_batch_floods(sub, mode);
      if (rc) return fail(c, rc, "%s", sub->err.c_str());
    }
  (void)hipSetDevice(c->dev);
  c->many = mode;
  c->auto_key = -1;  // mode 3 probes again
  c->auto_mode = -1;
  if (mode == 0) {  // the mode's per-frame workspaces (~44 B/px each) are released with it
    if (hipSetDevice(c->dev) != hipSuccess) return fail(c, MSG_EHIP, "hipSetDevice failed");
    release_many(c);
  }
  return MSG_OK;
}

int msg_gray_hist_dev(msg_ctx* c, const void* d_bgr, int rows, int cols, void* d_gray,
                      int32_t* hist256, void* stream) {
  if (!c) return MSG_EINVAL;
  int rc = check_size(c, rows, cols);
  if (rc) return rc;
  if (!hist256) return fail(c, MSG_EINVAL, "null histogram pointer");
  const long long N = (long long)rows * cols;
  if (N > 0 && (!d_bgr || !d_gray)) return fail(c, MSG_EINVAL, "null device pointer");
  if (!aligned(d_bgr, 4) || !aligned(d_gray, 4))
    return fail(c, MSG_EINVAL, "d_bgr and d_gray must be 4-byte aligned");
  HIPCHK(c, hipSetDevice(c->dev));
  StreamScope scope(c, stream);
  if (scope.rc) return scope.rc;
  hipStream_t st = scope.st;
  return gray_hist(c, (const uint8_t*)d_bgr, N, (uint8_t*)d_gray, hist256, st);
}

int msg_nc_markers_dev(msg_ctx* c, const void* d_gray, int rows, int cols, const int32_t* lut256,
                       void* d_markers, void* stream) {
  if (!c) return MSG_EINVAL;
  int rc = check_size(c, rows, cols);
  if (rc) return rc;
  if (!lut256) return fail(c, MSG_EINVAL, "null marker table");
  const long long N = (long long)rows * cols;
  if (N > 0 && (!d_gray || !d_markers)) return fail(c, MSG_EINVAL, "null device pointer");
  if (!aligned(d_gray, 4) || !aligned(d_markers, 16))
    return fail(c, MSG_EINVAL, "d_gray must be 4-byte and d_markers 16-byte aligned");
  HIPCHK(c, hipSetDevice(c->dev));
  StreamScope scope(c, stream);
  if (scope.rc) return scope.rc;
  hipStream_t st = scope.st;
  return nc_markers(c, (const uint8_t*)d_gray, N, lut256, (int32_t*)d_markers, st);
}

// The BILATERIAL branch's gray -> bilateral pass into g (N > 0: gray into the scratch plane, then
// k_bilateral).  The set-up restates bilateralFilter_8u's (OpenCV 3.4.2 imgproc): sigmas
// 2d <= 0 become 1, radius = d / 2 (d <= 0: cvRound(1.5 sigma_space)), at least 1, colour
// weights (float)exp(i^2 c), taps (dy, dx, (float)exp(r^2 s)) for r = sqrt(dy^2 + dx^2) <= radius
// in row-major order.  The tap table's host copy stays in the context: the caller's histogram
// read-back synchronises the stream before the next call can overwrite it.
static int nc_bilateral(msg_ctx* c, const uint8_t* d_bgr, int rows, int cols, int d, uint8_t* g,
                 hipStream_t st) {
  const long long N = (long long)rows * cols;
  double sc = 2.0 * d, ss = 2.0 * d;
  if (sc <= 0) sc = 1;
  if (ss <= 0) ss = 1;
  const double gcc = -0.5 / (sc * sc), gsc = -0.5 / (ss * ss);
  int radius = d <= 0 ? (int)std::nearbyint(ss * 1.5) : d / 2;
  radius = std::max(radius, 1);
  BilColor cw;
  for (int i = 0; i < 256; ++i) cw.v[i] = (float)std::exp(i * i * gcc);
  c->h_btaps.clear();
  for (int i = -radius; i <= radius; ++i)
    for (int j = -radius; j <= radius; ++j) {
      const double r = std::sqrt((double)i * i + (double)j * j);
      if (r > radius) continue;
      c->h_btaps.push_back(BilTap{(float)std::exp(r * r * gsc), i, j});
    }
  const long long maxk = (long long)c->h_btaps.size();
  if (N == 0) return MSG_OK;
  if (c->btaps_n < maxk) {
    dfree(c->d_btaps);
    c->btaps_n = 0;
    HIPCHK(c, hipMalloc((void**)&c->d_btaps, maxk * sizeof(BilTap)));
    c->btaps_n = maxk;
  }
  if (c->gscr2_n < N) {
    dfree(c->d_gscr2);
    c->gscr2_n = 0;
    HIPCHK(c, hipMalloc((void**)&c->d_gscr2, N + 16));
    c->gscr2_n = N;
  }
  HIPCHK(c, hipMemcpyAsync(c->d_btaps, c->h_btaps.data(), maxk * sizeof(BilTap), hipMemcpyHostToDevice, st));
  const int grid = (int)std::max<long long>(1, std::min<long long>(8192, (N + 255) / 256));
  LAUNCH(c, KID_GRAY, st, k_gray, dim3(grid), dim3(256), 0, d_bgr, N, c->d_gscr2);
  LAUNCH(c, KID_BILATERAL, st, k_bilateral, dim3((cols + 63) / 64, (rows + BIL_ROWS - 1) / BIL_ROWS),
         dim3(64 * BIL_ROWS), 0, c->d_gscr2, g, rows, cols, c->d_btaps, (int)maxk, radius, cw);
  HIPCHK(c, hipGetLastError());
  return MSG_OK;
}

int msg_nc_marker_stage_dev(msg_ctx* c, const void* d_bgr, int rows, int cols, int depth,
                            unsigned options, void* d_gray, void* d_markers,
                            msg_bright_level* levels, int max_levels, int* n_levels,
                            void* stream) {
  if (!c) return MSG_EINVAL;
  int rc = check_size(c, rows, cols);
  if (rc) return rc;
  if (!n_levels || (max_levels > 0 && !levels)) return fail(c, MSG_EINVAL, "null level array");
  *n_levels = 0;
  if (depth <= 0) return fail(c, MSG_EINVAL, "depth must be positive (256 / depth)");
  const long long N = (long long)rows * cols;
  if (N > 0 && (!d_bgr || !d_markers)) return fail(c, MSG_EINVAL, "null device pointer");
  if (!aligned(d_bgr, 4) || !aligned(d_gray, 4) || !aligned(d_markers, 16))
    return fail(c, MSG_EINVAL, "d_bgr/d_gray must be 4-byte and d_markers 16-byte aligned");
  HIPCHK(c, hipSetDevice(c->dev));
  StreamScope scope(c, stream);
  if (scope.rc) return scope.rc;
  hipStream_t st = scope.st;
  uint8_t* g = (uint8_t*)d_gray;
  if (!g && N > 0) {
    if (c->gscr_n < N) {
      dfree(c->d_gscr);
      c->gscr_n = 0;
      HIPCHK(c, hipMalloc((void**)&c->d_gscr, N + 16));
      c->gscr_n = N;
    }
    g = c->d_gscr;
  }
  int32_t hist[256];
  if (options & MSG_NC_MEDIAN_BLUR) {
    // medianBlur(srcGray, srcGray, filterMaskSize) (:481-483), then the histogram of the result
    const int k = (int)((options >> 8) & 0xffu);
    if (k < 1 || (k & 1) == 0)
      return fail(c, MSG_EINVAL, "MEDIAN_BLUR mask size %d: must be odd (medianBlur's assertion)", k);
    if (N > 0) {
      if (c->gscr2_n < N) {
        dfree(c->d_gscr2);
        c->gscr2_n = 0;
        HIPCHK(c, hipMalloc((void**)&c->d_gscr2, N + 16));
        c->gscr2_n = N;
      }
      const int grid = (int)std::max<long long>(1, std::min<long long>(8192, (N + 255) / 256));
      LAUNCH(c, KID_GRAY, st, k_gray, dim3(grid), dim3(256), 0, (const uint8_t*)d_bgr, N, c->d_gscr2);
      if (k > 1)
        LAUNCH(c, KID_MEDIAN, st, k_median, dim3((cols + MED_BS - 1) / MED_BS, (rows + MED_ROWS - 1) / MED_ROWS),
               dim3(MED_BS), 0, c->d_gscr2, g, rows, cols, k);
      else
        HIPCHK(c, hipMemcpyAsync(g, c->d_gscr2, N, hipMemcpyDeviceToDevice, st));
      HIPCHK(c, hipGetLastError());
    }
    rc = gray_hist(c, g, N, nullptr, hist, st, true);
  } else if (options & MSG_NC_BILATERAL) {
    // bilateralFilter(srcGray, dst, d, 2d, 2d) (:488-495), then the histogram of dst
    rc = nc_bilateral(c, (const uint8_t*)d_bgr, rows, cols, (int)((options >> 8) & 0xffu), g, st);
    if (rc) return rc;
    rc = gray_hist(c, g, N, nullptr, hist, st, true);
  } else {
    rc = gray_hist(c, (const uint8_t*)d_bgr, N, g, hist, st);
  }
  if (rc) return rc;
  int n = 0;
  std::vector<msg_bright_level> all(256);  // at most one level closes per bin 1..255
  rc = msg_nc_levels(hist, rows, cols, depth, options, all.data(), (int)all.size(), &n);
  if (rc == MSG_ERANGE && n == 0)
    return fail(c, MSG_ERANGE, "multi-Otsu search space too large (the reference's otsuPart "
                               "enumerates ~C(128, k) splits)");
  if (rc == MSG_ESTATE)
    return fail(c, MSG_ESTATE, "no brightness level (the reference throws here)");
  if (rc) return fail(c, rc, "level computation failed (%d)", rc);
  int32_t lut[256];
  msg_nc_marker_lut(all.data(), n, options, lut);
  rc = nc_markers(c, g, N, lut, (int32_t*)d_markers, st);
  if (rc) return rc;
  for (int i = 0; i < n && i < max_levels; ++i) levels[i] = all[i];
  *n_levels = n;
  if (n > max_levels) return fail(c, MSG_ERANGE, "%d levels, array holds %d", n, max_levels);
  return MSG_OK;
}

int msg_nc_marker_stage(msg_ctx* c, const uint8_t* bgr, size_t bgr_stride, int rows, int cols,
                        int depth, unsigned options, int32_t* markers, size_t marker_stride,
                        msg_bright_level* levels, int max_levels, int* n_levels) {
  int rc = host_args(c, bgr, bgr_stride, markers, marker_stride, rows, cols);
  if (rc) return rc;
  if (!n_levels || (max_levels > 0 && !levels)) return fail(c, MSG_EINVAL, "null level array");
  const long long N = (long long)rows * cols;
  HIPCHK(c, hipSetDevice(c->dev));
  rc = ensure_stage(c, std::max(N, 1ll));
  if (rc) return rc;
  hipStream_t st = c->own;
  if (N > 0)
    HIPCHK(c, hipMemcpy2DAsync(c->d_img, (size_t)cols * 3, bgr, bgr_stride, (size_t)cols * 3, rows,
                               hipMemcpyHostToDevice, st));
  rc = msg_nc_marker_stage_dev(c, c->d_img, rows, cols, depth, options, c->d_gray, c->d_mk, levels,
                               max_levels, n_levels, st);
  if (rc) return rc;
  if (N > 0)
    HIPCHK(c, hipMemcpy2DAsync(markers, marker_stride, c->d_mk, (size_t)cols * 4, (size_t)cols * 4,
                               rows, hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipStreamSynchronize(st));
  return MSG_OK;
}

int msg_blur_mask_size(int rows, int cols) { return blur_mask_size(rows, cols); }

int msg_shape_markers_dev(msg_ctx* c, const void* d_bgr, int rows, int cols, int ksize,
                          void* d_markers, int* depth, int* ncomp, void* d_blur, void* d_edges,
                          void* d_mask, void* stream) {
  if (!c) return MSG_EINVAL;
  int rc = check_size(c, rows, cols);
  if (rc) return rc;
  if (!depth || !ncomp) return fail(c, MSG_EINVAL, "null depth / ncomp pointer");
  *depth = *ncomp = 0;
  const long long N = (long long)rows * cols;
  if (N == 0) return MSG_OK;
  if (!d_bgr || !d_markers) return fail(c, MSG_EINVAL, "null device pointer");
  const int k = ksize > 0 ? ksize : blur_mask_size(rows, cols);
  if (k % 2 == 0 || k > 255) return fail(c, MSG_EINVAL, "median size %d: odd and <= 255", k);
  HIPCHK(c, hipSetDevice(c->dev));
  StreamScope scope(c, stream);
  if (scope.rc) return scope.rc;
  hipStream_t st = scope.st;
  const int H = rows, W = cols;
  const long long nb = (long long)((H + 1) >> 1) * ((W + 1) >> 1);
  rc = ensure_shape(c, N, nb);
  if (rc) return rc;
  uint8_t* gray = c->d_sh8;
  uint8_t* blur = gray + N;
  uint8_t* cls = blur + N;
  uint8_t* edges = cls + N;
  uint8_t* mask = edges + N;
  uint8_t* flag = mask + N;
  int* L = c->d_sh32;
  int* K = L + N;
  const int grid = stream_grid(N);
  LAUNCH(c, KID_GRAY, st, k_gray, dim3(grid), dim3(256), 0, (const uint8_t*)d_bgr, N, gray);
  const uint8_t* b = gray;
  if (k > 1) {
    LAUNCH(c, KID_MEDIAN, st, k_median, dim3((W + MED_BS - 1) / MED_BS, (H + MED_ROWS - 1) / MED_ROWS),
           dim3(MED_BS), 0, gray, blur, H, W, k);
    b = blur;
  }
  LAUNCH(c, KID_CANNY, st, k_canny_nms, dim3((W + CN_TX - 1) / CN_TX, (H + CN_TY - 1) / CN_TY), dim3(256), 0,
         b, cls, H, W, 5, 50);  // Canny(brdGray, brdGray, 5, 5 * 10): cvFloor of both thresholds
  HIPCHK(c, hipGetLastError());
  // hysteresis: candidates 8-connected to a strong candidate
  rc = ccl(c, cls, L, H, W, 0, st);
  if (rc) return rc;
  HIPCHK(c, hipMemsetAsync(flag, 0, N, st));
  LAUNCH(c, KID_CCL, st, k_hyst_mark, dim3(grid), dim3(256), 0, cls, L, flag, N);
  LAUNCH(c, KID_CCL, st, k_hyst_edges, dim3(grid), dim3(256), 0, cls, L, flag, edges, N);
  LAUNCH(c, KID_RING, st, k_ring_median3, dim3((W + RG_T - 1) / RG_T, (H + RG_T - 1) / RG_T), dim3(256), 0,
         edges, mask, H, W);
  HIPCHK(c, hipGetLastError());
  // markers: 8-connected components of the mask, numbered by their first 2x2 block
  rc = ccl(c, mask, L, H, W, 1, st);
  if (rc) return rc;
  HIPCHK(c, hipMemsetAsync(K, 0x7f, N * sizeof(int), st));
  HIPCHK(c, hipMemsetAsync(c->d_shF, 0, nb * sizeof(int), st));
  LAUNCH(c, KID_NUMBER, st, k_cc_minkey, dim3((W + 255) / 256, H), dim3(256), 0, L, K, H, W);
  LAUNCH(c, KID_NUMBER, st, k_cc_firstflag, dim3(grid), dim3(256), 0, L, K, c->d_shF, N, W);
  size_t tb = c->scan_tmp_bytes;
  HIPCHK(c, hipcub::DeviceScan::ExclusiveSum(c->d_scan_tmp, tb, c->d_shF, c->d_shP, (int)nb, st));
  LAUNCH(c, KID_NUMBER, st, k_cc_label, dim3(grid), dim3(256), 0, L, K, c->d_shP, (int32_t*)d_markers, N);
  HIPCHK(c, hipGetLastError());
  int tailv[2] = {0, 0};
  HIPCHK(c, hipMemcpyAsync(&tailv[0], c->d_shP + nb - 1, sizeof(int), hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipMemcpyAsync(&tailv[1], c->d_shF + nb - 1, sizeof(int), hipMemcpyDeviceToHost, st));
  // holes: background components (4-connected) that do not touch the frame
  rc = ccl(c, mask, L, H, W, 2, st);
  if (rc) return rc;
  HIPCHK(c, hipMemsetAsync(flag, 0, N, st));
  HIPCHK(c, hipMemsetAsync(c->d_shcnt, 0, sizeof(int), st));
  LAUNCH(c, KID_HOLES, st, k_hole_border, dim3(std::max(1, (int)std::min<long long>(1024, (2ll * (H + W) + 255) / 256))),
         dim3(256), 0, L, flag, H, W);
  LAUNCH(c, KID_HOLES, st, k_hole_count, dim3(grid), dim3(256), 0, L, flag, c->d_shcnt, N);
  HIPCHK(c, hipGetLastError());
  int holes = 0;
  HIPCHK(c, hipMemcpyAsync(&holes, c->d_shcnt, sizeof(int), hipMemcpyDeviceToHost, st));
  if (d_blur) HIPCHK(c, hipMemcpyAsync(d_blur, b, N, hipMemcpyDeviceToDevice, st));
  if (d_edges) HIPCHK(c, hipMemcpyAsync(d_edges, edges, N, hipMemcpyDeviceToDevice, st));
  if (d_mask) HIPCHK(c, hipMemcpyAsync(d_mask, mask, N, hipMemcpyDeviceToDevice, st));
  HIPCHK(c, hipStreamSynchronize(st));
  if (c->prof) collect_profile(c);
  *ncomp = tailv[0] + tailv[1];
  *depth = *ncomp + holes;
  return MSG_OK;
}

int msg_color_markers_dev(msg_ctx* c, const void* d_bgr, int rows, int cols, void* d_sharp,
                          void* d_markers, int* depth, void* stream) {
  if (!c) return MSG_EINVAL;
  int rc = check_size(c, rows, cols);
  if (rc) return rc;
  if (!depth) return fail(c, MSG_EINVAL, "null depth pointer");
  *depth = 0;
  const long long N = (long long)rows * cols;
  if (N == 0) return MSG_OK;
  if (!d_bgr || !d_sharp || !d_markers) return fail(c, MSG_EINVAL, "null device pointer");
  if (d_bgr == d_sharp) return fail(c, MSG_EINVAL, "d_sharp must not alias d_bgr");
  if (!aligned(d_sharp, 4)) return fail(c, MSG_EINVAL, "d_sharp must be 4-byte aligned");
  HIPCHK(c, hipSetDevice(c->dev));
  StreamScope scope(c, stream);
  if (scope.rc) return scope.rc;
  hipStream_t st = scope.st;
  const int H = rows, W = cols;
  rc = ensure_shape(c, N, 1);
  if (rc) return rc;
  rc = ensure_color(c, N);
  if (rc) return rc;
  uint8_t* gray = c->d_sh8;
  uint8_t* thr = gray + N;
  uint8_t* pk = thr + N;
  uint8_t* frame = pk + N;
  unsigned* dt = (unsigned*)c->d_cm32;
  int* L = c->d_cm32 + N;
  int* L2 = L + N;
  int* R1 = L2 + N;
  int* R2 = R1 + N;
  int2* comps = c->d_cmreg;
  int2* holes = comps + N;
  int* cnt = c->d_cmcnt;  // [0,1] region counts, [2,3] min/max distance, [8..15] sweep flags
  const int grid = stream_grid(N);
  const dim3 rowg((W + 255) / 256, H);
  uint8_t* sharp = (uint8_t*)d_sharp;
  LAUNCH(c, KID_COLOR, st, k_cm_sharpen, rowg, dim3(256), 0, (const uint8_t*)d_bgr, sharp, H, W);
  HIPCHK(c, hipGetLastError());
  int32_t hist[256];
  rc = gray_hist(c, sharp, N, gray, hist, st);  // bwMat: cvtColor(BGR2GRAY) + its histogram
  if (rc) return rc;
  const int t = (int)otsu_threshold(hist, N);
  LAUNCH(c, KID_COLOR, st, k_cm_dt_init, dim3(grid), dim3(256), 0, gray, t, dt, N);
  // chamfer distance: relaxation sweeps until one changes nothing (flags checked per 8 sweeps)
  int flags[8];
  const int max_sweeps = H + W + 16;
  bool done = false;
  for (int s0 = 0; s0 < max_sweeps && !done; s0 += 8) {
    HIPCHK(c, hipMemsetAsync(cnt + 8, 0, 8 * sizeof(int), st));
    for (int k = 0; k < 8; ++k) LAUNCH(c, KID_COLOR, st, k_cm_dt_sweep, rowg, dim3(256), 0, dt, H, W, cnt + 8 + k);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(flags, cnt + 8, sizeof(flags), hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    for (int k = 0; k < 8; ++k) done = done || flags[k] == 0;
  }
  if (!done) return fail(c, MSG_ESTATE, "distance transform did not converge");
  // normalize(NORM_MINMAX): min / max of the float distances (monotone in the fixed point)
  unsigned mm[2] = {0xffffffffu, 0};
  HIPCHK(c, hipMemcpyAsync(cnt + 2, mm, sizeof(mm), hipMemcpyHostToDevice, st));
  LAUNCH(c, KID_COLOR, st, k_cm_minmax, dim3(grid), dim3(256), 0, dt, N, (unsigned*)(cnt + 2));
  HIPCHK(c, hipMemcpyAsync(mm, cnt + 2, sizeof(mm), hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipStreamSynchronize(st));
  const float dlo = (float)mm[0] * (1.0f / 65536.0f), dhi = (float)mm[1] * (1.0f / 65536.0f);
  float scf = 0.f, shf = 0.f;
  int use_shift = 0;
  if ((double)dhi - (double)dlo > 2.220446049250313e-16) {
    const double sc = 1.0 / ((double)dhi - (double)dlo);
    scf = (float)sc;
    shf = (float)(-(double)dlo * sc);
    use_shift = dlo != 0.f;
  }
  LAUNCH(c, KID_COLOR, st, k_cm_peaks, dim3(grid), dim3(256), 0, dt, scf, shf, use_shift, thr, N);
  LAUNCH(c, KID_COLOR, st, k_cm_dilate3, rowg, dim3(256), 0, thr, pk, H, W);
  HIPCHK(c, hipGetLastError());
  // contours through components: foreground 8-connected, background 4-connected, holes = the
  // background components that do not touch the frame
  rc = ccl(c, pk, L, H, W, 1, st);
  if (rc) return rc;
  rc = ccl(c, pk, L2, H, W, 2, st);
  if (rc) return rc;
  HIPCHK(c, hipMemsetAsync(frame, 0, N, st));
  LAUNCH(c, KID_HOLES, st, k_hole_border, dim3(std::max(1, (int)((2ll * W + 2ll * H + 255) / 256))), dim3(256), 0,
         L2, frame, H, W);
  HIPCHK(c, hipMemsetAsync(cnt, 0, 2 * sizeof(int), st));
  LAUNCH(c, KID_COLOR, st, k_cm_regions, dim3(grid), dim3(256), 0, pk, L, L2, frame, W, N, comps, holes, cnt);
  HIPCHK(c, hipGetLastError());
  int nreg[2];
  HIPCHK(c, hipMemcpyAsync(nreg, cnt, sizeof(nreg), hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipStreamSynchronize(st));
  const int nc = nreg[0], nh = nreg[1];
  std::vector<int2> hc(nc), hh(nh);
  if (nc) HIPCHK(c, hipMemcpyAsync(hc.data(), comps, nc * sizeof(int2), hipMemcpyDeviceToHost, st));
  if (nh) HIPCHK(c, hipMemcpyAsync(hh.data(), holes, nh * sizeof(int2), hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipStreamSynchronize(st));
  // RETR_CCOMP order: components (outer borders, discovered at their first pixel) in reverse
  // discovery order, each followed by its holes (discovered left of their first pixel) in
  // reverse discovery order -- cvInsertNodeIntoTree prepends, cvTreeToNodeSeq walks depth-first
  std::sort(hc.begin(), hc.end(), [](const int2& a, const int2& b) { return a.x > b.x; });
  std::sort(hh.begin(), hh.end(), [](const int2& a, const int2& b) { return a.x > b.x; });
  std::vector<std::pair<int, int>> cidx;  // (root, index)
  std::vector<std::pair<int, int>> hidx;
  {
    // holes grouped by parent component root, already in descending key order
    std::vector<std::pair<int, int>> byparent(nh);  // (parent root, position in hh)
    for (int k = 0; k < nh; ++k) byparent[k] = {hh[k].y, k};
    std::stable_sort(byparent.begin(), byparent.end(),
                     [](const std::pair<int, int>& a, const std::pair<int, int>& b) { return a.first < b.first; });
    int idx = 0;
    cidx.reserve(nc);
    hidx.reserve(nh);
    for (int k = 0; k < nc; ++k) {
      const int r = hc[k].x;
      cidx.push_back({r, idx++});
      auto lo = std::lower_bound(byparent.begin(), byparent.end(), std::make_pair(r, -1));
      for (auto it = lo; it != byparent.end() && it->first == r; ++it) hidx.push_back({hh[it->second].x, idx++});
    }
    if ((int)hidx.size() != nh) return fail(c, MSG_ESTATE, "a hole without its component");
  }
  *depth = nc + nh;
  // covering labels: 1 + the highest index among the contours whose fill covers a region
  std::vector<std::pair<int, int>> hinfo(nh);  // sorted by root: (root, position in hidx)
  for (int k = 0; k < nh; ++k) hinfo[k] = {hidx[k].first, k};
  std::sort(hinfo.begin(), hinfo.end());
  std::vector<std::pair<int, int>> cinfo(nc);
  for (int k = 0; k < nc; ++k) cinfo[k] = {cidx[k].first, k};
  std::sort(cinfo.begin(), cinfo.end());
  auto hpos = [&](int root) -> int {
    auto it = std::lower_bound(hinfo.begin(), hinfo.end(), std::make_pair(root, -1));
    return (it != hinfo.end() && it->first == root) ? it->second : -1;
  };
  auto cpos = [&](int root) -> int {
    auto it = std::lower_bound(cinfo.begin(), cinfo.end(), std::make_pair(root, -1));
    return (it != cinfo.end() && it->first == root) ? it->second : -1;
  };
  std::vector<int> cenc(nc, -2);  // highest index among the holes enclosing component k
  std::vector<int> hpar(nh), cholepar(nc);
  for (int k = 0; k < nh; ++k) {
    const int pc = cpos(hh[k].y);
    if (pc < 0) return fail(c, MSG_ESTATE, "hole parent is not a component root");
    hpar[hpos(hh[k].x)] = pc;
  }
  for (int k = 0; k < nc; ++k) cholepar[cpos(hc[k].x)] = (hc[k].y >= 0) ? hpos(hc[k].y) : -1;
  std::vector<int> stack;
  for (int k0 = 0; k0 < nc; ++k0) {
    int k = k0;
    while (cenc[k] == -2) {  // walk up the chain of enclosing holes, then unwind
      stack.push_back(k);
      const int h = cholepar[k];
      if (h < 0) {
        cenc[k] = -1;
        stack.pop_back();
        break;
      }
      k = hpar[h];
      if ((int)stack.size() > nc) return fail(c, MSG_ESTATE, "component nesting cycle");
    }
    while (!stack.empty()) {
      const int j = stack.back();
      stack.pop_back();
      const int h = cholepar[j];
      cenc[j] = std::max(hidx[h].second, cenc[hpar[h]]);
    }
  }
  std::vector<int> up_root(nc + nh), up_r1(nc + nh), up_r2(nc + nh);
  for (int k = 0; k < nc; ++k) {
    up_root[k] = cidx[k].first;
    up_r1[k] = 1 + std::max(cidx[k].second, cenc[k]);
    up_r2[k] = 0;
  }
  for (int k = 0; k < nh; ++k) {
    up_root[nc + k] = hidx[k].first;
    up_r1[nc + k] = 1 + std::max(hidx[k].second, cenc[hpar[k]]);
    up_r2[nc + k] = 1 + hidx[k].second;
  }
  if (nc + nh) {
    // region labels at their roots: (root, r1, r2) triples through the region-list buffer
    int* tri = (int*)c->d_cmreg;
    const int n3 = nc + nh;
    HIPCHK(c, hipMemcpyAsync(tri, up_root.data(), n3 * sizeof(int), hipMemcpyHostToDevice, st));
    HIPCHK(c, hipMemcpyAsync(tri + n3, up_r1.data(), n3 * sizeof(int), hipMemcpyHostToDevice, st));
    HIPCHK(c, hipMemcpyAsync(tri + 2 * n3, up_r2.data(), n3 * sizeof(int), hipMemcpyHostToDevice, st));
    LAUNCH(c, KID_COLOR, st, k_cm_scatter, dim3(std::max(1, (n3 + 255) / 256)), dim3(256), 0, tri, n3, R1, R2);
  }
  // circle((5,5), 3, 255, FILLED): half widths per |dy| from OpenCV's integer circle walk
  int half[4] = {-1, -1, -1, -1};
  {
    int err = 0, dx = 3, dy = 0, plus = 1, minus = (3 << 1) - 1;
    while (dx >= dy) {
      half[dy] = std::max(half[dy], dx);
      if (dx <= 3) half[dx] = std::max(half[dx], dy);
      ++dy;
      err += plus;
      plus += 2;
      const int mask = (err <= 0) - 1;
      err -= minus & mask;
      dx += mask;
      minus -= mask & 2;
    }
  }
  LAUNCH(c, KID_COLOR, st, k_cm_paint, rowg, dim3(256), 0, pk, L, L2, frame, R1, R2, (int32_t*)d_markers, H, W,
         make_int4(half[0], half[1], half[2], half[3]), make_int4(0, 0, 0, 0));
  HIPCHK(c, hipGetLastError());
  if (c->prof) {
    HIPCHK(c, hipStreamSynchronize(st));
    collect_profile(c);
  }
  return MSG_OK;
}

int msg_color_markers(msg_ctx* c, const uint8_t* bgr, size_t bgr_stride, int rows, int cols,
                      uint8_t* sharp, size_t sharp_stride, int32_t* markers, size_t marker_stride,
                      int* depth) {
  int rc = host_args(c, bgr, bgr_stride, markers, marker_stride, rows, cols);
  if (rc) return rc;
  const long long N = (long long)rows * cols;
  if (N > 0 && (!sharp || sharp_stride < (size_t)cols * 3)) return fail(c, MSG_EINVAL, "bad sharp buffer");
  HIPCHK(c, hipSetDevice(c->dev));
  rc = ensure_stage(c, std::max(N, 1ll));
  if (rc) return rc;
  hipStream_t st = c->own;
  if (N > 0)
    HIPCHK(c, hipMemcpy2DAsync(c->d_img, (size_t)cols * 3, bgr, bgr_stride, (size_t)cols * 3, rows,
                               hipMemcpyHostToDevice, st));
  rc = msg_color_markers_dev(c, c->d_img, rows, cols, c->d_dst, c->d_mk, depth, st);
  if (rc) return rc;
  if (N > 0) {
    HIPCHK(c, hipMemcpy2DAsync(sharp, sharp_stride, c->d_dst, (size_t)cols * 3, (size_t)cols * 3, rows,
                               hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipMemcpy2DAsync(markers, marker_stride, c->d_mk, (size_t)cols * 4, (size_t)cols * 4,
                               rows, hipMemcpyDeviceToHost, st));
  }
  HIPCHK(c, hipStreamSynchronize(st));
  return MSG_OK;
}

int msg_shape_markers(msg_ctx* c, const uint8_t* bgr, size_t bgr_stride, int rows, int cols,
                      int ksize, int32_t* markers, size_t marker_stride, int* depth, int* ncomp) {
  int rc = host_args(c, bgr, bgr_stride, markers, marker_stride, rows, cols);
  if (rc) return rc;
  const long long N = (long long)rows * cols;
  HIPCHK(c, hipSetDevice(c->dev));
  rc = ensure_stage(c, std::max(N, 1ll));
  if (rc) return rc;
  hipStream_t st = c->own;
  if (N > 0)
    HIPCHK(c, hipMemcpy2DAsync(c->d_img, (size_t)cols * 3, bgr, bgr_stride, (size_t)cols * 3, rows,
                               hipMemcpyHostToDevice, st));
  rc = msg_shape_markers_dev(c, c->d_img, rows, cols, ksize, c->d_mk, depth, ncomp, nullptr, nullptr,
                             nullptr, st);
  if (rc) return rc;
  if (N > 0)
    HIPCHK(c, hipMemcpy2DAsync(markers, marker_stride, c->d_mk, (size_t)cols * 4, (size_t)cols * 4,
                               rows, hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipStreamSynchronize(st));
  return MSG_OK;
}

}  // extern "C"
