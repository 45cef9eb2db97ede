// ws_shared.h -- types shared by the gfx950 kernels (ws_kernels.hip) and the host engine
// (msegment_capi.hip).  See ws_kernels.hip for the algorithm and the HBM layout.
#pragma once
#include <stdint.h>

namespace msg {

constexpr int NQ = 256;          // bucket levels = L-inf BGR distances 0..255 (cv::watershed NQ)
constexpr int BS = 256;          // threads per block of the chunk kernels
constexpr int CH = 4096;         // items per chunk of the ordered multi-bucket append
constexpr int SUB = CH / BS;     // sub-rounds per chunk
constexpr int WSHED = -1;        // cv::watershed WSHED
constexpr int INQ = -2;          // cv::watershed IN_QUEUE, before the pixel has a queue slot
// A queued pixel's state word also carries its queue slot (one random load instead of two):
// state = -3 - slot  (<= -3).  Slots are < 4N + 16 < 2^31 - 512 (check_size), clear of the
// phase-1 states 0x80000000 | level.
__host__ __device__ inline int queued_state(int slot) { return -3 - slot; }
__host__ __device__ inline int state_slot(int state) { return -3 - state; }
constexpr int NONE = 0x7fffffff;
constexpr int RBS = 512;           // threads per k_resolve block (3 per CU at its 80-VGPR budget)
constexpr int SMALL_MAX = 4096;    // batches up to this size run in k_scan's one-workgroup loop
constexpr int PAL_LDS_MAX = 16384; // palettes up to this many labels are staged in LDS
constexpr int MERGE_CAP = 1 << 22; // largest multi-segment batch (items)
constexpr int WMIN = 64;           // smallest batch window (one wave: the tiny-batch loop)
constexpr int FAST_CH = 120;       // k_commit_fast: 4 FAST_CH + 1 blocks of 1024 threads (resident
                                   // at 2 per CU), each sub-round block taking up to FAST_PASS
constexpr int FAST_PASS = 4;       // 1024-item sub-rounds: batches of up to FAST_PASS * FAST_CH chunks
// Batch window after committing ncommit of n items: an interrupt cut (a push below the item's
// level) means the queue order is turning over fast, so the next batch is a short prefix; a
// batch that filled its window uncut quadruples it.  Prefixes of the queue order: exact.
__host__ __device__ inline int next_wcap(int wcap, int n, int ncommit, bool icut) {
  const int cap = wcap ? wcap : MERGE_CAP;
  if (icut) return ncommit * 2 > WMIN ? ncommit * 2 : WMIN;
  if (n >= cap) return (cap >= MERGE_CAP / 4) ? 0 : cap * 4;
  return wcap;
}
constexpr long long SPIN_LIMIT_TICKS = 200000000ll;  // 2 s of s_memrealtime (100 MHz)
constexpr long long YIELD_TICKS = 5000;              // 50 us: a k_resolve wait this long checks its owner

// Per-pixel flood state is TILED: 4x4-pixel tiles of 8-byte {state, w4} words (128 B = one L2
// line per tile), tiles row-major, Wt tiles per tile row.  A pixel and its 4 neighbours mostly
// share a line, so a queue item costs ~2 random lines instead of ~4.
constexpr int CAP_SLOTS = 64;  // spread of the capacity-histogram atomics (same-address contention)
constexpr int RSEG = 512;   // columns per raster chunk of the phase-1 compaction (128 tiles) = k_prep threads
__host__ __device__ inline long long tix(int r, int c, int Wt) {
  return ((long long)((long long)(r >> 2) * Wt + (c >> 2)) << 4) | ((r & 3) << 2) | (c & 3);
}
// neighbour of tiled pixel t in direction d (0 left, 1 right, 2 up, 3 down); must exist
__host__ __device__ inline long long nb_of(long long t, int d, int Wt) {
  const long long row = (long long)Wt << 4;
  switch (d) {
    case 0: return (t & 3) ? t - 1 : t - 13;
    case 1: return ((t & 3) != 3) ? t + 1 : t + 13;
    case 2: return (t & 12) ? t - 4 : t - row + 12;
    default: return ((t & 12) != 12) ? t + 4 : t + row - 12;
  }
}
// phase-1 marker (k_prep -> k_compact): IN_QUEUE with its initial level lv
__host__ __device__ inline int p1_state(int lv) { return (int)(0x80000000u | (unsigned)lv); }
__host__ __device__ inline bool is_p1(int s) { return ((unsigned)s ^ 0x80000000u) < 256u; }

constexpr int ERR_TIMEOUT = 1;
constexpr int ERR_STATE = 2;
constexpr int ERR_CAPACITY = 4;
constexpr int ERR_LEFTOVER = 8;  // a queued (or phase-1) state survived the flood (k_untile)

// Speculative generations (k_spec_round / k_spec_flatten, ws_kernels.hip): the interrupt-dense
// regime.  A generation is the whole lowest bucket; each item's execution is its own pop plus its
// cascade (every level below the bucket's, to exhaustion), repeated in rounds until no execution
// changes (the serial result is the unique fixed point: item i depends only on items < i).
constexpr int SPEC_WIN = 1 << 20;   // items per generation (claim ranks have 22 bits)
constexpr int SPEC_BS = 256;        // threads per k_spec_round block
constexpr int SPEC_QCAP = 32;      // per-lane cascade queue in LDS ("hot": the smallest keys)
constexpr int SPEC_RL = 256;       // records per execution in lane scratch, the rest in pool chunks
constexpr int SPEC_CCAP = 4096;     // "cold" cascade entries of one execution (a pool chunk): more = overflow
constexpr int SPEC_XCH = 2048;      // records per pool chunk past the first SPEC_RL
constexpr int SPEC_NX = 4;          // such chunks per execution: more records = overflow
constexpr int SPEC_MAXREC = SPEC_RL + SPEC_NX * SPEC_XCH;  // longest execution a lane runs
constexpr int SPEC_MAXREC_SHORT = 256;  // pops an execution may run (more: a capacity overflow,
                                        // serial pops) -- except the stable prefix's head and, in
                                        // deep mode, executions from round 2 on (k_spec_round)
constexpr int SPEC_ROUNDS_MAX = 64; // rounds per generation before the stable prefix is committed
constexpr int SPEC_FT = 1024;       // items per k_spec_flatten tile
constexpr int SPEC_QUIET = 4096;    // a generation this large without a cascade ends the regime
// The regime is judged on COUNTS, not on the clock (round 5): a generation is priced by a model of
// its device time fitted to the round-5 flood probes -- 37 us per round (launches, gather, dealing,
// the round's end) + 1.9 us per pop of each round's longest execution (a round lasts as long as
// its longest cascade; spec_longest_pops) -- against serial pops at 0.8 us each.  The wall clock
// it replaced flipped decisions whenever the device stalled (a first flood's allocations, a
// profiler, concurrent floods): album.jpg's flood varied 1084-1497 ms from run to run.  A/B of the
// serial price (profiles/r05k_regime_probe*.log): 0.5 us -> album.jpg 1226 ms (mostly serial pops,
// 0.53 us each there), 0.8 us -> 1088 ms; notConnectedMarkers' seeds at 1024^2 882 / 921 ms.
constexpr int SPEC_ROUND_TICKS = 3700;       // model: 10 ns ticks per round
constexpr int SPEC_POP_TICKS = 190;          // model: ticks per pop of a round's longest execution
constexpr int SPEC_SERIAL_TICKS = 80;        // ~0.8 us per serial pop: a regime slower than that per
constexpr int SPEC_JUDGE_GENS = 16;          // committed pop (its fallbacks' serial pops included),
                                             // after this many generations, ends for
constexpr int SPEC_COOL_POPS = 65536;        // this many serial pops (doubling per repeat)
constexpr int SPEC_JUDGE_TICKS = 200000;     // slow generations are judged after 4 once 2 ms (model) passed
constexpr int SPEC_COMMIT_TICKS = 3000;      // ~30 us: a generation's ordered append (k_scan, k_scatter)

// A tiled pixel's speculative-generation words (k_spec_round reads a neighbour's whole record
// with two 16-B loads).
struct alignas(32) SpecPx {
  unsigned long long cl[2];  // round claims by round parity: {round tag, inverted rank, popped}
  unsigned long long fin;    // final claim: {generation tag, popped, label}
  int lab[2];                // label of the popper, by round parity
};
static_assert(sizeof(SpecPx) == 32, "SpecPx is one 32-byte record");

struct SpecCtl {
  unsigned T;     // current round tag: round claims in scl[T & 1], labels in slab[T & 1]
  unsigned G;     // tag of the generation's first round (final claims carry it)
  int L, n, bstart;
  int P;          // stable prefix: items < P are final
  int Pold;       // items [Pold, P) are final but not yet promoted (their claims -> sfin)
  int Pprom;      // at flatten: items < Pprom were promoted (records via sfrec)
  int rounds;     // rounds of this generation so far
  int state;      // 0 none, 1 rounds running, 2 ready to flatten
  int on;         // regime: batches are speculative generations
  int block;      // after a fallback: the regime may resume once the lowest level is >= block
  int ticket;     // blocks finished this round
  int fallback;   // the commit ends the regime (overflow at the stable prefix)
  int ftile;      // k_spec_flatten tile dealing
  int cool;       // serial pops to go before the regime may start again
  int accg;       // generations since the regime started (fallback resumptions included)
  int fails;      // consecutive times the regime ended for being slower than serial pops
  int cools;      // all such times in this flood
  int fresh;      // the next start opens a new judging span (flood start, after such an end)
  long long tstart, pstart;  // regime start: s_memrealtime, Ctl.pops
  long long tgen;            // s_memrealtime at the current generation's start (spec_begin)
  long long gpops_total, gticks_total;  // whole flood: pops the generations committed, their time
  long long tspec, pspec;    // since the regime start: generations' modelled time (+ a commit
                             // estimate each) and the pops they committed -- what the regime is
                             // judged on
  long long gens, rounds_total, execs, cpops, fallbacks;
  unsigned long long rmax;  // diagnostics: longest wave of this round (10 ns ticks) | waits | cascades
  unsigned long long rmax2; // ... | its dealing + promotion | its post-execution work
  int ov1, ov2;             // lowest overflowing rank of the last / the one-before-last round
  int deep;                 // 1: from round 2 on every execution may run SPEC_MAXREC pops; set
                            // by the flood's first cooldown, 2 (off for good) by a second one
  long long replays;        // executions whose cascade was replayed from the previous round
  long long xpops;          // pops k_spec_round ran pop by pop (top pops + cascade pops of the
                            // executions that were not replayed): its algorithmic unit
  int rxmax;                // this round's longest execution run pop by pop (pops)
  int pad_x;
  long long xlong;          // sum over the flood's rounds of rxmax (a round lasts about as long as
                            // its longest execution)
  long long gxlong0;        // xlong at the current generation's start
};

// desc word of a batch item: bits 0-31 the 4 edge weights, 32-35 push (or 0-neighbour) mask,
// 40-47 the item's level, 48-55 its segment.
__host__ __device__ inline unsigned long long make_desc(unsigned wts, unsigned mask, int lv, int sg) {
  return (unsigned long long)wts | ((unsigned long long)mask << 32) | ((unsigned long long)lv << 40) |
         ((unsigned long long)sg << 48);
}

// One segment of a batch: the current contents of bucket L, ranks [rank, rank + n).
struct Seg {
  int L;
  int bstart;      // absolute qbuf slot of the segment's first item
  int rank;        // batch rank of that item
  int n;
};

struct Batch {
  int L;           // level of the first segment (-1 for the phase-1 pseudo-batch)
  int bstart;      // absolute qbuf slot of rank 0
  int n;           // items in the batch, all segments (0 = nothing to do / finished)
  int nseg;        // segments (consecutive non-empty buckets in level order)
  unsigned epoch;  // tag of this batch's tl granules
  int ncommit;     // committed prefix (set by k_scan)
  int nchunk;      // chunks of the committed prefix (set by k_scan)
  int mode;        // 0 = flood batch, 1 = phase-1 pseudo-batch (items = ilist), 3 = speculative
                   // generation
  int rrun;        // k_resolve re-runs of this batch so far (chunks given up: see k_resolve)
};

struct Ctl {
  int qbase[NQ + 1];
  int qhead[NQ];
  int qtail[NQ];
  Batch bat;    // current batch (written by k_init_scan / k_scan, incl. its small-batch loop)
  Batch cbat;   // batch being committed by k_scatter (written by k_scan)
  Seg seg[NQ];  // segments of the current batch
  int cut;      // first rank of the current batch that pushes below its own level (NONE: none)
  int segcut;   // first segment invalidated by a push below its level (NONE: none)
  int minpush;  // lowest level pushed by the current batch (merge heuristic)
  int wcap;         // batch window (0 = whole buckets): shrinks after interrupt cuts, regrows
  int done;
  int error;      // (8-aligned: k_resolve's waits load {error, rgive} as one word)
  int rgive;      // a k_resolve block gave its chunk up this run (k_scan re-runs the batch)
  int remaining;  // queued items after the last batch was formed (host polling hint)
  long long batches;
  long long pops;
  long long items;   // sum of batch sizes resolved (committed or not)
  long long pushes;  // committed pushes appended to buckets
  unsigned rsv;      // epoch of the last batch k_resolve (or k_spec_flatten) decided
  int pad;
  SpecCtl spec;
  int spec_want;     // the serial regime was entered while the speculative engine was enabled but
                     // its workspace not yet allocated (Ws.spec_lazy): the host allocates it
  unsigned hold;     // epoch of a decided batch k_commit_fast declined (k_resolve must not re-run it)
  int ser_go;        // k_scan stopped at serial pops for k_serial_one, queued right after it
  int ser_seen;      // the flood has reached the serial regime (the host then queues k_serial_one)
  int pad4;
  // k_commit_fast: sub-round blocks done reading, by blockIdx % 8 (zeroed after): 480 atomics per
  // launch and the finalizer's polls, one 128-B line per counter (atomics on one line serialise at
  // the L2: with all 8 counters on one line k_commit_fast took 14.8 us per launch, round 4)
  struct alignas(128) Arrive {
    unsigned v;
    unsigned pad[31];
  };
  Arrive farrive[8];
  // k_spec_round's contended words, one 128-B line each: device-scope atomics on one line
  // serialise (~11 ns each), and a round issues thousands of them
  struct alignas(128) Hot {
    int v;
    int pad[31];
  };
  Hot sdeal;     // dispatch-order rank dealing
  Hot sfc, sovf; // lowest changed / overflowing rank of this round
  Hot slogtop;   // generation log records used
  Hot sxtop;     // k_spec_round's chunk pool used this round (cold cascade queues, record chunks)
  // where the committed items went (bench.py's per-kernel algorithmic bytes), counted off the
  // critical paths: k_commit_fast's share is what the other paths leave (no atomics in it)
  long long spops, s0pops, spushes;  // committed by k_scan + k_scatter: all modes, flood batches only
  long long lpops, lpushes;          // popped one workgroup / one wave at a time (k_scan's loop,
                                     // k_serial_multi)
  long long ritems;                  // items of the batches k_resolve decided (re-runs included):
                                     // k_resolve's algorithmic unit
};

static_assert(__builtin_offsetof(Ctl, error) % 8 == 0 && __builtin_offsetof(Ctl, rgive) == __builtin_offsetof(Ctl, error) + 4,
              "Ctl.error and Ctl.rgive must share one aligned 8-byte word");

struct Ws {
  const uint8_t* img;
  int32_t* mk;       // TILED pixel states (see tix): state of tiled pixel t at mk[t]
  int32_t* w4;       // the same tiling: 4 packed 8-bit weights (L,R,T,B) of pixel t at w4[t]
  int32_t* qbuf;     // bucket regions of tiled pixel indices
  int32_t* ilist;
  unsigned long long* tl;
  unsigned long long* desc;
  int32_t* ipx;      // pixel of each rank of the current batch (k_resolve -> k_scatter)
  int32_t* cnt;
  int32_t* coff;
  int32_t* tot;      // phase-1 pixels per raster chunk (k_prep -> k_init_scan)
  int32_t* choff;
  unsigned* capp;    // CAP_SLOTS x NQ partial bucket-capacity histograms (k_prep -> k_init_scan)
  unsigned long long* cflag;  // per k_resolve chunk: {epoch, run} of its claim, epoch of its completion
  Ctl* ctl;
  unsigned long long* diag;  // nullptr = off; else 8 counters (msg_set_diag)
  int* hmir;         // host-mapped progress mirror {iteration, done, error, remaining, spec, spec_want,
                     // fast batch}
  // speculative generations (nullptr when the engine is off): one 32-byte record per tiled
  // pixel (indexed like mk) holding both round parities' claims and labels and the final claim,
  // so that a pixel's view is one 128-B line instead of five arrays
  SpecPx* spx;
  unsigned long long* stl;   // SPEC_WIN top-pop granules {round tag, label}
  unsigned long long* slog;  // generation log: records {label, dmask, pixel}
  int4* srec;                // 2 x SPEC_WIN {log base, records, round tag, capacity overflow} per round parity
  unsigned long long* ssig;  // 2 x SPEC_WIN execution signatures
  int2* sfrec;               // SPEC_WIN {log base, records} of promoted items
  unsigned long long* stmp;  // lane scratch: SPEC_RL records per k_spec_round thread
  unsigned long long* sflag; // k_spec_flatten tile prefixes {generation tag, inclusive sum}
  unsigned* sdirt;           // 2 x snp change marks per round parity: round tag of the last changed
                             // execution whose claims (old or new) covered the pixel
  long long snp;
  long long slogcap;
  int spec_lazy;     // 1: engine enabled, workspace not allocated yet (k_scan reports spec_want)
  int H, W;
  int Wt;            // tiles per tile row = ceil(W / 4)
  int marg;          // tiled entries of margin before mk / w4 (mk - marg starts the state array)
  int nseg;          // raster chunks per image row = ceil(W / RSEG)
  long long N;
  long long qcap;
  // round 4 (after the fields every flood kernel reads, which keep their offsets)
  unsigned long long* sxp;   // chunk pool of a round: an execution's cold cascade queue (SPEC_CCAP
                             // keys) and its records past SPEC_RL (SPEC_XCH each), reset every round
  long long sxcap;
  int multi;                 // 1: a flood of a many-floods batch: k_scan stops after each commit (no
                             // small-batch loop), k_serial_multi pops it together with the others
};

}  // namespace msg
