// spec_kernels.hip -- speculative generations: the exact flood's interrupt-dense regime (gfx950).
//
// cv::watershed (OpenCV 3.4.2, reached from PictureService.java:909) pops the
// oldest item of the lowest non-empty bucket.  On textured frames almost every few pops push a
// neighbour below the popped level (an "interrupt"), and the batch engine of ws_kernels.hip, which
// cuts a batch right after such an item, degenerates to a few pops per batch.  Here a GENERATION
// is the whole lowest bucket L instead (ranks 0..n-1 in FIFO order), never cut at interrupts:
//
//   * item j's EXECUTION is what the serial run does from its pop until the next item of bucket L
//     pops: the pop of its pixel (label = fold of labelled neighbours, pushes of unknown ones in
//     L,R,T,B order) followed by its CASCADE -- every push below L, popped lowest level first,
//     FIFO within a level, to exhaustion (a cascade only ever pops pixels it pushed itself);
//     pushes at levels >= L are deferred to the buckets in execution order;
//   * executions are speculative and repeated in ROUNDS.  Item j reads what items < j wrote:
//     the top pops of earlier adjacent items of the CURRENT round (waited for, as k_resolve
//     does: ranks are dealt in dispatch order, so every wait is on a running wave), everything
//     else through the PREVIOUS round's claims.  The serial order is the unique fixed point of
//     this triangular system, reached when no execution changes between two rounds; the stable
//     prefix P (items unchanged since the previous round, all of whose inputs are therefore
//     final) grows every round and is never executed again;
//   * CLAIMS: per pixel and round parity one 64-bit word {round tag, rank, popped} written with
//     atomicMax on the inverted rank (the lowest rank wins, newer rounds win), the popper's label
//     in a parallel array; an item recognises its own writes by its own rank.  Final items'
//     claims are promoted to one word {generation tag, popped, label} per pixel;
//   * commit (k_spec_flatten): the final executions of items 0..P-1 in rank order ARE the serial
//     pop sequence of the generation.  Flattened into "virtual items" (one per pop, with its
//     deferred pushes) they go through the batch engine's own ordered append (k_scan,
//     k_scatter), which keeps every bucket in exact serial FIFO order;
//   * a lane's cascade queue keeps its SPEC_QCAP smallest keys in LDS and spills the rest to a
//     chunk of the round's pool (cold keys, each larger than every LDS key); records past SPEC_RL
//     go to pool chunks too.  Only an execution beyond those chunks (SPEC_CCAP live entries,
//     SPEC_RL + SPEC_NX * SPEC_XCH records) while all its inputs are final ends the regime: the
//     prefix before it is committed and the batch engine pops that item and its cascade (serial
//     pops), after which the regime resumes (SpecCtl.block).
// scripts/exp/spec_rounds.c is the CPU prototype of exactly this scheme (bit-exact against the
// oracle on mosaic+noise, random and album frames; it also counts the rounds).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ws_shared.h"

namespace msg {

constexpr unsigned SPEC_RMAX = (1u << 22) - 1;
constexpr int SPEC_MINB = 2;  // blocks per CU the register budget allows (the LDS allows two)
constexpr int SPEC_RFW = 8;   // cold keys loaded together in a refill pass
constexpr int SPEC_HSW = 8;   // hot keys loaded together in a scan of a lane's LDS queue
static_assert(SPEC_QCAP % SPEC_HSW == 0, "hot-key scans read whole groups of SPEC_HSW entries");
static_assert(SPEC_NX == 4, "k_spec_round keeps SPEC_NX record chunk bases in four registers");

__device__ __forceinline__ unsigned long long spec_claim(unsigned tag, int rank, unsigned popped) {
  return ((unsigned long long)tag << 32) | ((unsigned long long)(SPEC_RMAX - (unsigned)rank) << 1) | popped;
}
__device__ __forceinline__ unsigned sc_tag(unsigned long long c) { return (unsigned)(c >> 32); }
__device__ __forceinline__ int sc_rank(unsigned long long c) {
  return (int)(SPEC_RMAX - (unsigned)((c >> 1) & SPEC_RMAX));
}
// Words written inside a round are read with agent-scope atomics (L2, never a stale L1 line).
__device__ __forceinline__ unsigned long long ld_ag64(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ld_ag32(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_ag64(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_ag32(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void claim_max(unsigned long long* p, unsigned long long k) {
  __hip_atomic_fetch_max(p, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// vm_drain (ws_kernels.hip): a pop's loads are waited for explicitly BEFORE the previous pop's
// claims, label and record are issued: the counter retires in issue order, and with those writes
// issued after the loads in branches some lanes (or the whole wave) skip, the compiler's own wait at
// the first use of a loaded value is vmcnt(0) behind the writes too -- their acknowledgements
// (atomics at the L2 or beyond) then sat on every pop's critical path.  Issued after the wait, the
// writes complete while the pop is decided and the next pop's loads are in flight.

__device__ __forceinline__ unsigned long long fin_word(unsigned G, unsigned popped, int lab) {
  return ((unsigned long long)G << 33) | ((unsigned long long)popped << 32) | (uint32_t)lab;
}
// generation log record: label | deferred-push mask | tiled pixel (< 2^28)
__device__ __forceinline__ unsigned long long srec_pack(int p, int lab, unsigned dm) {
  return ((unsigned long long)(uint32_t)lab << 32) | ((unsigned long long)dm << 28) | (unsigned)p;
}
__device__ __forceinline__ unsigned long long smix(unsigned long long h, unsigned long long v) {
  h ^= v + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2);
  return h * 0xff51afd7ed558ccdull;
}

// Record k of an execution: lane scratch, then the pool chunks xb0..xb3 (SPEC_XCH records each).
__device__ __forceinline__ unsigned long long* spec_rec_at(unsigned long long* tmp, unsigned long long* sxp, int k,
                                                           int xb0, int xb1, int xb2, int xb3) {
  if (k < SPEC_RL) return tmp + k;
  const int c = (k - SPEC_RL) / SPEC_XCH, o = (k - SPEC_RL) % SPEC_XCH;
  const int xb = c == 0 ? xb0 : c == 1 ? xb1 : c == 2 ? xb2 : xb3;
  return sxp + (size_t)xb + o;
}

struct SpecView {
  const SpecPx* spx;
  int par;          // this round's parity (T & 1): cl[par], lab[par]; the previous round's 1 - par
  unsigned T, G;
  bool hasprev;
};

// A pixel's record and state as loaded for spec_decide: relaxed agent-scope loads (sc1, L2-served,
// never a stale L1 line of words written inside this round) and no wait of their own, so a
// cascade pop issues all four neighbours' loads before the first use (volatile loads would put
// a full vmcnt(0) wait behind each one).
struct SpecRec {
  unsigned long long cl0, cl1, fin, labs;
  int s;
};
__device__ __forceinline__ SpecRec spec_load(const Ws& ws, const SpecView& V, int z) {
  SpecRec r;
  r.cl0 = ld_ag64(&V.spx[z].cl[0]);
  r.cl1 = ld_ag64(&V.spx[z].cl[1]);
  r.fin = ld_ag64(&V.spx[z].fin);
  r.labs = ld_ag64((const unsigned long long*)&V.spx[z].lab[0]);
  r.s = ws.mk[z];
  return r;
}

// The same record for the top pop's gather, before the item writes anything this round: plain
// loads (L1-cacheable, two 16-B loads).  A line cached before another wave's write of this round
// only hides words spec_decide ignores or reads equivalently: other items' round-T claims and
// labels are not used for a non-own view, and a final claim promoted this round equals that
// item's round T - 1 claim, which the view then takes instead.
__device__ __forceinline__ SpecRec spec_load_pre(const Ws& ws, const SpecView& V, int z) {
  const ulonglong2 a = *reinterpret_cast<const ulonglong2*>(&V.spx[z].cl[0]);
  const ulonglong2 b = *reinterpret_cast<const ulonglong2*>(&V.spx[z].fin);
  SpecRec r;
  r.cl0 = a.x;
  r.cl1 = a.y;
  r.fin = b.x;
  r.labs = b.y;
  r.s = ws.mk[z];
  return r;
}

// State of pixel z as item j sees it: > 0 label, WSHED, 0 unknown, INQ queued or pushed.
// Own writes first, then final items' writes, then the previous round's lower ranks, else the
// pre-generation state.
__device__ __forceinline__ int spec_decide(const SpecView& V, const SpecRec& r, int j, bool own) {
  const unsigned long long o = own ? (V.par ? r.cl1 : r.cl0) : 0ull;
  const int lc = (int)(uint32_t)(V.par ? (r.labs >> 32) : r.labs);
  const unsigned long long f = r.fin;
  const unsigned long long c = V.hasprev ? (V.par ? r.cl0 : r.cl1) : 0ull;
  const int lp = (int)(uint32_t)(V.par ? r.labs : (r.labs >> 32));
  if (own && sc_tag(o) == V.T && sc_rank(o) == j) return (o & 1ull) ? lc : INQ;
  if ((unsigned)(f >> 33) == V.G) return ((f >> 32) & 1ull) ? (int)(uint32_t)f : INQ;
  if (V.hasprev && sc_tag(c) == V.T - 1 && sc_rank(c) < j) return (c & 1ull) ? lp : INQ;
  return (r.s >= WSHED) ? r.s : INQ;
}

// a value per lane from five wave-uniform ones (lane 0: a0, ... lane 3: a3, others a4), as
// sequential selects (a chain of conditional expressions compiled to a branch tree)
__device__ __forceinline__ int lane_pick(int lane, int a0, int a1, int a2, int a3, int a4) {
  int r = a4;
  r = (lane == 3) ? a3 : r;
  r = (lane == 2) ? a2 : r;
  r = (lane == 1) ? a1 : r;
  r = (lane == 0) ? a0 : r;
  return r;
}

// spec_decide for an own view, as selects only (the cooperative pops run it on four lanes; its
// early returns compiled to a tree of exec-masked branches there)
__device__ __forceinline__ int spec_decide_own(const SpecView& V, const SpecRec& r, int j) {
  const unsigned long long o = V.par ? r.cl1 : r.cl0;
  const int lc = (int)(uint32_t)(V.par ? (r.labs >> 32) : r.labs);
  const unsigned long long f = r.fin;
  const unsigned long long c = V.par ? r.cl0 : r.cl1;
  const int lp = (int)(uint32_t)(V.par ? r.labs : (r.labs >> 32));
  const bool c1 = (int)(sc_tag(o) == V.T) & (int)(sc_rank(o) == j);  // (no short-circuit: no branches)
  const bool c2 = (unsigned)(f >> 33) == V.G;
  const bool c3 = (int)V.hasprev & (int)(sc_tag(c) == V.T - 1) & (int)(sc_rank(c) < j);
  const int v1 = (o & 1ull) ? lc : INQ;
  const int v2 = ((f >> 32) & 1ull) ? (int)(uint32_t)f : INQ;
  const int v3 = (c & 1ull) ? lp : INQ;
  const int v4 = (r.s >= WSHED) ? r.s : INQ;
  return c1 ? v1 : c2 ? v2 : c3 ? v3 : v4;
}

// the same for another item's view (the top pop's gather): final claims, the previous round's, state
__device__ __forceinline__ int spec_decide_other(const SpecView& V, const SpecRec& r, int j) {
  const unsigned long long f = r.fin;
  const unsigned long long c = V.par ? r.cl0 : r.cl1;
  const int lp = (int)(uint32_t)(V.par ? r.labs : (r.labs >> 32));
  const bool c2 = (unsigned)(f >> 33) == V.G;
  const bool c3 = (int)V.hasprev & (int)(sc_tag(c) == V.T - 1) & (int)(sc_rank(c) < j);
  const int v2 = ((f >> 32) & 1ull) ? (int)(uint32_t)f : INQ;
  const int v3 = (c & 1ull) ? lp : INQ;
  const int v4 = (r.s >= WSHED) ? r.s : INQ;
  return c2 ? v2 : c3 ? v3 : v4;
}

// top-pop granule of item k as item j may use it in round T: this round's, or a final item's.
// Word: label | round tag << 32 | (label differs from item k's previous round) << 63; chg
// collects that bit of the non-final items read (an input of the reader changed).
constexpr unsigned long long SPEC_GDIFF = 1ull << 63;
__device__ __forceinline__ bool spec_granule(const Ws& ws, int k, int P, unsigned T, unsigned G, int& v, bool& chg) {
  const unsigned long long g = ld_ag64(ws.stl + k);
  const unsigned tg = (unsigned)(g >> 32) & 0x7fffffffu;
  if (tg == T || (k < P && tg >= G && tg <= T)) {
    v = (int)(uint32_t)g;
    if (k >= P && (g & SPEC_GDIFF)) chg = true;
    return true;
  }
  return false;
}

// Replay (round T >= G + 2): item j's top pop came out as in round T - 1 (same record, no changed
// granule read) and no pixel its previous cascade viewed -- the neighbours of its pops -- was
// marked in round T - 1 (a claim of a changed execution, old or new): its inputs are those of
// round T - 1, so its cascade is that round's, replayed from the log without the dependent
// round trip per pop.  Checks first (all loads independent), then the claims.
__device__ __forceinline__ bool spec_replay_clean(const Ws& ws, int base, int nrec, int ppar, unsigned T,
                                                  const int* nbp) {
  const unsigned* const dirt = ws.sdirt + (size_t)ppar * ws.snp;
  const unsigned tp = T - 1u;
  bool dirty = false;
#pragma unroll
  for (int d = 0; d < 4; ++d) dirty |= dirt[nbp[d]] == tp;
  const int Wt = ws.Wt, marg = ws.marg;
  for (int k0 = 1; k0 < nrec && !dirty; k0 += 4) {
    unsigned long long r[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) r[k] = (k0 + k < nrec) ? ws.slog[base + k0 + k] : 0ull;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (k0 + k >= nrec) continue;
      const int yb = (int)(r[k] & 0x0fffffffu) + marg;
#pragma unroll
      for (int d = 0; d < 4; ++d) dirty |= dirt[nbi(yb, d, Wt) - marg] == tp;
    }
  }
  return !dirty;
}

// End of a round (last block): grow the stable prefix, or hand the generation to the commit.
__device__ void spec_finalize(Ctl* ctl, int P, int n, unsigned T, unsigned G, unsigned long long* dg) {
  SpecCtl& s = ctl->spec;
  if (dg) {  // diagnostics: sums over rounds of the round's longest wave and of its split
    const unsigned long long k = __hip_atomic_load(&s.rmax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    dg[5] += k >> 40;              // its lifetime
    dg[4] += (k >> 20) & 0xfffffu; // its waits for earlier items' top pops
    dg[6] += k & 0xfffffu;         // its top-pop writes + cascades
    const unsigned long long k2 = __hip_atomic_load(&s.rmax2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    dg[0] += (k2 >> 20) & 0xfffffu;  // its cascades run wave-cooperatively (spec_coop)
    dg[1] += k2 & 0xfffffu;          // its log copy, change marks, candidates
    s.rmax = 0;
    s.rmax2 = 0;
  }
  // written by this kernel's atomics: read at L2, not through a line cached at kernel start
  const int fc = __hip_atomic_load(&ctl->sfc.v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int ov = __hip_atomic_load(&ctl->sovf.v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int newP = min(fc, n);
  s.rounds_total += 1;
  s.xlong += __hip_atomic_load(&s.rxmax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  s.rxmax = 0;
  s.ov2 = s.ov1;
  s.ov1 = ov;
  if (newP >= n) {
    s.Pprom = P;
    s.P = n;
    s.state = 2;
  } else if ((newP == P && T > G && ov == newP) || (s.rounds >= SPEC_ROUNDS_MAX && newP == 0)) {
    // item newP read only final inputs and still overflowed: commit the prefix, pop it serially
    s.Pprom = P;
    s.P = newP;
    s.state = 2;
    s.fallback = 1;
  } else if (s.rounds >= SPEC_ROUNDS_MAX) {
    s.Pprom = P;
    s.P = newP;
    s.state = 2;
  } else {
    s.Pold = P;
    s.P = newP;
    s.T = T + 1;
    s.rounds += 1;
    ctl->sdeal.v = P;
    ctl->sfc.v = NONE;
    ctl->sovf.v = NONE;
    ctl->sxtop.v = 0;  // every execution of this round has copied its records to the log
  }
  s.ticket = 0;
}

// ---------------------------------------------------------------------------------------------
// Wave-cooperative cascades (round 5).  A round lasts as long as its longest execution, and that
// execution is usually one lane's long cascade running alone in its wave after the other 63
// lanes' executions ended: round 4 measured ~7000 wave cycles per lone-lane cascade pop (a serial
// scan of the lane's 32 hot keys, four neighbour records decided one after another, the claims and
// the record written by one lane), against one dependent memory round trip that a pop needs.
// When a single lane of the wave is left with a cascade, the whole wave takes its execution over
// and finishes it with the SAME pop sequence -- the cascade's serial order (lowest level first,
// FIFO within a level) is a property of the keys, not of who pops them:
//   * queue: the wave's 64 LDS columns (the per-lane queues of the finished lanes, 2048 slots)
//     hold the hot entries {ord = level << 16 | push sequence, pixel}, any lane's column, each
//     lane tracking its column's smallest ord; the next pop is a DPP wave minimum over those, and
//     the popped column's new minimum is found by the wave in parallel while the pop's loads are
//     in flight.  Cold keys stay in the execution's pool chunk (every cold key larger than every
//     hot one, as in the per-lane queue); an empty hot set takes every cold key up to the largest
//     level that fits back in one parallel pass (level histogram in LDS, then a scatter);
//   * a pop: lanes 0-3 load and decide one neighbour each (the same spec_decide, patched with the
//     previous pop's writes, which are issued after these loads exactly as in the per-lane loop),
//     the fold and the pushes are uniform, and the claims, label and record go out as one masked
//     instruction each;
//   * capacities: 2048 hot entries (more: a capacity overflow, as a lane's 32 + 4096), the cold
//     chunk and the record chunks exactly as in the per-lane loop, and the same length caps.
// The execution's results (records, signature, overflow flags, record chunks) land where the
// per-lane loop leaves them, so the rest of the round does not know which form ran it.
constexpr int COOP_HOT = SPEC_QCAP * 64;  // hot slots of a cooperating wave (its LDS columns)
constexpr int COOP_LANES = 2;             // the wave takes cascades over once this few lanes are left
constexpr int COOP_MAXORD = 0x7fffffff;
static_assert(4 * SPEC_MAXREC < (1 << 16), "an execution's push sequence fits the 16 bits of a coop ord");

struct CoopSt {
  int y;                      // the pop selected next (already out of the queue)
  int py, plab;               // the previous pop: pixel, label, pushes (for the patch) ...
  unsigned ppm;
  int pz0, pz1, pz2, pz3;
  unsigned long long prec;    // ... its record, and whether its writes are still to be issued
  bool pwrite;
  int nrec;
  unsigned long long sig;
  unsigned qseq;
  int nq;                     // hot keys in the owner's LDS column (per-lane format), at entry
  int nc, cb;                 // cold keys in the pool chunk cb (-1 none yet, -2 pool full)
  unsigned cmin;
  int xb0, xb1, xb2, xb3;     // record chunks past SPEC_RL
  bool ovf, cap;
};

// lq: the block's per-lane queues ([entry][thread]); wb: the wave's first thread; w: the owner lane.
__device__ __forceinline__ void spec_coop(const Ws& ws, const SpecView& V, unsigned long long* lq, int wb,
                                                    int w, int j, int L, bool longok, unsigned long long* tmp,
                                                    CoopSt& S) {
  Ctl* const ctl = ws.ctl;
  const int lane = lane_id();
  const int Wt = ws.Wt, marg = ws.marg;
  const unsigned T = V.T;
  const int par = V.par;
  SpecPx* const spx = const_cast<SpecPx*>(V.spx);
  unsigned long long* const col = lq + wb + lane;  // this lane's column: entry e at col[e * SPEC_BS]
  auto pool_get = [&](int sz) -> int {             // lane 0 asks, the wave gets the answer
    int b = -1;
    if (lane == 0 && ld_ag32(&ctl->sxtop.v) < ws.sxcap) {
      b = atomicAdd(&ctl->sxtop.v, sz);
      if (b < 0 || (long long)b + sz > ws.sxcap) b = -1;
    }
    return __builtin_amdgcn_readlane(b, 0);
  };
  // ---- entry: the owner's hot keys become coop entries, one per lane (lane e takes row e) ----
  int cnt = 0, m1 = COOP_MAXORD, m1row = 0, m1pix = 0;
  {
    const unsigned long long k = (lane < S.nq) ? lq[(size_t)lane * SPEC_BS + wb + w] : 0ull;
    if (lane < S.nq) {
      const int ord = (int)(((k >> 52) << 16) | ((k >> 28) & 0xffffu));
      m1pix = (int)(k & 0x0fffffffu);
      col[0] = ((unsigned long long)(unsigned)ord << 32) | (unsigned)m1pix;
      cnt = 1;
      m1 = ord;
    }
  }
  int H = S.nq, rr = S.nq & 63;
  int fix = -1;  // a column whose minimum was popped: refilled hole + new minimum still to be found
  auto rec_at = [&](int k) { return spec_rec_at(tmp, ws.sxp, k, S.xb0, S.xb1, S.xb2, S.xb3); };
  auto cold_add = [&](unsigned t, int pix, unsigned seq) {
    if (S.cb == -2 || S.nc >= SPEC_CCAP) {
      S.ovf = S.cap = true;
      return;
    }
    if (S.cb < 0 && (S.cb = pool_get(SPEC_CCAP)) < 0) {
      S.cb = -2;
      S.ovf = S.cap = true;
      return;
    }
    if (lane == 0)
      ws.sxp[(size_t)S.cb + S.nc] =
          ((unsigned long long)t << 52) | ((unsigned long long)(seq & 0xffffffu) << 28) | (unsigned)pix;
    ++S.nc;
    S.cmin = min(S.cmin, t);
  };
  auto qpush = [&](unsigned t, int pix) {
    const unsigned seq = S.qseq++;
    if (S.nc > 0 && t >= S.cmin) {  // above the smallest cold key: cold too
      cold_add(t, pix, seq);
      return;
    }
    if (H >= COOP_HOT) {
      S.ovf = S.cap = true;
      return;
    }
    // the next column with room, round robin from rr
    const unsigned long long room = __ballot(cnt < SPEC_QCAP);
    const unsigned long long hi = room & (~0ull << rr);
    const int tl = hi ? __builtin_ctzll(hi) : __builtin_ctzll(room);
    const int ord = (int)((t << 16) | (seq & 0xffffu));
    if (lane == tl) {
      col[(size_t)cnt * SPEC_BS] = ((unsigned long long)(unsigned)ord << 32) | (unsigned)pix;
      if (ord < m1) {
        m1 = ord;
        m1row = cnt;
        m1pix = pix;
      }
      ++cnt;
    }
    ++H;
    rr = (tl + 1) & 63;
  };
  // hot empty, cold not: every cold key up to the largest level whose count still fits the hot
  // slots moves hot (the rest stay cold: all larger than every hot key)
  auto refill = [&]() {
    unsigned* const hb = reinterpret_cast<unsigned*>(lq);  // 256 level bins in rows 0-1 of the columns
    auto bin = [&](int b) -> unsigned* { return hb + ((size_t)(b >> 7) * SPEC_BS + wb) * 2 + (b & 127); };
#pragma unroll
    for (int k = 0; k < 4; ++k) *bin(4 * lane + k) = 0u;
    const size_t cb = (size_t)S.cb;
    for (int b0 = 0; b0 < S.nc; b0 += 64) {
      if (b0 + lane < S.nc) atomicAdd(bin((int)(ws.sxp[cb + b0 + lane] >> 52)), 1u);
    }
    int h[4], s4 = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      h[k] = (int)*bin(4 * lane + k);
      s4 += h[k];
    }
    int c = wave_scan_add(s4) - s4;  // keys below level 4 * lane
    int best = -1, movc = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      c += h[k];
      if (c <= COOP_HOT) {
        best = 4 * lane + k;
        movc = c;
      }
    }
    const int vstar = -wave_min(-best);  // the largest level whose cumulative count fits
    const unsigned long long bw = __ballot(best == vstar);
    const int M = __builtin_amdgcn_readlane(movc, __builtin_ctzll(bw));
    if (vstar < (int)S.cmin || M == 0) {  // the lowest cold level alone is larger than the hot slots
      S.ovf = S.cap = true;
      return;
    }
    int moved = 0, kept = 0;
    unsigned ncmin = 256;
    for (int b0 = 0; b0 < S.nc; b0 += 64) {
      const bool valid = b0 + lane < S.nc;
      const unsigned long long k = valid ? ws.sxp[cb + b0 + lane] : 0ull;
      const unsigned lv = (unsigned)(k >> 52);
      const bool mv = valid && (int)lv <= vstar, kp = valid && !mv;
      const unsigned long long bm = __ballot(mv), bk = __ballot(kp);
      if (mv) {
        const int pos = moved + lanes_below(bm);
        const int ord = (int)((lv << 16) | ((k >> 28) & 0xffffu));
        lq[(size_t)(pos >> 6) * SPEC_BS + wb + (pos & 63)] =
            ((unsigned long long)(unsigned)ord << 32) | (unsigned)(k & 0x0fffffffu);
      }
      if (kp) {
        ws.sxp[cb + kept + lanes_below(bk)] = k;
        ncmin = min(ncmin, lv);
      }
      moved += __popcll(bm);
      kept += __popcll(bk);
    }
    S.nc = kept;
    S.cmin = (unsigned)wave_min((int)ncmin);
    H = moved;
    cnt = (moved >> 6) + (lane < (moved & 63) ? 1 : 0);
    rr = moved & 63;
    m1 = COOP_MAXORD;
    for (int e = 0; e < cnt; ++e) {
      const unsigned long long x = col[(size_t)e * SPEC_BS];
      if ((int)(x >> 32) < m1) {
        m1 = (int)(x >> 32);
        m1row = e;
        m1pix = (int)(unsigned)x;
      }
    }
  };
  // the previous pop's claims (lane 0 its pixel, lanes 1-4 its pushes), label and record, one
  // masked instruction each
  auto coop_writes = [&]() {
    const int za = lane_pick(lane, S.py, S.pz0, S.pz1, S.pz2, S.pz3);
    const bool cl = lane == 0 || (lane <= 4 && ((S.ppm >> ((lane - 1) & 3)) & 1u));
    const unsigned long long cv = spec_claim(T, j, lane == 0 ? 1u : 0u);
    if (cl) claim_max(&spx[za].cl[par], cv);
    if (lane == 5) st_ag32(&spx[S.py].lab[par], S.plab);
    if (lane == 6) *rec_at(S.nrec - 1) = S.prec;
    S.pwrite = false;
  };
  int y = S.y;
#ifdef MSEG_SPEC_PROF
  const long long c_t0 = (long long)__builtin_amdgcn_s_memtime();
  const int c_n0 = S.nrec;
#endif
#ifdef MSEG_SPEC_PROF
  long long cp0 = 0, cp1 = 0, cp2 = 0, cp3 = 0, cp4 = 0, cta = 0, ctb = 0;
#define CP_T(v) v = (long long)__builtin_amdgcn_s_memtime()
#else
#define CP_T(v) do { } while (0)
#endif
  for (;;) {
    // ---- the length caps and the record chunk of pop nrec, as at the per-lane loop's head ----
    if (S.nrec >= (longok ? SPEC_MAXREC : SPEC_MAXREC_SHORT)) {
      S.ovf = S.cap = true;
      break;
    }
    if (S.nrec >= SPEC_RL && (S.nrec - SPEC_RL) % SPEC_XCH == 0) {
      const int c = (S.nrec - SPEC_RL) / SPEC_XCH;
      const int b = c < SPEC_NX ? pool_get(SPEC_XCH) : -1;
      if (b < 0) {
        S.ovf = S.cap = true;
        break;
      }
      if (c == 0) S.xb0 = b;
      else if (c == 1) S.xb1 = b;
      else if (c == 2) S.xb2 = b;
      else S.xb3 = b;
    }
    CP_T(cta);
    // ---- the pop of y: its loads (lanes 0-3 one neighbour each), then the previous pop's writes ----
    const int yb = y + marg;
    int nb[4];  // uniform: scalar arithmetic, then one lane per direction
#pragma unroll
    for (int d = 0; d < 4; ++d) nb[d] = __builtin_amdgcn_readfirstlane(nbi(yb, d, Wt) - marg);
    const int nbd = lane_pick(lane, nb[0], nb[1], nb[2], nb[3], nb[3]);  // lane d: direction d
    // every lane loads (lanes 4-63 repeat lane 3's addresses: the same requests), so that no
    // branch puts the use of the loaded values -- and the wait for them -- before the hole fix
    const unsigned wyl = (unsigned)ws.w4[y];
    const SpecRec r = spec_load(ws, V, nbd);
    if (fix >= 0) {  // the column the last select popped from: fill its hole, find its new minimum
      if (lane == fix) {  // the last entry moves into the hole (itself when it was the last)
        --cnt;
        col[(size_t)m1row * SPEC_BS] = col[(size_t)cnt * SPEC_BS];
      }
      const int co = __builtin_amdgcn_readlane(cnt, fix);
      const unsigned long long x = lq[(size_t)(lane & (SPEC_QCAP - 1)) * SPEC_BS + wb + fix];
      const int ord = (lane < co) ? (int)(x >> 32) : COOP_MAXORD;
      const int mo = wave_min(ord);
      const unsigned long long bo = __ballot(lane < co && ord == mo);
      const int row = bo ? __builtin_ctzll(bo) : 0;
      const int pixo = __builtin_amdgcn_readlane((int)(unsigned)x, row);
      if (lane == fix) {
        m1 = co > 0 ? mo : COOP_MAXORD;
        m1row = row;
        m1pix = pixo;
      }
      fix = -1;
    }
#ifdef MSEG_SPEC_PROF
    CP_T(ctb);
    cp0 += ctb - cta;
#endif
    vm_drain();
#ifdef MSEG_SPEC_PROF
    CP_T(cta);
    cp1 += cta - ctb;
#endif
    if (S.pwrite) coop_writes();
    // ---- decide: lanes 0-3, patched with the previous pop's writes (issued after these loads) ----
    int v = 0;
    {
      v = spec_decide_own(V, r, j);
      v = (nbd == S.py) ? S.plab : v;
      const bool inq = (((S.ppm & 1u) != 0) & (nbd == S.pz0)) | (((S.ppm & 2u) != 0) & (nbd == S.pz1)) |
                       (((S.ppm & 4u) != 0) & (nbd == S.pz2)) | (((S.ppm & 8u) != 0) & (nbd == S.pz3));
      v = inq ? INQ : v;
    }
    const unsigned wy = (unsigned)__builtin_amdgcn_readfirstlane((int)wyl);
    int vd[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) vd[d] = __builtin_amdgcn_readlane(v, d);
    int lab = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d)
      if (vd[d] > 0) lab = fold_lab(lab, vd[d]);
    if (lab == 0) {  // own writes hidden by a conflicting lower rank: unstable
      S.ovf = true;
      lab = WSHED;
    }
#ifdef MSEG_SPEC_PROF
    CP_T(ctb);
    cp2 += ctb - cta;
#endif
    unsigned dmy = 0, pmy = 0;
    if (lab != WSHED) {
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        if (vd[d] != 0) continue;
        pmy |= 1u << d;
        const unsigned t = (wy >> (8 * d)) & 255u;
        if ((int)t < L) qpush(t, nb[d]);
        else dmy |= 1u << d;
      }
    }
#ifdef MSEG_SPEC_PROF
    CP_T(cta);
    cp3 += cta - ctb;
#endif
    S.prec = srec_pack(y, lab, dmy);
    S.sig = smix(S.sig, S.prec);
    S.py = y;
    S.plab = lab;
    S.ppm = pmy;
    S.pz0 = nb[0];
    S.pz1 = nb[1];
    S.pz2 = nb[2];
    S.pz3 = nb[3];
    S.pwrite = true;
    ++S.nrec;
    if (S.ovf || H + S.nc == 0) break;
    // ---- select: the smallest ord of all columns ----
    if (H == 0) {
      refill();
      if (S.ovf) break;
    }
    const int m = wave_min(m1);
    fix = __builtin_ctzll(__ballot(m1 == m));
    y = __builtin_amdgcn_readlane(m1pix, fix);
    --H;
    // the loop-carried state is wave-uniform: say so, so that the loop's branches stay scalar
    H = __builtin_amdgcn_readfirstlane(H);
    rr = __builtin_amdgcn_readfirstlane(rr);
    S.nrec = __builtin_amdgcn_readfirstlane(S.nrec);
    S.nc = __builtin_amdgcn_readfirstlane(S.nc);
    S.cb = __builtin_amdgcn_readfirstlane(S.cb);
    S.cmin = (unsigned)__builtin_amdgcn_readfirstlane((int)S.cmin);
    S.qseq = (unsigned)__builtin_amdgcn_readfirstlane((int)S.qseq);
    S.ovf = __builtin_amdgcn_readfirstlane((int)S.ovf) != 0;
    S.cap = __builtin_amdgcn_readfirstlane((int)S.cap) != 0;
#ifdef MSEG_SPEC_PROF
    CP_T(ctb);
    cp4 += ctb - cta;
#endif
  }
#undef CP_T
#ifdef MSEG_SPEC_PROF
  if (ws.diag && lane == 0) {  // bank 3: the cooperative pop's phases (cycles)
    atomicAdd(&ws.diag[24], (unsigned long long)cp0);
    atomicAdd(&ws.diag[25], (unsigned long long)cp1);
    atomicAdd(&ws.diag[26], (unsigned long long)cp2);
    atomicAdd(&ws.diag[27], (unsigned long long)cp3);
    atomicAdd(&ws.diag[28], (unsigned long long)cp4);
  }
#endif
  if (S.pwrite) coop_writes();  // the last pop's
#ifdef MSEG_SPEC_PROF
  if (ws.diag && lane == 0) {  // bank 2: cooperative pops, their cycles
    atomicAdd(&ws.diag[21], (unsigned long long)(S.nrec - c_n0));
    atomicAdd(&ws.diag[22], (unsigned long long)((long long)__builtin_amdgcn_s_memtime() - c_t0));
  }
#endif
}

// One round.  Waves take 64 consecutive ranks at a time from [Pold, n) in dispatch order:
// [Pold, P) promote their claims, [P, n) execute.
__global__ __launch_bounds__(SPEC_BS, SPEC_MINB) void k_spec_round(Ws ws) {
  Ctl* ctl = ws.ctl;
  if (ctl->bat.mode != 3 || ctl->spec.state != 1 || ctl->error) return;
  __shared__ unsigned long long lq[SPEC_QCAP * SPEC_BS];  // per-lane cascade queues, [entry][lane]
  __shared__ int s_exec, s_rep, s_xpop;
  const int tid = threadIdx.x, lane = lane_id();
  if (tid == 0) s_exec = s_rep = s_xpop = 0;
  const unsigned T = ctl->spec.T, G = ctl->spec.G;
  const int P = ctl->spec.P, n = ctl->spec.n, L = ctl->spec.L, bstart = ctl->spec.bstart;
  // An execution may run SPEC_MAXREC_SHORT pops (a lane's cascade pop costs several times a
  // serial pop, so a long cascade is cheaper as serial pops).  But a fallback restarts the rest of
  // the bucket as a new generation; where long cascades are everywhere (uniform noise at 4096^2:
  // invasion-percolation avalanches of thousands of pops) those re-runs and the regime's
  // cooldowns cost far more than slow lanes.  So the stable prefix's head (its inputs final, it
  // runs once more at most) may always run SPEC_MAXREC pops, and every execution from round 2 on
  // may too once the flood is in deep mode (SpecCtl.deep: a cooldown after large generations).
  // Round 4 A/B'd six such policies (profiles/r04v_ab_deep_mode.log); this one won.
  const bool lcap = ctl->spec.deep == 1;
  const int par = (int)(T & 1u), ppar = (int)((T - 1u) & 1u);
  // replays need complete change marks: no overflowing execution (claims never logged in full)
  // below the item in the last two rounds
  const int ovlim = min(ctl->spec.ov1, ctl->spec.ov2);
  int nrep = 0, nxpop = 0;  // this lane's replayed executions; pops it ran pop by pop
  SpecView V;
  V.spx = ws.spx;
  V.par = par;
  V.T = T;
  V.G = G;
  V.hasprev = T > G;
  SpecPx* const spx = ws.spx;
  unsigned long long* const tmp = ws.stmp + (size_t)(blockIdx.x * SPEC_BS + tid) * SPEC_RL;
  const unsigned long long etag = (unsigned long long)T << 32;
  const int Wt = ws.Wt, marg = ws.marg;
  bool stop = false;
#ifdef MSEG_SPEC_PROF
  long long pf_n = 0, pf_q = 0, pf_sel = 0, pf_load = 0, pf_write = 0;  // cascade-pop phases (lane sums)
#endif
  unsigned long long* const dg = ws.diag ? ws.diag + 8 : nullptr;  // msg_set_diag: the round's wall-clock split (10 ns ticks)
  const long long tk0 = dg ? (long long)__builtin_amdgcn_s_memrealtime() : 0;
  long long tw = 0, tc = 0, tco = 0, tpo = 0;  // diag: waits, cascades (cooperative part), post
  __syncthreads();
  while (!stop) {
    const long long tq0 = dg ? (long long)__builtin_amdgcn_s_memrealtime() : 0;
    int r0 = 0;
    // (pre-checking the word with a load before the atomic, sharding the log counter per
    // blockIdx % 8 and skipping rank-minimum atomics already beaten measured 26% slower)
    if (lane == 0) r0 = atomicAdd(&ctl->sdeal.v, 64);
    r0 = __builtin_amdgcn_readlane(r0, 0);
    if (r0 >= n) break;
    const int j = r0 + lane;
    // ---- promote: final since the last round; their claims become permanent ----
    if (j < P) {
      const int4 r4 = ws.srec[(size_t)ppar * SPEC_WIN + j];
      const int2 rc = make_int2(r4.x, r4.y);
      ws.sfrec[j] = rc;
      for (int k = 0; k < rc.y; ++k) {
        const unsigned long long r = ws.slog[rc.x + k];
        const int y = (int)(r & 0x0fffffffu);
        const unsigned dm = (unsigned)(r >> 28) & 15u;
        st_ag64(&ws.spx[y].fin, fin_word(G, 1u, (int)(uint32_t)(r >> 32)));
#pragma unroll
        for (int d = 0; d < 4; ++d)
          if ((dm >> d) & 1u) st_ag64(&ws.spx[nbi(y + marg, d, Wt) - marg].fin, fin_word(G, 0u, 0));
      }
    }
    (void)tq0;
    // ---- execute [P, n): gather the top pop ----
    const bool ex = j >= P && j < n;
    int p = 0;
    unsigned wp = 0, zm = 0;
    int nbp[4] = {0, 0, 0, 0}, dep[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) dep[k] = -1;
    int base_lab = 0;
    unsigned long long gold = 0;
    if (ex) {
      gold = ld_ag64(ws.stl + j);
      p = ws.qbuf[bstart + j];
      wp = (unsigned)ws.w4[p];
      const int pb = p + marg;
#pragma unroll
      for (int d = 0; d < 4; ++d) nbp[d] = nbi(pb, d, Wt) - marg;
      SpecRec rr[4];  // all four records in flight before the first decision
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        rr[d] = spec_load_pre(ws, V, nbp[d]);
      }
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        if (rr[d].s <= -3) {  // an earlier item of this generation: its top pop of this round
          const int k = state_slot(rr[d].s) - bstart;
          if (k >= 0 && k < j) {
            dep[d] = k;
            continue;
          }
        }
        const int v = spec_decide_other(V, rr[d], j);
        if (v > 0) base_lab = fold_lab(base_lab, v);
        else if (v == 0) zm |= 1u << d;
      }
      if (base_lab != WSHED) {  // competitors for the unknown neighbours: earlier adjacent items
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          if (!((zm >> d) & 1u)) continue;
          const int zb = nbp[d] + marg;
          const int ee[3] = {(d == 1) ? 1 : 0, (d <= 1) ? 2 : 1, (d == 2) ? 2 : 3};
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            const int sz = ws.mk[nbi(zb, ee[k], Wt) - marg];
            if (sz <= -3) {
              const int r = state_slot(sz) - bstart;
              if (r >= 0 && r < j) dep[4 + 3 * d + k] = r;
            }
          }
        }
      }
    }
    const long long tka = dg ? (long long)__builtin_amdgcn_s_memrealtime() : 0;
    // ---- wait for the earlier adjacent top pops of this round (lower ranks only) ----
    bool labd = !ex, pushd = !ex;
    int mylab = 0;
    unsigned pm = 0;
    bool ovf = false, cap = false;  // unstable; capacity overflow
    bool gchg = T < G + 2u;         // a granule input changed since round T - 1 (or unknown)
    long long t0 = 0;
    int spins = 0;
    for (;;) {
      if (!labd) {
        int lab = base_lab;
        bool unk = false;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          if (dep[d] < 0) continue;
          int v;
          if (spec_granule(ws, dep[d], P, T, G, v, gchg)) {
            if (v > 0) lab = fold_lab(lab, v);
          } else {
            unk = true;
          }
        }
        if (lab == WSHED || !unk) {
          if (lab == 0) {  // cannot happen for a queued pixel; unstable, never committed
            ovf = true;
            lab = WSHED;
          }
          mylab = lab;
          labd = true;
          if (unk) gchg = true;
          const bool same = T > G && (unsigned)(gold >> 32 & 0x7fffffffu) == T - 1u && (int)(uint32_t)gold == lab;
          st_ag64(ws.stl + j, etag | (uint32_t)lab | (same ? 0ull : SPEC_GDIFF));
        }
      }
      if (labd && !pushd) {
        if (mylab == WSHED) {
          pushd = true;
        } else {
          bool und = false;
          unsigned m = 0;
#pragma unroll
          for (int d = 0; d < 4; ++d) {
            if (!((zm >> d) & 1u)) continue;
            bool lose = false, u = false;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
              const int r = dep[4 + 3 * d + k];
              if (r < 0) continue;
              int v;
              if (spec_granule(ws, r, P, T, G, v, gchg)) {
                if (v > 0) lose = true;  // that item pushed the neighbour first
              } else {
                u = true;
              }
            }
            if (!lose) {
              if (u) und = true;
              else m |= 1u << d;
            } else if (u) {
              gchg = true;
            }
          }
          if (!und) {
            pm = m;
            pushd = true;
          }
        }
      }
      if (!__any(!pushd)) break;
      if (++spins > 16) {
        __builtin_amdgcn_s_sleep(1);
        if (ld_ag32(&ctl->error)) {
          stop = true;
          break;
        }
        const long long now = (long long)__builtin_amdgcn_s_memrealtime();
        if (t0 == 0) {
          t0 = now;
        } else if (now - t0 > SPIN_LIMIT_TICKS) {
          if (!pushd) atomicOr(&ctl->error, ERR_TIMEOUT);
          stop = true;
          break;
        }
      }
    }
    if (stop) break;
    const long long tkb = dg ? (long long)__builtin_amdgcn_s_memrealtime() : 0;
    unsigned long long sig = 0;
    int nrec = 0;
    int rbase = -1;  // >= 0: the cascade was replayed from the previous round's log records here
    int xb0 = -1, xb1 = -1, xb2 = -1, xb3 = -1;  // record chunks past SPEC_RL (SPEC_NX = 4)
#define rec_at(k) spec_rec_at(tmp, ws.sxp, (k), xb0, xb1, xb2, xb3)
    {
      // ---- the top pop, then the cascade (levels < L, lowest first, FIFO) ----
      // Every pop's writes (claims, label, record) are issued AFTER the loads of the next pop's
      // neighbours have completed (vm_drain): the wave's memory counter retires in issue order, so
      // a load issued behind stores waits for their acknowledgements too.  The next pop therefore
      // sees its predecessor's writes through a patch (that pop's pixel and pushes) instead of
      // memory; everything older was issued before its loads.
      // The lane's cascade queue: keys {level, push sequence, pixel} (the serial order of a
      // cascade is the key order: lowest level first, FIFO within a level).  The SPEC_QCAP
      // smallest live keys are "hot" in LDS; the rest are "cold" in a chunk of the round's pool,
      // every cold key larger than every hot one.
      int nq = 0, nc = 0;   // hot / cold keys
      int cb = -1;          // cold chunk in ws.sxp (-2: the pool was full, never asked again)
      unsigned cmin = 256;  // lowest level among the cold keys
      unsigned long long hmx = 0;  // largest hot key (pops take the smallest: it stays valid)
      unsigned qseq = 0;    // pushes of this execution
      // a chunk of sz entries of the round's pool, or -1 once it is full.  The counter is only
      // bumped while it is below the pool's size, so it stays far from 2^31 (at most one chunk per
      // lane in flight past the end), and a negative offset is refused regardless
      auto pool_get = [&](int sz) -> int {
        if (ld_ag32(&ctl->sxtop.v) >= ws.sxcap) return -1;
        const int b = atomicAdd(&ctl->sxtop.v, sz);
        return (b >= 0 && (long long)b + sz <= ws.sxcap) ? b : -1;
      };
      auto cold_add = [&](unsigned long long k) {
        if (cb == -2) {
          ovf = cap = true;
          return;
        }
        if (cb < 0 && (cb = pool_get(SPEC_CCAP)) < 0) {
          cb = -2;
          ovf = cap = true;
          return;
        }
        if (nc >= SPEC_CCAP) {
          ovf = cap = true;
          return;
        }
        ws.sxp[(size_t)cb + nc++] = k;
        cmin = min(cmin, (unsigned)(k >> 52));
      };
      auto qpush = [&](unsigned t, int pix) {
        const unsigned long long k =
            ((unsigned long long)t << 52) | ((unsigned long long)(qseq++ & 0xffffffu) << 28) | (unsigned)pix;
        if (nc > 0 && t >= cmin) {  // above the smallest cold key: cold too
          cold_add(k);
          return;
        }
        if (nq < SPEC_QCAP) {
          lq[(nq++) * SPEC_BS + tid] = k;
          hmx = max(hmx, k);
          return;
        }
        if (k > hmx) {  // hot is full: the larger of k and the largest hot key goes cold
          cold_add(k);
          return;
        }
        // one pass: where the largest hot key is, and the largest of the others (keys are unique)
        int mi = 0;
        unsigned long long h2 = k;
        #pragma unroll 1
        for (int k0 = 0; k0 < SPEC_QCAP; k0 += SPEC_HSW) {
          unsigned long long e[SPEC_HSW];
  #pragma unroll
          for (int i = 0; i < SPEC_HSW; ++i) e[i] = lq[(k0 + i) * SPEC_BS + tid];
  #pragma unroll
          for (int i = 0; i < SPEC_HSW; ++i) {
            if (e[i] == hmx) mi = k0 + i;
            else h2 = max(h2, e[i]);
          }
        }
        cold_add(hmx);
        lq[mi * SPEC_BS + tid] = k;
        hmx = h2;
      };
      // hot empty, cold not: the SPEC_QCAP smallest cold keys become hot (one pass keeping the
      // smallest seen, one pass compacting the rest in place)
      auto refill = [&]() {
        const size_t b = (size_t)cb;
        unsigned long long hmax = 0;
        int hmi = 0;
        #pragma unroll 1
        for (int k0 = 0; k0 < nc; k0 += SPEC_RFW) {
          unsigned long long v[SPEC_RFW];
  #pragma unroll
          for (int k = 0; k < SPEC_RFW; ++k) v[k] = (k0 + k < nc) ? ws.sxp[b + k0 + k] : 0ull;
  #pragma unroll
          for (int k = 0; k < SPEC_RFW; ++k) {
            if (k0 + k >= nc) continue;
            if (nq < SPEC_QCAP) {
              lq[nq * SPEC_BS + tid] = v[k];
              if (v[k] > hmax) {
                hmax = v[k];
                hmi = nq;
              }
              ++nq;
            } else if (v[k] < hmax) {
              lq[hmi * SPEC_BS + tid] = v[k];
              hmax = 0;
              #pragma unroll 1
              for (int e0 = 0; e0 < SPEC_QCAP; e0 += SPEC_HSW) {
                unsigned long long u[SPEC_HSW];
  #pragma unroll
                for (int i = 0; i < SPEC_HSW; ++i) u[i] = lq[(e0 + i) * SPEC_BS + tid];
  #pragma unroll
                for (int i = 0; i < SPEC_HSW; ++i)
                  if (u[i] > hmax) {
                    hmax = u[i];
                    hmi = e0 + i;
                  }
              }
            }
          }
        }
        hmx = hmax;
        int w = 0;
        cmin = 256;
        #pragma unroll 1
        for (int k0 = 0; k0 < nc; k0 += SPEC_RFW) {
          unsigned long long v[SPEC_RFW];
  #pragma unroll
          for (int k = 0; k < SPEC_RFW; ++k) v[k] = (k0 + k < nc) ? ws.sxp[b + k0 + k] : 0ull;
  #pragma unroll
          for (int k = 0; k < SPEC_RFW; ++k) {
            if (k0 + k >= nc || v[k] <= hmax) continue;
            ws.sxp[b + w++] = v[k];
            cmin = min(cmin, (unsigned)(v[k] >> 52));
          }
        }
        nc = w;
      };
      unsigned dm = 0, ppm = 0;  // deferred pushes; the pending pop's pushes (all levels)
      if (ex && mylab != WSHED) {
  #pragma unroll
        for (int d = 0; d < 4; ++d) {
          if (!((pm >> d) & 1u)) continue;
          ppm |= 1u << d;
          const unsigned t = (wp >> (8 * d)) & 255u;
          if ((int)t < L) qpush(t, nbp[d]);
          else dm |= 1u << d;
        }
      }
      unsigned long long rec = srec_pack(p, mylab, dm);
      if (ex) {
        sig = smix(0x6a09e667f3bcc908ull, rec);
        nrec = 1;
      }
      // the pending pop: its writes are not issued yet
      int py = ex ? p : -1, plab = mylab;
      int pz[4] = {nbp[0], nbp[1], nbp[2], nbp[3]};
      auto issue_writes = [&](int k) {  // pop k of this execution: pixel py, label plab, pushes ppm
        claim_max(&spx[py].cl[par], spec_claim(T, j, 1u));
        st_ag32(&spx[py].lab[par], plab);
  #pragma unroll
        for (int d = 0; d < 4; ++d)
          if ((ppm >> d) & 1u) claim_max(&spx[pz[d]].cl[par], spec_claim(T, j, 0u));
        *rec_at(k) = rec;
      };
      if (ex && nq > 0 && !ovf && !gchg && j < ovlim) {
        const int4 pr = ws.srec[(size_t)ppar * SPEC_WIN + j];
        if (pr.z == (int)(T - 1u) && pr.y > 1 && ws.slog[pr.x] == rec &&
            spec_replay_clean(ws, pr.x, pr.y, ppar, T, nbp)) {
          issue_writes(0);
          for (int k = 1; k < pr.y; ++k) {  // round T's claims, as the cascade writes them
            const unsigned long long r = ws.slog[pr.x + k];
            const int y = (int)(r & 0x0fffffffu);
            const unsigned dmy = (unsigned)(r >> 28) & 15u;
            claim_max(&spx[y].cl[par], spec_claim(T, j, 1u));
            st_ag32(&spx[y].lab[par], (int)(uint32_t)(r >> 32));
  #pragma unroll
            for (int d = 0; d < 4; ++d)
              if ((dmy >> d) & 1u) claim_max(&spx[nbi(y + marg, d, Wt) - marg].cl[par], spec_claim(T, j, 0u));
            sig = smix(sig, r);
          }
          nrec = pr.y;
          rbase = pr.x;
          nq = nc = 0;
          ppm = 0;
          py = -1;
        }
      }
      // next pop: the smallest key (lowest level, oldest push) of the lane's queue
      auto select = [&]() -> int {
        if (nq == 0) refill();
        // SPEC_HSW hot keys per LDS round trip (loads past nq read dead entries, ignored)
        int bi = 0;
        unsigned long long be = ~0ull;
        #pragma unroll 1
        for (int k0 = 0; k0 < nq; k0 += SPEC_HSW) {
          unsigned long long e[SPEC_HSW];
  #pragma unroll
          for (int i = 0; i < SPEC_HSW; ++i) e[i] = lq[(k0 + i) * SPEC_BS + tid];
  #pragma unroll
          for (int i = 0; i < SPEC_HSW; ++i)
            if (k0 + i < nq && e[i] < be) {
              be = e[i];
              bi = k0 + i;
            }
        }
        --nq;
        lq[bi * SPEC_BS + tid] = lq[nq * SPEC_BS + tid];
        if (nq == 0) hmx = 0;
        return (int)(be & 0x0fffffffull);
      };
      int y = 0;
      unsigned wy = 0;
      SpecRec r0, r1, r2, r3;  // four named records (an indexed array of them lands in scratch)
      int nby[4];
      auto issue_loads = [&]() {
        wy = (unsigned)ws.w4[y];
        const int yb = y + marg;
  #pragma unroll
        for (int d = 0; d < 4; ++d) nby[d] = nbi(yb, d, Wt) - marg;
        r0 = spec_load(ws, V, nby[0]);
        r1 = spec_load(ws, V, nby[1]);
        r2 = spec_load(ws, V, nby[2]);
        r3 = spec_load(ws, V, nby[3]);
      };
      bool more = ex && nq + nc > 0 && !ovf;
      if (more) {
        y = select();
        issue_loads();
      }
      vm_drain();
      if (ex && py >= 0) issue_writes(0);
      // the execution length cap (see lcap above)
      const bool longok = j == P || (lcap && T > G);
      for (;;) {
       if (more) {
        bool go = true;
        if (nrec >= (longok ? SPEC_MAXREC : SPEC_MAXREC_SHORT)) {  // a long cascade: cheaper as serial pops
          ovf = cap = true;
          go = false;
        } else if (nrec >= SPEC_RL && (nrec - SPEC_RL) % SPEC_XCH == 0) {  // the next record starts a chunk
          const int c = (nrec - SPEC_RL) / SPEC_XCH;
          const int b = c < SPEC_NX ? pool_get(SPEC_XCH) : -1;
          if (b < 0) {
            ovf = cap = true;
            go = false;
          }
          if (c == 0) xb0 = b;
          else if (c == 1) xb1 = b;
          else if (c == 2) xb2 = b;
          else xb3 = b;
        }
        if (!go) more = false;
       }
       if (more) {
#ifdef MSEG_SPEC_PROF
        const long long q1 = (long long)__builtin_amdgcn_s_memtime();
        pf_n += 1;
        pf_q += nq + 1;
#endif
        int v[4];
        v[0] = spec_decide_own(V, r0, j);
        v[1] = spec_decide_own(V, r1, j);
        v[2] = spec_decide_own(V, r2, j);
        v[3] = spec_decide_own(V, r3, j);
  #pragma unroll
        for (int d = 0; d < 4; ++d) {  // the pending pop's writes, not in memory yet (selects)
          bool inq = false;
  #pragma unroll
          for (int e = 0; e < 4; ++e) inq |= (((ppm >> e) & 1u) != 0) & (nby[d] == pz[e]);
          v[d] = inq ? INQ : (nby[d] == py) ? plab : v[d];
        }
        int lab = 0;
  #pragma unroll
        for (int d = 0; d < 4; ++d)
          if (v[d] > 0) lab = fold_lab(lab, v[d]);
#ifdef MSEG_SPEC_PROF
        const long long q2 = (long long)__builtin_amdgcn_s_memtime();
        pf_load += q2 - q1;
#endif
        if (lab == 0) {  // own writes hidden by a conflicting lower rank: unstable
          ovf = true;
          lab = WSHED;
        }
        unsigned dmy = 0, pmy = 0;
        if (lab != WSHED) {
  #pragma unroll
          for (int d = 0; d < 4; ++d) {
            if (v[d] != 0) continue;
            pmy |= 1u << d;
            const unsigned t = (wy >> (8 * d)) & 255u;
            if ((int)t < L) qpush(t, nby[d]);
            else dmy |= 1u << d;
          }
        }
        rec = srec_pack(y, lab, dmy);
        sig = smix(sig, rec);
        py = y;
        plab = lab;
        ppm = pmy;
  #pragma unroll
        for (int d = 0; d < 4; ++d) pz[d] = nby[d];
        const int k = nrec++;
        more = nq + nc > 0 && !ovf;
#ifdef MSEG_SPEC_PROF
        const long long q3 = (long long)__builtin_amdgcn_s_memtime();
#endif
        if (more) {
          y = select();
          issue_loads();
        }
        vm_drain();
#ifdef MSEG_SPEC_PROF
        const long long q4 = (long long)__builtin_amdgcn_s_memtime();
        pf_sel += q4 - q3;
#endif
        issue_writes(k);
#ifdef MSEG_SPEC_PROF
        pf_write += (long long)__builtin_amdgcn_s_memtime() - q4 + (q3 - q2);
#endif
       }
        // at most COOP_LANES lanes left with cascades: the wave takes them over (spec_coop) and
        // finishes them one after another; every one but the first first moves its hot keys to
        // its cold chunk (the cooperative queue reuses the wave's LDS columns)
        unsigned long long bal = __ballot(more);
        if (bal == 0) break;
        if (__popcll(bal) <= COOP_LANES) {
          const int w0 = __builtin_ctzll(bal);
          const bool canspill = !more || lane == w0 || nq == 0 || (cb != -2 && nc + nq <= SPEC_CCAP);
          if (!__all(canspill)) continue;  // (pool full: those lanes carry on alone)
          if (more && lane != w0 && nq > 0) {
            if (cb < 0 && (cb = pool_get(SPEC_CCAP)) < 0) {
              cb = -2;
              ovf = cap = true;  // a capacity overflow, as a failed cold push would be
              more = false;
            } else {
              for (int e = 0; e < nq; ++e) {
                const unsigned long long k = lq[(size_t)e * SPEC_BS + tid];
                ws.sxp[(size_t)cb + nc + e] = k;
                cmin = min(cmin, (unsigned)(k >> 52));
              }
              nc += nq;
              nq = 0;
              hmx = 0;
            }
          }
          bal = __ballot(more);
        }
        if (bal != 0 && __popcll(bal) <= COOP_LANES) for (unsigned long long lb = bal; lb; lb &= lb - 1) {
          const int w = __builtin_ctzll(lb);
          CoopSt S;
          S.y = __builtin_amdgcn_readlane(y, w);
          S.py = __builtin_amdgcn_readlane(py, w);
          S.plab = __builtin_amdgcn_readlane(plab, w);
          S.ppm = (unsigned)__builtin_amdgcn_readlane((int)ppm, w);
          S.pz0 = __builtin_amdgcn_readlane(pz[0], w);
          S.pz1 = __builtin_amdgcn_readlane(pz[1], w);
          S.pz2 = __builtin_amdgcn_readlane(pz[2], w);
          S.pz3 = __builtin_amdgcn_readlane(pz[3], w);
          S.prec = 0;
          S.pwrite = false;  // the per-lane loop issued them
          S.nrec = __builtin_amdgcn_readlane(nrec, w);
          S.sig = ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(sig >> 32), w) << 32) |
                  (unsigned)__builtin_amdgcn_readlane((int)(unsigned)sig, w);
          S.qseq = (unsigned)__builtin_amdgcn_readlane((int)qseq, w);
          S.nq = __builtin_amdgcn_readlane(nq, w);
          S.nc = __builtin_amdgcn_readlane(nc, w);
          S.cb = __builtin_amdgcn_readlane(cb, w);
          S.cmin = (unsigned)__builtin_amdgcn_readlane((int)cmin, w);
          S.xb0 = __builtin_amdgcn_readlane(xb0, w);
          S.xb1 = __builtin_amdgcn_readlane(xb1, w);
          S.xb2 = __builtin_amdgcn_readlane(xb2, w);
          S.xb3 = __builtin_amdgcn_readlane(xb3, w);
          S.ovf = S.cap = false;
          const int jw = __builtin_amdgcn_readlane(j, w);
          const int wb = tid & ~63;
          const long long tco0 = dg ? (long long)__builtin_amdgcn_s_memrealtime() : 0;
          spec_coop(ws, V, lq, wb, w, jw, L, jw == P || (lcap && T > G),
                    ws.stmp + (size_t)(blockIdx.x * SPEC_BS + wb + w) * SPEC_RL, S);
          if (dg) tco += (long long)__builtin_amdgcn_s_memrealtime() - tco0;
          if (lane == w) {
            nrec = S.nrec;
            sig = S.sig;
            ovf = S.ovf;
            cap = S.cap;
            xb0 = S.xb0;
            xb1 = S.xb1;
            xb2 = S.xb2;
            xb3 = S.xb3;
            nq = nc = 0;
            more = false;
          }
        }
      }
    }  // the execution
    if (dg) {
      tw += tkb - tka;
      tc += (long long)__builtin_amdgcn_s_memrealtime() - tkb;
      tpo -= (long long)__builtin_amdgcn_s_memrealtime();  // + the chunk's end below
    }
    // ---- log space for the wave's records (one atomic per wave), signatures, change words ----
    const int want = (ex && !ovf && rbase < 0) ? nrec : 0;
    const int incl = wave_scan_add(want);
    const int wtot = __builtin_amdgcn_readlane(incl, 63);
    int wbase = 0;
    if (lane == 0 && wtot) wbase = atomicAdd(&ctl->slogtop.v, wtot);
    wbase = __builtin_amdgcn_readlane(wbase, 0);
    int fcand = NONE, ocand = NONE;
    // this lane's log copy, its marks of the new / the previous round's records: done per lane for
    // short executions, by the whole wave (64 records per step, one execution at a time) for long
    // ones -- a long cascade's records used to be copied and marked by its lane alone, record by
    // record, on the round's critical path (~9% of uniform noise's round time, round 5)
    constexpr int LONGREC = 16;
    bool cpy = false, mkn = false, mkp = false;
    int4 prv = make_int4(0, 0, 0, 0);
    int base = 0;
    unsigned* const dn = ws.sdirt + (size_t)par * ws.snp;
    auto mark = [&](unsigned long long r) {
      const int y = (int)(r & 0x0fffffffu);
      const unsigned dmy = (unsigned)(r >> 28) & 15u;
      dn[y] = T;
#pragma unroll
      for (int d = 0; d < 4; ++d)
        if ((dmy >> d) & 1u) dn[nbi(y + marg, d, Wt) - marg] = T;
    };
    if (ex) {
      base = rbase >= 0 ? rbase : wbase + incl - want;
      if (!ovf && rbase < 0) {
        if ((long long)base + nrec > ws.slogcap) ovf = cap = true;  // generation log full
        else cpy = true;
      }
      sig = smix(sig, ((unsigned long long)nrec << 1) | (ovf ? 1ull : 0ull));
      ws.srec[(size_t)par * SPEC_WIN + j] = make_int4(base, ovf ? 0 : nrec, (int)T, cap ? 1 : 0);
      ws.ssig[(size_t)par * SPEC_WIN + j] = sig;
      // unchanged = the same execution in the immediately preceding round
      const bool changed = !V.hasprev || ovf || ws.srec[(size_t)ppar * SPEC_WIN + j].z != (int)(T - 1u) ||
                           ws.ssig[(size_t)ppar * SPEC_WIN + j] != sig;
      if (changed) fcand = j;
      if (ovf) ocand = j;
      if (rbase >= 0) ++nrep;
      else nxpop += nrec;
      if (changed) {  // mark both executions' claims: round T + 1 replays nothing that viewed them
        mkn = rbase < 0;
        prv = ws.srec[(size_t)ppar * SPEC_WIN + j];
        mkp = V.hasprev && prv.z == (int)(T - 1u) && prv.y > 0;
      }
      if (cpy && nrec <= LONGREC)
        for (int k = 0; k < nrec; ++k) ws.slog[base + k] = *rec_at(k);
      if (mkn && nrec <= LONGREC)
        for (int k = 0; k < nrec; ++k) mark(*rec_at(k));
      if (mkp && prv.y <= LONGREC)
        for (int k = 0; k < prv.y; ++k) mark(ws.slog[prv.x + k]);
    }
    {
      const int wb = tid & ~63;
      for (unsigned long long lb = __ballot((cpy || mkn) && nrec > LONGREC); lb; lb &= lb - 1) {
        const int w = __builtin_ctzll(lb);
        const int nw = __builtin_amdgcn_readlane(nrec, w), bw = __builtin_amdgcn_readlane(base, w);
        const bool cw = __builtin_amdgcn_readlane((int)cpy, w) != 0, mw = __builtin_amdgcn_readlane((int)mkn, w) != 0;
        const int x0 = __builtin_amdgcn_readlane(xb0, w), x1 = __builtin_amdgcn_readlane(xb1, w);
        const int x2 = __builtin_amdgcn_readlane(xb2, w), x3 = __builtin_amdgcn_readlane(xb3, w);
        unsigned long long* const tw_ = ws.stmp + (size_t)(blockIdx.x * SPEC_BS + wb + w) * SPEC_RL;
        for (int k = lane; k < nw; k += 64) {
          const unsigned long long r = *spec_rec_at(tw_, ws.sxp, k, x0, x1, x2, x3);
          if (cw) ws.slog[bw + k] = r;
          if (mw) mark(r);
        }
      }
      for (unsigned long long lb = __ballot(mkp && prv.y > LONGREC); lb; lb &= lb - 1) {
        const int w = __builtin_ctzll(lb);
        const int px = __builtin_amdgcn_readlane(prv.x, w), py_ = __builtin_amdgcn_readlane(prv.y, w);
        for (int k = lane; k < py_; k += 64) mark(ws.slog[px + k]);
      }
    }
    fcand = wave_min(fcand);
    ocand = wave_min(ocand);
    const int wxmax = -wave_min((ex && rbase < 0) ? -nrec : 0);  // the wave's longest execution
    if (lane == 0) {
      if (wxmax > 0) atomicMax(&ctl->spec.rxmax, wxmax);
      // ranks are dealt in increasing order: once a lower rank is in, later waves skip the atomic
      if (fcand != NONE) atomicMin(&ctl->sfc.v, fcand);
      if (ocand != NONE) atomicMin(&ctl->sovf.v, ocand);
      const int nex = max(0, min(n, r0 + 64) - max(P, r0));
      if (nex) atomicAdd(&s_exec, nex);
    }
    if (dg) tpo += (long long)__builtin_amdgcn_s_memrealtime();
  }
  if (dg) {
    if (lane == 0) {
      const long long tot = (long long)__builtin_amdgcn_s_memrealtime() - tk0;
      atomicAdd(&dg[2], (unsigned long long)tot); // wave time in the kernel
      atomicMax(&dg[3], (unsigned long long)tot); // longest wave
      atomicAdd(&dg[7], 1ull);
      // the round's longest wave with its wait / cascade split (10 ns ticks, 20 bits each)
      atomicMax(&ctl->spec.rmax, ((unsigned long long)tot << 40) | ((unsigned long long)min(tw, 0xfffffll) << 20) |
                                     (unsigned long long)min(tc, 0xfffffll));
      // ... and its cooperative-cascade / post-execution split (the same wave unless two tie)
      atomicMax(&ctl->spec.rmax2, ((unsigned long long)tot << 40) | ((unsigned long long)min(tco, 0xfffffll) << 20) |
                                      (unsigned long long)min(tpo, 0xfffffll));
    }
  }
#ifdef MSEG_SPEC_PROF
  if (ws.diag) {  // bank 2 (msg_set_diag 3): cascade pops, queue entries scanned, phase cycles
    atomicAdd(&ws.diag[16], (unsigned long long)pf_n);
    atomicAdd(&ws.diag[17], (unsigned long long)pf_q);
    atomicAdd(&ws.diag[18], (unsigned long long)pf_sel);
    atomicAdd(&ws.diag[19], (unsigned long long)pf_load);
    atomicAdd(&ws.diag[20], (unsigned long long)pf_write);
  }
#endif
  if (nrep) atomicAdd(&s_rep, nrep);
  nxpop = wave_sum(nxpop);
  if (lane == 0 && nxpop) atomicAdd(&s_xpop, nxpop);
  __syncthreads();
  if (tid == 0) {
    atomicAdd((unsigned long long*)&ctl->spec.execs, (unsigned long long)s_exec);
    if (s_rep) atomicAdd((unsigned long long*)&ctl->spec.replays, (unsigned long long)s_rep);
    if (s_xpop) atomicAdd((unsigned long long*)&ctl->spec.xpops, (unsigned long long)s_xpop);
    __threadfence();
    if (atomicAdd(&ctl->spec.ticket, 1) == (int)gridDim.x - 1) {
      __threadfence();
      spec_finalize(ctl, P, n, T, G, dg);
    }
  }
}

// The generation's commit as an ordinary batch of "virtual items" (one per pop, in serial
// order) for k_scan / k_scatter: pixel, label and deferred-push descriptor per virtual rank, the
// per-chunk level histograms, and the batch header: n = pops, one segment advancing bucket L's
// head by P.  Tiles of SPEC_FT items are dealt in dispatch order and chained (a tile waits only
// for the tile before it, held by a running block).
__global__ __launch_bounds__(SPEC_FT) void k_spec_flatten(Ws ws) {
  Ctl* ctl = ws.ctl;
  if (ctl->bat.mode != 3 || ctl->spec.state != 2 || ctl->error) return;
  SpecCtl& s = ctl->spec;
  const int P = s.P, Pprom = s.Pprom, L = s.L, bstart = s.bstart;
  const unsigned T = s.T, G = s.G;
  const int tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
  const unsigned long long etag = (unsigned long long)ctl->bat.epoch << 32;
  __shared__ int s_tile, s_off, s_tot;
  __shared__ int wsum[SPEC_FT / 64];
  __shared__ int s_ex[SPEC_FT], s_bx[SPEC_FT];  // the tile's items: first virtual rank, log base
  if (P == 0) {  // nothing final (overflow at rank 0): the batch engine takes the bucket's head
    if (blockIdx.x == 0 && tid == 0) {
      Batch nb = ctl->bat;
      nb.mode = 0;
      nb.n = min(s.n, WMIN);
      nb.nseg = 1;
      nb.ncommit = 0;
      nb.nchunk = 0;
      nb.rrun = 0;
      Seg sg;
      sg.L = L;
      sg.bstart = bstart;
      sg.rank = 0;
      sg.n = nb.n;
      ctl->seg[0] = sg;
      ctl->cut = NONE;
      ctl->segcut = NONE;
      ctl->minpush = 0;
      ctl->wcap = WMIN;
      s.on = 0;
      s.block = L;
      s.fallbacks += 1;
      s.state = 0;
      ctl->bat = nb;  // undecided (rsv != epoch): k_scan leaves it to the small-batch loop
    }
    return;
  }
  const int ntiles = (P + SPEC_FT - 1) / SPEC_FT;
  for (;;) {
    if (tid == 0) s_tile = atomicAdd(&s.ftile, 1);
    __syncthreads();
    const int tile = s_tile;
    if (tile >= ntiles) break;
    const int j = tile * SPEC_FT + tid;
    int2 rc = make_int2(0, 0);
    if (j < P) {
      if (j < Pprom) {
        rc = ws.sfrec[j];
      } else {
        const int4 r4 = ws.srec[(size_t)(T & 1u) * SPEC_WIN + j];
        rc = make_int2(r4.x, r4.y);
      }
    }
    const int x = wave_scan_add(rc.y);
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    int excl = x - rc.y, tot = 0;
#pragma unroll
    for (int k = 0; k < SPEC_FT / 64; ++k) {
      if (k < wv) excl += wsum[k];
      tot += wsum[k];
    }
    s_ex[tid] = excl;
    s_bx[tid] = rc.x;
    if (tid == 0) {
      int prev = 0;
      if (tile > 0) {
        long long t0 = 0;
        for (;;) {
          const unsigned long long f = ld_ag64(ws.sflag + tile - 1);
          if ((unsigned)(f >> 32) == G) {
            prev = (int)(uint32_t)f;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          const long long now = (long long)__builtin_amdgcn_s_memrealtime();
          if (t0 == 0) t0 = now;
          else if (now - t0 > SPIN_LIMIT_TICKS) {
            atomicOr(&ctl->error, ERR_TIMEOUT);
            break;
          }
        }
      }
      st_ag64(ws.sflag + tile, ((unsigned long long)G << 32) | (uint32_t)(prev + tot));
      s_off = prev;
      s_tot = prev + tot;
    }
    __syncthreads();
    // the tile's records, dealt over the whole block (an item's records used to be one thread's
    // loop: a long execution's thousands of records held the commit for milliseconds)
    for (int q = tid; q < tot; q += SPEC_FT) {
      int lo = 0;  // the last item whose first virtual rank is <= q (empty items share the next's)
#pragma unroll
      for (int h = SPEC_FT / 2; h > 0; h >>= 1)
        if (s_ex[lo + h] <= q) lo += h;
      const unsigned long long r = ws.slog[s_bx[lo] + (q - s_ex[lo])];
      const int y = (int)(r & 0x0fffffffu);
      const unsigned dm = (unsigned)(r >> 28) & 15u;
      const int v = s_off + q;
      const unsigned wy = (unsigned)ws.w4[y];
      ws.ipx[v] = y;
      ws.tl[v] = etag | (uint32_t)(r >> 32);
      ws.desc[v] = make_desc(wy, dm, L, 0);
#pragma unroll
      for (int d = 0; d < 4; ++d)
        if ((dm >> d) & 1u) atomicAdd(&ws.cnt[(long long)(v / CH) * NQ + ((wy >> (8 * d)) & 255u)], 1);
    }
    if (tile == ntiles - 1 && tid == 0) {  // the batch header (read by the next kernel)
      const int Vn = s_tot;
      Batch nb = ctl->bat;
      nb.mode = 0;
      nb.n = Vn;
      nb.nseg = 1;
      nb.ncommit = 0;
      nb.nchunk = 0;
      nb.rrun = 0;
      Seg sg;
      sg.L = L;
      sg.bstart = bstart;
      sg.rank = 0;
      sg.n = P;  // k_scan advances bucket L's head by min(pops, P) = P
      ctl->seg[0] = sg;
      ctl->cut = NONE;
      ctl->segcut = NONE;
      ctl->minpush = 0;  // no multi-segment merge right after a generation
      ctl->rsv = nb.epoch;
      s.gens += 1;
      s.cpops += Vn - P;
      // every generation (fallbacks included) is judged against serial pops over the span since
      // the regime's start: slower per committed pop (small generations: a round costs launch
      // floors and its longest execution; frequent fallbacks) -> serial pops for a while
      const long long now = (long long)__builtin_amdgcn_s_memrealtime();
      s.gpops_total += Vn;
      s.gticks_total += now - s.tgen;  // (measured: reported in msg_stats, never judged on)
      ++s.accg;
      // judged on the generations' modelled time (ws_shared.h: rounds and each round's longest
      // execution, + a commit estimate each) per pop they committed, not on the wall time since
      // the regime started: a fallback's serial pops cost the same either way (round 3 A/B:
      // neutral on every frame, profiles/r03l_ab_regimes.log)
      // (leaving the generations that fell back out of this judgement kept the regime on where it
      // re-ran the rest of a bucket after every long cascade: uniform noise at 4096^2 went from 15.7
      // to 48 s, round 4)
      s.tspec += (long long)SPEC_ROUND_TICKS * s.rounds + (long long)SPEC_POP_TICKS * (s.xlong - s.gxlong0) +
                 SPEC_COMMIT_TICKS;
      s.pspec += Vn;
      const bool judge = s.accg >= SPEC_JUDGE_GENS || (s.accg >= 4 && s.tspec > SPEC_JUDGE_TICKS);
      const bool slow = judge && s.tspec > (long long)SPEC_SERIAL_TICKS * s.pspec;
      if (s.fallback) {
        // the batch engine pops the overflowing item and its cascade (serial pops); the regime
        // resumes once the lowest level is back at L (generations inside a cascade that
        // overflowed a lane are small: measured slower)
        s.on = 0;
        s.block = slow ? 0 : L;
        s.fallbacks += 1;
        ctl->wcap = WMIN;
      } else if (Vn == P && s.n >= SPEC_QUIET) {  // a large generation without a cascade: batches pay
        s.on = 0;
        s.block = 0;
      }
      // judged slower than serial pops: maybe long final cascades serialised one per round as heads
      // of the stable prefix (uniform noise at 4096^2: invasion-percolation avalanches everywhere).
      // Besides the cooldown, from here on every execution may run long from round 2 on
      // (SpecCtl.deep; round 4 A/B: 16.7 -> 1.66 s there).  Judged slow again in deep mode, the
      // flood's generations are small ones that long executions only slow down (album.jpg): off
      if (slow) s.deep = s.deep == 0 ? 1 : 2;
      if (slow) {
        s.on = 0;
        s.block = 0;
        s.cool = SPEC_COOL_POPS << min(s.fails, 6);
        s.fails += 1;
        s.cools += 1;
        s.fresh = 1;
      }
      s.state = 0;
      ctl->bat = nb;
    }
    __syncthreads();  // s_tile / wsum reused
  }
}

}  // namespace msg
