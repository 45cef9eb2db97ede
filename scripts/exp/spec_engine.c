// CPU prototype of the exact speculative-cascade batch (design study for the GPU small loop).
//
// A batch is the first n items x_0..x_{n-1} of the lowest non-empty bucket L.  Serially, each
// x_r pops, and if it pushes below L its cascade C_r (a full drain of levels < L) runs before
// x_{r+1}.  Here every phase is computed as the GPU would, against the pre-batch state:
//   1. top items: labels/pushes with only earlier TOP items visible (k_resolve's semantics);
//   2. cascades run speculatively (in a shuffled order, to prove order independence): reads see
//      the pre-batch state + top items <= r (labels, and 0-pixels they push) + own writes;
//      ownership own[z] = min rank of the cascades writing z;
//   3. validation: x_j is cut if a 4-neighbour is owned by a cascade r < j; C_r is dropped (cut
//      after x_r, whose low pushes then queue normally) if it read a pixel owned by r' < r or
//      exceeded its pop budget;
//   4. commit of the prefix, ordered append: per item, its own >= L pushes then its cascade's
//      deferred pushes, in serial order.
// usage: spec_engine H W window budget < (bgr H*W*3 bytes, markers H*W int32) > labels (int32)
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define WSHED (-1)
#define INQ (-2)
static int H, W;
static const uint8_t* IMG;
static int32_t* M;  // state: >0 label, -1 WSHED, 0 unknown, -2 queued (in some bucket)

static int cd(int p, int q) {
  const uint8_t *a = IMG + 3 * (size_t)p, *b = IMG + 3 * (size_t)q;
  int d0 = abs(a[0] - b[0]), d1 = abs(a[1] - b[1]), d2 = abs(a[2] - b[2]);
  int m = d0 > d1 ? d0 : d1;
  return m > d2 ? m : d2;
}
typedef struct { int32_t* v; size_t h, n, c; } Q;
static Q q[256];
static void qpush(Q* b, int32_t x) {
  if (b->n == b->c) { b->c = b->c ? b->c * 2 : 1024; b->v = realloc(b->v, b->c * 4); }
  b->v[b->n++] = x;
}
static inline void nb4(int p, int* n) { n[0] = p - 1; n[1] = p + 1; n[2] = p - W; n[3] = p + W; }

// per-batch scratch (pixel-indexed arrays tagged by batch id)
static int64_t *own_tag, *prank_tag, *priv_tag;
static int32_t *own_rank, *prank, *priv_val;
static int32_t* trank;  // rank of a top item at its pixel (valid while prank_tag... uses own tag)
static int64_t* trank_tag;
static long long bid = 0;

// cascade logs
typedef struct { int pix, lv, seq; } Ent;
typedef struct {
  int n, cap;
  int* pops;    // popped pixels (order)
  int npops;
  Ent* def;     // deferred (>= L) pushes in order
  int ndef, capdef;
  Ent* loc;     // local queue entries
  int nloc, caploc;
  int overflow;
} Casc;

static int* tlab;            // top item labels
static unsigned* tmask;      // top item push masks
static int32_t* tpix;        // top item pixels

static int top_view(int z, int r) {  // state of z seen by cascade r (excluding its own writes)
  int v = M[z];
  if (v == INQ && trank_tag[z] == bid) {  // a batch item
    int j = trank[z];
    return j <= r ? tlab[j] : INQ;
  }
  if (v == 0 && prank_tag[z] == bid && prank[z] <= r) return INQ;
  return v;
}
static int cview(int z, int r) {
  if (priv_tag[z] == bid && own_tag[z] == bid && own_rank[z] == r) return priv_val[z];
  return top_view(z, r);
}
static void cwrite(int z, int r, int v) {
  if (own_tag[z] != bid || own_rank[z] > r) { own_tag[z] = bid; own_rank[z] = r; }
  if (own_rank[z] == r) { priv_tag[z] = bid; priv_val[z] = v; }
}

static long long st_batches, st_pops, st_casc, st_cascpops, st_drop, st_cut_a, st_over, st_maxc;

static void run_cascade(Casc* C, int r, int L, int budget) {
  C->npops = C->ndef = C->nloc = 0;
  C->overflow = 0;
  int seq = 0;
  int p = tpix[r];
  int n[4];
  nb4(p, n);
  // x_r's pushes below L seed the cascade (direction order)
  for (int d = 0; d < 4; d++)
    if ((tmask[r] >> d) & 1) {
      int t = cd(p, n[d]);
      if (t < L) { C->loc[C->nloc++] = (Ent){n[d], t, seq++}; }
    }
  for (;;) {
    int best = -1;
    for (int k = 0; k < C->nloc; k++)
      if (C->loc[k].pix >= 0 && (best < 0 || C->loc[k].lv < C->loc[best].lv ||
                                 (C->loc[k].lv == C->loc[best].lv && C->loc[k].seq < C->loc[best].seq)))
        best = k;
    if (best < 0) break;
    if (C->npops >= budget) { C->overflow = 1; return; }
    int y = C->loc[best].pix;
    C->loc[best].pix = -1;
    C->pops[C->npops++] = y;
    int m[4];
    nb4(y, m);
    int lab = 0;
    for (int d = 0; d < 4; d++) {
      int t = cview(m[d], r);
      if (t > 0) lab = lab == 0 ? t : (lab == t ? t : WSHED);
    }
    if (lab == 0) lab = WSHED;  // garbage from a conflicting read (dropped at validation)
    cwrite(y, r, lab);
    if (lab == WSHED) continue;
    for (int d = 0; d < 4; d++) {
      if (cview(m[d], r) != 0) continue;
      int t = cd(y, m[d]);
      cwrite(m[d], r, INQ);
      if (t < L) {
        if (C->nloc >= C->caploc) { C->overflow = 1; return; }
        C->loc[C->nloc++] = (Ent){m[d], t, seq++};
      } else {
        if (C->ndef >= C->capdef) { C->overflow = 1; return; }
        C->def[C->ndef++] = (Ent){m[d], t, seq++};
      }
    }
  }
}

int main(int argc, char** argv) {
  H = atoi(argv[1]); W = atoi(argv[2]);
  int WIN = argc > 3 ? atoi(argv[3]) : 4096;
  int BUDGET = argc > 4 ? atoi(argv[4]) : 64;
  size_t N = (size_t)H * W;
  uint8_t* img = malloc(N * 3);
  M = malloc(N * 4);
  if (fread(img, 1, N * 3, stdin) != N * 3 || fread(M, 4, N, stdin) != N) return 2;
  IMG = img;
  own_tag = calloc(N, 8); prank_tag = calloc(N, 8); priv_tag = calloc(N, 8); trank_tag = calloc(N, 8);
  own_rank = calloc(N, 4); prank = calloc(N, 4); priv_val = calloc(N, 4); trank = calloc(N, 4);
  // phase 0/1 (oracle semantics)
  for (int c = 0; c < W; c++) { M[c] = WSHED; M[(H - 1) * W + c] = WSHED; }
  for (int r = 1; r < H - 1; r++) {
    M[r * W] = WSHED; M[r * W + W - 1] = WSHED;
    for (int c = 1; c < W - 1; c++) {
      int p = r * W + c;
      if (M[p] < 0) M[p] = 0;
      if (M[p]) continue;
      int l = 256, n[4];
      nb4(p, n);
      for (int k = 0; k < 4; k++) if (M[n[k]] > 0) { int t = cd(p, n[k]); if (t < l) l = t; }
      if (l < 256) { qpush(&q[l], p); M[p] = INQ; }
    }
  }
  tlab = malloc(sizeof(int) * WIN); tmask = malloc(4 * WIN); tpix = malloc(4 * WIN);
  Casc* cs = calloc(WIN, sizeof(Casc));
  for (int k = 0; k < WIN; k++) {
    cs[k].pops = malloc(4 * BUDGET);
    cs[k].capdef = 4 * BUDGET; cs[k].def = malloc(sizeof(Ent) * cs[k].capdef);
    cs[k].caploc = 4 * BUDGET + 4; cs[k].loc = malloc(sizeof(Ent) * cs[k].caploc);
  }
  int* has = malloc(4 * WIN);
  int* order = malloc(4 * WIN);
  unsigned rng = 12345;
  int win = 64;
  for (;;) {
    int L = 0;
    while (L < 256 && q[L].h == q[L].n) L++;
    if (L == 256) break;
    bid++;
    st_batches++;
    int n = (int)(q[L].n - q[L].h);
    if (n > win) n = win;
    // 1. top items in rank order, only earlier top items visible (overlay on M via tlab)
    for (int i = 0; i < n; i++) { tpix[i] = q[L].v[q[L].h + i]; trank_tag[tpix[i]] = bid; trank[tpix[i]] = i; }
    int icut = -1;  // first item pushing below L
    for (int i = 0; i < n; i++) {
      int p = tpix[i], nn[4];
      nb4(p, nn);
      int lab = 0;
      for (int d = 0; d < 4; d++) {
        int t = M[nn[d]];
        if (t == INQ && trank_tag[nn[d]] == bid && trank[nn[d]] < i) t = tlab[trank[nn[d]]];
        if (t > 0) lab = lab == 0 ? t : (lab == t ? t : WSHED);
      }
      tlab[i] = lab;
      unsigned m = 0;
      has[i] = 0;
      if (lab != WSHED)
        for (int d = 0; d < 4; d++) {
          int z = nn[d];
          if (M[z] != 0) continue;
          if (prank_tag[z] == bid && prank[z] < i) continue;  // pushed by an earlier top item
          m |= 1u << d;
          prank_tag[z] = bid; prank[z] = i;
          if (cd(p, z) < L) has[i] = 1;
        }
      tmask[i] = m;
      if (has[i] && icut < 0) icut = i;
    }
    // 2. cascades, speculative, in a shuffled order
    int nc = 0;
    for (int i = 0; i < n; i++) if (has[i]) order[nc++] = i;
    for (int k = nc - 1; k > 0; k--) { rng = rng * 1103515245u + 12345u; int j = (rng >> 8) % (k + 1); int t = order[k]; order[k] = order[j]; order[j] = t; }
    for (int k = 0; k < nc; k++) { run_cascade(&cs[order[k]], order[k], L, BUDGET); st_casc++; }
    // 3. validation -> ncommit; dropped cascade index (cut after it), or none
    int ncommit = n, drop = -1;
    for (int j = 0; j < n; j++) {
      int nn[4];
      nb4(tpix[j], nn);
      int bad = 0;
      for (int d = 0; d < 4; d++) if (own_tag[nn[d]] == bid && own_rank[nn[d]] < j) bad = 1;
      if (bad) { ncommit = j; st_cut_a++; break; }
      if (has[j]) {
        Casc* C = &cs[j];
        int cbad = C->overflow;
        for (int k = 0; k < C->npops && !cbad; k++) {
          int mm[4];
          nb4(C->pops[k], mm);
          if (own_rank[C->pops[k]] < j) cbad = 1;  // (pops are always owned this batch)
          for (int d = 0; d < 4; d++) if (own_tag[mm[d]] == bid && own_rank[mm[d]] < j) cbad = 1;
        }
        for (int k = 0; k < C->ndef && !cbad; k++) if (own_rank[C->def[k].pix] < j) cbad = 1;
        if (cbad) { ncommit = j + 1; drop = j; if (C->overflow) st_over++; else st_drop++; break; }
      }
    }
    // 4. commit: labels, then the ordered append
    for (int i = 0; i < ncommit; i++) {
      int p = tpix[i], nn[4];
      nb4(p, nn);
      M[p] = tlab[i];
      st_pops++;
      for (int d = 0; d < 4; d++)
        if ((tmask[i] >> d) & 1) {
          int t = cd(p, nn[d]);
          if (t < L && has[i] && i != drop) continue;  // handled by the committed cascade
          M[nn[d]] = INQ;
          qpush(&q[t], nn[d]);
        }
      if (has[i] && i != drop) {
        Casc* C = &cs[i];
        for (int k = 0; k < C->npops; k++) M[C->pops[k]] = priv_val[C->pops[k]];
        for (int k = 0; k < C->ndef; k++) { M[C->def[k].pix] = INQ; qpush(&q[C->def[k].lv], C->def[k].pix); }
        st_cascpops += C->npops;
        st_pops += C->npops;
        if (C->npops > st_maxc) st_maxc = C->npops;
      }
    }
    q[L].h += ncommit;
    // window: grow on a full uncut batch, shrink to twice the committed prefix after a cut
    if (ncommit == n && n == win) win = win * 2 > WIN ? WIN : win * 2;
    else if (ncommit < n) win = ncommit * 2 > 64 ? (ncommit * 2 > WIN ? WIN : ncommit * 2) : 64;
    (void)icut;
  }
  fwrite(M, 4, N, stdout);
  fprintf(stderr, "batches %lld pops %lld (%.1f/batch) cascades %lld cascade-pops %lld max %lld | cuts: item %lld cascade %lld overflow %lld\n",
          st_batches, st_pops, (double)st_pops / st_batches, st_casc, st_cascpops, st_maxc, st_cut_a, st_drop, st_over);
  return 0;
}
