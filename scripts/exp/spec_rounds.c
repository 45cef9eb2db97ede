// CPU prototype of the speculative-generation engine (design study for k_spec_round; not product).
//
// A generation = the whole lowest non-empty bucket L (up to a window), never cut at interrupts.
// Item j's execution = cv::watershed's own pop of its pixel followed by its cascade (every level
// < L, FIFO within a level, to exhaustion), as in the serial run.  Executions are repeated in
// rounds until no item's result changes; the serial result is the unique fixed point because
// item j only depends on items < j (triangular system).
//   * top pops (the item's own pixel) see the CURRENT round's top-pop results of earlier adjacent
//     top items (the GPU waits for them, as k_resolve does); everything an earlier item's cascade
//     wrote is seen through the PREVIOUS round's claims (Jacobi);
//   * claims: per pixel and round parity, one 64-bit word {tag, rank, popped, record}; the lowest
//     rank wins (atomicMax on inverted ranks); newer tags win; an item recognises its own writes
//     by its own rank in the current buffer;
//   * the stable prefix P (items unchanged since the previous round) is final: its claims are
//     promoted to a per-generation final array and it is not executed again;
//   * commit: the executions of items 0..P-1 flattened in rank order = the serial pop sequence.
// Cascades are executed in a shuffled order inside a round (the GPU gives no order).
// usage: spec_rounds H W window qcap < (bgr, markers) > labels
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define WSHED (-1)
#define INQ (-2)
static int H, W;
static const uint8_t* IMG;
static int32_t* M;
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
// claim word: tag(26) | (RMAX - rank)(21) | popped(1) | rec(16)
#define RMAX ((1u << 21) - 1)
static inline uint64_t ckey(uint32_t tag, uint32_t rank, int popped, uint32_t rec) {
  return ((uint64_t)tag << 38) | ((uint64_t)(RMAX - rank) << 17) | ((uint64_t)popped << 16) | rec;
}
static inline uint32_t c_tag(uint64_t c) { return (uint32_t)(c >> 38); }
static inline uint32_t c_rank(uint64_t c) { return RMAX - (uint32_t)((c >> 17) & RMAX); }
static inline int c_pop(uint64_t c) { return (int)((c >> 16) & 1); }
static inline uint32_t c_rec(uint64_t c) { return (uint32_t)(c & 0xffff); }
static uint64_t *cl[2], *fin;
static int* lastpar;  // round parity of each final item's last execution

typedef struct { int pix, lab, dmask; } Rec;
#define MAXREC 4096
typedef struct { Rec* r; int n; uint64_t sig; int ovf; } Exec;
static Exec *ex[2];  // per parity, per rank
static int QCAP = 16;

static uint32_t T, G;  // current round tag, generation tag (first round)
static int L, P, n;
static int32_t* tpix;       // batch pixels
static int* rank_of;        // pixel -> rank (valid if tag_of == gen)
static uint32_t* rank_tag;
static int* toplab;         // current round top labels (by rank), -100 = not yet
static uint64_t mix(uint64_t h, uint64_t v) { h ^= v + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2); return h * 0xff51afd7ed558ccdull; }

// status of pixel z for item j: >0 label, -1 WSHED, 0 unknown, INQ queued/pushed
static int view(int z, int j, int own_ok, const Exec* me) {
  uint64_t o = cl[T & 1][z];
  if (own_ok && c_tag(o) == T && c_rank(o) == (uint32_t)j) return c_pop(o) ? me->r[c_rec(o)].lab : INQ;
  uint64_t f = fin[z];
  if (c_tag(f) == G && f) {
    uint32_t k = c_rank(f);
    if (c_pop(f)) return ex[lastpar[k]][k].r[c_rec(f)].lab;
    return INQ;
  }
  if (T > G) {
    uint64_t c = cl[(T - 1) & 1][z];
    if (c_tag(c) == T - 1 && c_rank(c) < (uint32_t)j) {
      if (c_pop(c)) return ex[(T - 1) & 1][c_rank(c)].r[c_rec(c)].lab;
      return INQ;
    }
  }
  return M[z];
}
static void claim(int z, uint64_t k) { if (k > cl[T & 1][z]) cl[T & 1][z] = k; }

static long long st_rounds, st_exec, st_execpops, st_gens, st_maxr, st_serial, st_serialpops;

// top pop of item j (phase A, rank order); returns the push mask of 0-neighbours
static void top_pop(int j) {
  Exec* e = &ex[T & 1][j];
  e->n = 0; e->sig = 0x1234; e->ovf = 0;
  int p = tpix[j], nb[4] = {p - 1, p + 1, p - W, p + W};
  int lab = 0;
  for (int d = 0; d < 4; d++) {
    int z = nb[d], v;
    if (rank_tag[z] == G && rank_of[z] < j) v = toplab[rank_of[z]];  // earlier top item: this round
    else v = view(z, j, 0, e);
    if (v > 0) lab = lab == 0 ? v : (lab == v ? v : WSHED);
  }
  if (lab == 0) { lab = WSHED; e->ovf = 2; }  // impossible when exact: marks the item unstable
  toplab[j] = lab;
  e->r[0] = (Rec){p, lab, 0};
  e->n = 1;
  claim(p, ckey(T, j, 1, 0));
}

// the rest of item j's execution: the top pop's pushes and the cascade (phase B)
static void cascade(int j) {
  Exec* e = &ex[T & 1][j];
  int lq[64][2], nq = 0;  // local queue: pixel, level (append order = FIFO within a level)
  int cur = 0;             // record being expanded
  for (;;) {
    Rec* r = &e->r[cur];
    if (r->lab != WSHED) {
      int y = r->pix, nb[4] = {y - 1, y + 1, y - W, y + W};
      for (int d = 0; d < 4; d++) {
        int z = nb[d], v;
        if (cur == 0) {  // top pop: earlier top items adjacent to z push it first when non-WSHED
          int zz[4] = {z - 1, z + 1, z - W, z + W}, lose = 0;
          for (int k = 0; k < 4; k++)
            if (rank_tag[zz[k]] == G && rank_of[zz[k]] < j && toplab[rank_of[zz[k]]] != WSHED) lose = 1;
          if (lose) continue;
        }
        v = view(z, j, 1, e);
        if (v != 0) continue;
        int t = cd(y, z);
        claim(z, ckey(T, j, 0, 0));
        if (t < L) {
          if (nq >= QCAP) { e->ovf = 1; goto done; }
          lq[nq][0] = z; lq[nq][1] = t; nq++;
        } else r->dmask |= 1 << d;
      }
    }
    e->sig = mix(mix(mix(e->sig, (uint64_t)r->pix), (uint64_t)(uint32_t)r->lab), (uint64_t)r->dmask);
    if (nq == 0) break;
    int b = 0;
    for (int k = 1; k < nq; k++) if (lq[k][1] < lq[b][1]) b = k;
    int y = lq[b][0];
    for (int k = b; k + 1 < nq; k++) { lq[k][0] = lq[k + 1][0]; lq[k][1] = lq[k + 1][1]; }
    nq--;
    if (e->n >= MAXREC) { e->ovf = 1; goto done; }
    int nb[4] = {y - 1, y + 1, y - W, y + W}, lab = 0;
    for (int d = 0; d < 4; d++) {
      int v = view(nb[d], j, 1, e);
      if (v > 0) lab = lab == 0 ? v : (lab == v ? v : WSHED);
    }
    if (lab == 0) { lab = WSHED; e->ovf = 2; }
    cur = e->n++;
    e->r[cur] = (Rec){y, lab, 0};
    claim(y, ckey(T, j, 1, (uint32_t)cur));
  }
done:
  e->sig = mix(e->sig, (uint64_t)e->n * 31 + (uint64_t)e->ovf);
}

int main(int argc, char** argv) {
  H = atoi(argv[1]); W = atoi(argv[2]);
  int WIN = argc > 3 ? atoi(argv[3]) : 65536;
  QCAP = argc > 4 ? atoi(argv[4]) : 16;
  if (QCAP > 64) QCAP = 64;
  size_t N = (size_t)H * W;
  uint8_t* img = malloc(N * 3);
  M = malloc(N * 4);
  if (fread(img, 1, N * 3, stdin) != N * 3 || fread(M, 4, N, stdin) != N) return 2;
  IMG = img;
  cl[0] = calloc(N, 8); cl[1] = calloc(N, 8); fin = calloc(N, 8);
  rank_of = calloc(N, 4); rank_tag = calloc(N, 4);
  for (int k = 0; k < 2; k++) {
    ex[k] = calloc(WIN, sizeof(Exec));
    for (int i = 0; i < WIN; i++) ex[k][i].r = malloc(sizeof(Rec) * MAXREC);
  }
  tpix = malloc(4 * WIN); toplab = malloc(4 * WIN); lastpar = calloc(WIN, 4);
  int* order = malloc(4 * WIN);
  uint64_t* prevsig = malloc(8 * WIN);
  for (int c = 0; c < W; c++) { M[c] = WSHED; M[(H - 1) * W + c] = WSHED; }
  for (int r = 1; r < H - 1; r++) {
    M[r * W] = WSHED; M[r * W + W - 1] = WSHED;
    for (int c = 1; c < W - 1; c++) {
      int p = r * W + c;
      if (M[p] < 0) M[p] = 0;
      if (M[p]) continue;
      int l = 256, nn[4] = {p - 1, p + 1, p - W, p + W};
      for (int k = 0; k < 4; k++) if (M[nn[k]] > 0) { int t = cd(p, nn[k]); if (t < l) l = t; }
      if (l < 256) { qpush(&q[l], p); M[p] = INQ; }
    }
  }
  unsigned rng = 777;
  const int genlog = getenv("SPEC_GENLOG") != NULL;
  T = 0;
  for (;;) {
    L = 0;
    while (L < 256 && q[L].h == q[L].n) L++;
    if (L == 256) break;
    n = (int)(q[L].n - q[L].h);
    if (n > WIN) n = WIN;
    st_gens++;
    G = ++T;
    const long long gexec0 = st_exec;
    for (int i = 0; i < n; i++) { tpix[i] = q[L].v[q[L].h + i]; rank_of[tpix[i]] = i; rank_tag[tpix[i]] = G; }
    P = 0;
    int rounds = 0, pstart = 0;
    for (;;) {
      if (rounds) ++T;
      rounds++;
      // promote the items that became final after the previous round
      for (int i = pstart; i < P; i++) {
        Exec* e = &ex[(T - 1) & 1][i];
        for (int k = 0; k < e->n; k++) {
          Rec* r = &e->r[k];
          fin[r->pix] = ckey(G, i, 1, k);
          if (r->lab == WSHED) continue;
          int y = r->pix, nb[4] = {y - 1, y + 1, y - W, y + W};
          for (int d = 0; d < 4; d++) if ((r->dmask >> d) & 1) fin[nb[d]] = ckey(G, i, 0, 0);
        }
      }
      pstart = P;
      for (int i = P; i < n; i++) lastpar[i] = T & 1;
      for (int i = P; i < n; i++) top_pop(i);
      int nc = 0;
      for (int i = P; i < n; i++) order[nc++] = i;
      for (int k = nc - 1; k > 0; k--) { rng = rng * 1103515245u + 12345u; int a = (rng >> 8) % (k + 1); int t = order[k]; order[k] = order[a]; order[a] = t; }
      for (int k = 0; k < nc; k++) { cascade(order[k]); st_exec++; st_execpops += ex[T & 1][order[k]].n; }
      // stable prefix
      int newP = n;
      for (int i = P; i < n; i++) {
        Exec* e = &ex[T & 1][i];
        if (rounds == 1 || e->sig != prevsig[i] || e->ovf) { newP = i; break; }
      }
      for (int i = P; i < n; i++) prevsig[i] = ex[T & 1][i].sig;
      // items before newP unchanged since the previous round: their current results are final
      if (newP == n) { P = n; break; }
      // the first unstable item read only final inputs this round: an overflow there is genuine
      const int genuine = newP == P && rounds > 1 && ex[T & 1][newP].ovf == 1;
      P = newP;
      if (rounds >= 64 || genuine) break;
    }
    st_rounds += rounds;
    if (rounds > st_maxr) st_maxr = rounds;
    if (genlog) fprintf(stderr, "gen L=%d n=%d rounds=%d P=%d execs=%lld\n", L, n, rounds, P, st_exec - gexec0);
    int serial_item = (P < n && ex[lastpar[P] = T & 1][P].ovf == 1);  // overflow: the item runs serially after the commit
    // commit items 0..P-1: serial order = rank order, then each item's records in order
    for (int i = 0; i < P; i++) {
      // final results: parity of the round in which the item last executed
      Exec* e = NULL;
      // an item < pstart last ran in an earlier round: find its parity via fin of its pixel
      e = &ex[lastpar[i]][i];
      for (int k = 0; k < e->n; k++) {
        Rec* r = &e->r[k];
        M[r->pix] = r->lab;
        if (r->lab == WSHED) continue;
        int y = r->pix, nb[4] = {y - 1, y + 1, y - W, y + W};
        for (int d = 0; d < 4; d++)
          if ((r->dmask >> d) & 1) { M[nb[d]] = INQ; qpush(&q[cd(y, nb[d])], nb[d]); }
      }
    }
    q[L].h += P;
    if (serial_item) {  // the regular engine's job: pop the item, then its cascade to exhaustion
      st_serial++;
      int active = L;
      long long c0 = 0;
      for (;;) {
        while (active < 256 && q[active].h == q[active].n) active++;
        if (active >= L && c0 > 0) break;
        int y = q[active].v[q[active].h++];
        c0++;
        int nb[4] = {y - 1, y + 1, y - W, y + W}, lab = 0;
        for (int d = 0; d < 4; d++) { int v = M[nb[d]]; if (v > 0) lab = lab == 0 ? v : (lab == v ? v : WSHED); }
        M[y] = lab;
        if (lab == WSHED) continue;
        for (int d = 0; d < 4; d++) {
          if (M[nb[d]] != 0) continue;
          int t = cd(y, nb[d]);
          qpush(&q[t], nb[d]); M[nb[d]] = INQ;
          if (t < active) active = t;
        }
      }
      st_serialpops += c0;
    }
  }
  fwrite(M, 4, N, stdout);
  fprintf(stderr, "generations %lld rounds %lld (max %lld) executions %lld exec-pops %lld | serial items %lld pops %lld\n",
          st_gens, st_rounds, st_maxr, st_exec, st_execpops, st_serial, st_serialpops);
  return 0;
}
