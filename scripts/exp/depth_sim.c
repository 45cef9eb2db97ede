// Design study: how many dependent "rounds" does a batch need if it is never cut at interrupts?
//
// Batch = the first n items of the lowest non-empty bucket L (n <= window).  The batch is run in
// serial order: each item pops, and an item that pushes below L runs its cascade (every level
// < L, to exhaustion) before the next item -- i.e. exactly cv::watershed's order.  For every item
// j we record depth(j) = 1 + max depth(i) over earlier items i of the same batch whose writes
// (their pop, their cascade's pops, the pixels they marked queued) are read by j (j's pop or its
// cascade's pops: the 4-neighbours of every pop).  Top-item -> top-item edges (k_resolve's
// in-kernel waits) are counted separately as free ("free" model) or as rounds ("all" model).
// Output: batches, sum over batches of max depth (rounds), cascade statistics.
// usage: depth_sim H W window < (bgr H*W*3, markers H*W int32)
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
static int64_t* wbatch;  // batch id of the last write
static int32_t* wdep_all;
static int32_t* wdep_free;
static uint8_t* wcasc;  // written by a cascade pop/push (1) or a top item (0)
static int32_t* wrank;
static long long bid;

// pop p at the current active level; returns 1 if it pushed below `lim`
static int cur_rank, cur_dall, cur_dfree, in_casc;
static int lvl_pushed_min;
static void readpx(int z) {
  if (wbatch[z] != bid || wrank[z] == cur_rank) return;
  int da = wdep_all[z] + 1;
  if (da > cur_dall) cur_dall = da;
  int df = wdep_free[z] + ((wcasc[z] || in_casc) ? 1 : 0);
  if (df > cur_dfree) cur_dfree = df;
}
static void writepx(int z) { wbatch[z] = bid; wrank[z] = cur_rank; wcasc[z] = (uint8_t)in_casc; wdep_all[z] = -1; }
static int pend[1 << 20], npend;  // written pixels of the current item (depth assigned at the end)

static void pop(int p, int* active) {
  int nb[4] = {p - 1, p + 1, p - W, p + W};
  for (int k = 0; k < 4; k++) readpx(nb[k]);
  int lab = 0;
  for (int k = 0; k < 4; k++) {
    int t = M[nb[k]];
    if (t > 0) lab = lab == 0 ? t : (lab == t ? t : WSHED);
  }
  M[p] = lab;
  writepx(p); pend[npend++] = p;
  if (lab == WSHED) return;
  for (int k = 0; k < 4; k++) {
    int z = nb[k];
    if (M[z] != 0) continue;
    int t = cd(p, z);
    qpush(&q[t], z);
    if (t < *active) *active = t;
    if (t < lvl_pushed_min) lvl_pushed_min = t;
    M[z] = INQ;
    writepx(z); pend[npend++] = z;
  }
}

int main(int argc, char** argv) {
  H = atoi(argv[1]); W = atoi(argv[2]);
  int WIN = argc > 3 ? atoi(argv[3]) : 4096;
  size_t N = (size_t)H * W;
  uint8_t* img = malloc(N * 3);
  M = malloc(N * 4);
  if (fread(img, 1, N * 3, stdin) != N * 3 || fread(M, 4, N, stdin) != N) return 2;
  IMG = img;
  wbatch = calloc(N, 8); wdep_all = calloc(N, 4); wdep_free = calloc(N, 4); wcasc = calloc(N, 1);
  wrank = calloc(N, 4);
  for (int c = 0; c < W; c++) { M[c] = WSHED; M[(H - 1) * W + c] = WSHED; }
  for (int r = 1; r < H - 1; r++) {
    M[r * W] = WSHED; M[r * W + W - 1] = WSHED;
    for (int c = 1; c < W - 1; c++) {
      int p = r * W + c;
      if (M[p] < 0) M[p] = 0;
      if (M[p]) continue;
      int l = 256, n[4] = {p - 1, p + 1, p - W, p + W};
      for (int k = 0; k < 4; k++) if (M[n[k]] > 0) { int t = cd(p, n[k]); if (t < l) l = t; }
      if (l < 256) { qpush(&q[l], p); M[p] = INQ; }
    }
  }
  long long batches = 0, rounds_all = 0, rounds_free = 0, pops = 0, casc = 0, cpops = 0, maxc = 0;
  long long hist[8] = {0};
  for (;;) {
    int L = 0;
    while (L < 256 && q[L].h == q[L].n) L++;
    if (L == 256) break;
    bid++; batches++;
    int n = (int)(q[L].n - q[L].h);
    if (n > WIN) n = WIN;
    int bmax_all = 0, bmax_free = 0;
    for (int i = 0; i < n; i++) {
      int p = q[L].v[q[L].h++];
      cur_rank = i; cur_dall = 1; cur_dfree = 1; in_casc = 0; npend = 0; lvl_pushed_min = 256;
      int active = L;
      pop(p, &active);
      pops++;
      if (active < L) {
        casc++;
        in_casc = 1;
        long long c0 = pops;
        for (;;) {
          while (active < L && q[active].h == q[active].n) active++;
          if (active >= L) break;
          int y = q[active].v[q[active].h++];
          pop(y, &active);
          pops++;
        }
        cpops += pops - c0;
        if (pops - c0 > maxc) maxc = pops - c0;
      }
      for (int k = 0; k < npend; k++) { wdep_all[pend[k]] = cur_dall; wdep_free[pend[k]] = cur_dfree; }
      if (cur_dall > bmax_all) bmax_all = cur_dall;
      if (cur_dfree > bmax_free) bmax_free = cur_dfree;
    }
    rounds_all += bmax_all; rounds_free += bmax_free;
    int b = 0; while (b < 7 && (1 << (b * 2)) < n) b++;
    hist[b]++;
  }
  fwrite(M, 4, N, stdout);
  fprintf(stderr, "window %d: batches %lld pops %lld (%.1f/batch) rounds(all) %lld rounds(cascade edges) %lld | cascades %lld cascade-pops %lld max %lld\n",
          WIN, batches, pops, (double)pops / batches, rounds_all, rounds_free, casc, cpops, maxc);
  return 0;
}
