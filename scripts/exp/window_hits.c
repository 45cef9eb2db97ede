// Design study: how often does cv::watershed's next pop fall inside a small window around the last
// window-loading pop?  A one-wave serial loop (k_serial / k_serial_multi) could hold the states of
// a block of tiles around the pop in its 64 lanes' registers and skip the memory round trip for
// every pop whose 4 neighbours (and itself) lie in the block.  Windows: aligned 3x3 tiles of TxT
// pixels centred on the tile of the loading pop (T = 4: 12x12 pixels).
// usage: window_hits H W [T] < (bgr, markers)
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
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
int main(int argc, char** argv) {
  H = atoi(argv[1]); W = atoi(argv[2]);
  const int T = argc > 3 ? atoi(argv[3]) : 4;
  size_t N = (size_t)H * W;
  uint8_t* img = malloc(N * 3);
  M = malloc(N * 4);
  if (fread(img, 1, N * 3, stdin) != N * 3 || fread(M, 4, N, stdin) != N) return 2;
  IMG = img;
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
  long long pops = 0, hits = 0, hits_prev_adj = 0;
  int wr0 = -1000000, wc0 = -1000000;  // window: rows [wr0, wr0 + 3T), cols [wc0, wc0 + 3T)
  int prev = -1;
  int active = 0;
  for (;;) {
    while (active < 256 && q[active].h == q[active].n) active++;
    if (active == 256) break;
    int x = q[active].v[q[active].h++];
    pops++;
    int r = x / W, c = x % W;
    // the pop needs rows r-1..r+1 at column c and columns c-1..c+1 at row r
    if (r - 1 >= wr0 && r + 1 < wr0 + 3 * T && c - 1 >= wc0 && c + 1 < wc0 + 3 * T) hits++;
    else { wr0 = (r / T - 1) * T; wc0 = (c / T - 1) * T; }
    if (prev >= 0 && (x == prev - 1 || x == prev + 1 || x == prev - W || x == prev + W)) hits_prev_adj++;
    prev = x;
    int nb[4] = {x - 1, x + 1, x - W, x + W};
    int lab = 0;
    for (int k = 0; k < 4; k++) { int t = M[nb[k]]; if (t > 0) lab = lab == 0 ? t : (lab == t ? t : WSHED); }
    M[x] = lab;
    if (lab == WSHED) continue;
    for (int k = 0; k < 4; k++) {
      int z = nb[k];
      if (M[z] != 0) continue;
      int t = cd(x, z);
      qpush(&q[t], z);
      if (t < active) active = t;
      M[z] = INQ;
    }
  }
  fprintf(stderr, "pops %lld: window %dx%d hits %.1f%%, next pop adjacent to the previous one %.1f%%\n", pops,
          3 * T, 3 * T, 100.0 * hits / pops, 100.0 * hits_prev_adj / pops);
  return 0;
}
