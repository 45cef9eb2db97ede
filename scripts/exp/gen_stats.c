// Design study: the speculative engine's generations on a frame, measured on the serial flood.
//
// Runs cv::watershed's serial order (as oracle/ws_oracle.c) and cuts it the way k_spec_round
// does: a generation = the whole lowest bucket L at a moment when every lower bucket is empty;
// item j's execution = its pop + its cascade (every pop below L until the flood is back at L).
// Per generation it records the items, the pops, the longest execution and the most live
// cascade entries (an execution's below-L queue), and prints histograms plus a cost model
//   gen cost = rounds * (round floor + longest execution * pop latency) + commit
// so that engine changes can be priced before they are built.
// usage: gen_stats H W [qcap] < (bgr H*W*3, markers H*W int32)
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
static int active = 0;
// per generation: the executions' pop counts, for the cap model
static long long *ex_pops = NULL, ex_n = 0, ex_cap = 0;
static long long *gen_start = NULL, gen_n = 0, gen_cap = 0;
static void ex_add(long long c) {
  if (ex_n == ex_cap) { ex_cap = ex_cap ? 2 * ex_cap : 1 << 20; ex_pops = realloc(ex_pops, ex_cap * 8); }
  ex_pops[ex_n++] = c;
}
static void gen_add(long long start) {
  if (gen_n == gen_cap) { gen_cap = gen_cap ? 2 * gen_cap : 1 << 12; gen_start = realloc(gen_start, gen_cap * 8); }
  gen_start[gen_n++] = start;
}
static long long live_below = 0;  // entries queued below the generation level

static void pop_one(int x, int L) {
  int nb[4] = {x - 1, x + 1, x - W, x + W};
  int lab = 0;
  for (int k = 0; k < 4; k++) {
    int t = M[nb[k]];
    if (t > 0) lab = lab == 0 ? t : (lab == t ? t : WSHED);
  }
  M[x] = lab;
  if (lab == WSHED) return;
  for (int k = 0; k < 4; k++) {
    int z = nb[k];
    if (M[z] != 0) continue;
    int t = cd(x, z);
    qpush(&q[t], z);
    if (t < active) active = t;
    if (t < L) live_below++;
    M[z] = INQ;
  }
}

int main(int argc, char** argv) {
  H = atoi(argv[1]); W = atoi(argv[2]);
  int qcap = argc > 3 ? atoi(argv[3]) : 32;
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
  long long gens = 0, pops = 0, sum_max = 0, ovf_gens = 0, ovf_execs = 0, big_gens = 0;
  long long hist_n[32] = {0}, hist_max[32] = {0}, pops_by_max[32] = {0};
  double cost[4] = {0, 0, 0, 0};
  // cost models (us): {round floor, pop latency, rounds, commit}
  const double mdl[4][4] = {{10, 2.0, 2.5, 30}, {10, 1.0, 2.5, 30}, {5, 0.5, 2.5, 15}, {5, 0.25, 2.0, 10}};
  long long serial_if_ovf = 0, ovf_pops = 0, hist_live[32] = {0}, pops_by_live[32] = {0};
  for (;;) {
    while (active < 256 && q[active].h == q[active].n) active++;
    if (active == 256) break;
    const int L = active;
    const long long n = (long long)(q[L].n - q[L].h);
    long long mx = 0, gp = 0;
    int govf = 0;
    gen_add(ex_n);
    for (long long j = 0; j < n; j++) {
      int x = q[L].v[q[L].h++];
      live_below = 0;
      long long c = 1, livemax = 0;
      pop_one(x, L);
      for (;;) {
        while (active < L && q[active].h == q[active].n) active++;
        if (active >= L) break;
        int y = q[active].v[q[active].h++];
        live_below--;
        pop_one(y, L);
        if (live_below > livemax) livemax = live_below;
        c++;
      }
      active = L;
      if (livemax > qcap) { govf = 1; ovf_execs++; ovf_pops += c; }
      { int bl = 0; while ((1ll << (bl + 1)) <= livemax && bl < 31) bl++; hist_live[bl]++; pops_by_live[bl] += c; }
      if (c > mx) mx = c;
      gp += c;
      ex_add(c);
    }
    gens++;
    pops += gp;
    sum_max += mx;
    if (govf) { ovf_gens++; serial_if_ovf += gp; }
    int bn = 0; while ((1ll << (bn + 1)) <= n && bn < 31) bn++;
    int bm = 0; while ((1ll << (bm + 1)) <= mx && bm < 31) bm++;
    hist_n[bn]++; hist_max[bm]++; pops_by_max[bm] += gp;
    if (n >= 4096) big_gens++;
    for (int k = 0; k < 4; k++) cost[k] += mdl[k][2] * (mdl[k][0] + mx * mdl[k][1]) + mdl[k][3];
  }
  fprintf(stderr, "pops %lld generations %lld (%.1f pops/gen, %lld with >= 4096 items) sum of longest executions %lld\n",
          pops, gens, (double)pops / gens, big_gens, sum_max);
  fprintf(stderr, "generations with an execution over %d live cascade entries: %lld (%lld executions, %lld pops)\n",
          qcap, ovf_gens, ovf_execs, serial_if_ovf);
  fprintf(stderr, "pops inside the overflowing executions: %lld\n", ovf_pops);
  fprintf(stderr, "log2 bin of the most live cascade entries: executions (pops)\n");
  for (int b = 0; b < 32; b++)
    if (hist_live[b]) fprintf(stderr, "  %2d : %10lld (%lld)\n", b, hist_live[b], pops_by_live[b]);
  fprintf(stderr, "log2 bin : gens by items | gens by longest execution (pops in them)\n");
  for (int b = 0; b < 32; b++)
    if (hist_n[b] || hist_max[b])
      fprintf(stderr, "  %2d : %8lld | %8lld (%lld)\n", b, hist_n[b], hist_max[b], pops_by_max[b]);
  for (int k = 0; k < 4; k++)
    fprintf(stderr, "model floor %.0f us, %.2f us/pop, %.1f rounds, commit %.0f us: %.1f ms\n", mdl[k][0], mdl[k][1],
            mdl[k][2], mdl[k][3], cost[k] / 1e3);
  // cap model: executions of more than `cap` pops go to serial pops (the prefix before them is a
  // committed segment, the rest of the bucket a new one); argv[4..]: t_lane t_ser floor rounds commit fallback (us)
  double tl = argc > 4 ? atof(argv[4]) : 2.0, ts = argc > 5 ? atof(argv[5]) : 0.6, fl = argc > 6 ? atof(argv[6]) : 15;
  double rr = argc > 7 ? atof(argv[7]) : 2.7, cm = argc > 8 ? atof(argv[8]) : 30, fo = argc > 9 ? atof(argv[9]) : 50;
  gen_add(ex_n);
  const long long caps[] = {32, 64, 128, 256, 512, 1024, 2048, 8448, 1ll << 40};
  for (int ci = 0; ci < 9; ci++) {
    const long long cap = caps[ci];
    double t = 0, tser = 0;
    long long segs = 0, fb = 0;
    for (long long g = 0; g + 1 < gen_n; g++) {
      long long mx = 0, nseg = 0;
      for (long long e = gen_start[g]; e < gen_start[g + 1]; e++) {
        if (ex_pops[e] > cap) {
          if (nseg) { t += rr * (fl + mx * tl) + cm; segs++; }
          t += fo + ex_pops[e] * ts; tser += ex_pops[e] * ts; fb++;
          mx = 0; nseg = 0;
        } else {
          if (ex_pops[e] > mx) mx = ex_pops[e];
          nseg++;
        }
      }
      if (nseg) { t += rr * (fl + mx * tl) + cm; segs++; }
    }
    fprintf(stderr, "cap %lld pops: %.1f ms (serial %.1f ms, %lld fallbacks, %lld segments) [t_lane %.2f t_ser %.2f floor %.0f rounds %.1f commit %.0f fallback %.0f us]\n",
            cap, t / 1e3, tser / 1e3, fb, segs, tl, ts, fl, rr, cm, fo);
  }
  return 0;
}
