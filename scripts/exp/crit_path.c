// Design study: how parallel is cv::watershed's exact order on a given frame?
//
// Runs the serial flood (OpenCV 3.4.2 order, as oracle/ws_oracle.c) and measures two depths:
//  * dataflow depth: depth(x) = 1 + max(depth of the pop that pushed x, depth of the last write
//    (push or pop) of each 4-neighbour state x reads) -- the critical path of any engine that
//    knew the order for free;
//  * nested-generation depth: the flood as a tree of sub-floods (a pop at level v opens the
//    sub-flood of everything popped after it below v); a flood's time is the sum over its FIFO
//    generations of 1 + the deepest sub-flood opened by that generation's items, i.e. an engine
//    that runs a generation's items and all their sub-floods in parallel (no conflicts).
// usage: crit_path H W < (bgr H*W*3, markers H*W int32)
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

// flood tree
typedef struct { int thr; int parent; long long acc; int cur_gen_max; int cur_gen; int cur_lvl; } Flood;
static Flood* F;
static int nf;

int main(int argc, char** argv) {
  H = atoi(argv[1]); W = atoi(argv[2]);
  size_t N = (size_t)H * W;
  uint8_t* img = malloc(N * 3);
  M = malloc(N * 4);
  if (fread(img, 1, N * 3, stdin) != N * 3 || fread(M, 4, N, stdin) != N) return 2;
  IMG = img;
  int32_t* dd = calloc(N, 4);       // dataflow depth of the last write of a pixel's state
  int32_t* pdep = calloc(N, 4);     // dataflow depth of the pusher of a queued pixel
  int32_t* pflood = calloc(N, 4);   // (leader) flood of the pusher's F-leader chain: see below
  int32_t* gen = calloc(N, 4);      // generation index of a leader within its flood's level phase
  int32_t* pgen = calloc(N, 4);     // generation of the pushing item's top ancestor (+1 = pushed item's gen)
  int32_t* plvl = calloc(N, 4);
  for (int c = 0; c < W; c++) { M[c] = WSHED; M[(H - 1) * W + c] = WSHED; }
  for (int r = 1; r < H - 1; r++) {
    M[r * W] = WSHED; M[r * W + W - 1] = WSHED;
    for (int c = 1; c < W - 1; c++) {
      int p = r * W + c;
      if (M[p] < 0) M[p] = 0;
      if (M[p]) continue;
      int l = 256, n[4] = {p - 1, p + 1, p - W, p + W};
      for (int k = 0; k < 4; k++) if (M[n[k]] > 0) { int t = cd(p, n[k]); if (t < l) l = t; }
      if (l < 256) { qpush(&q[l], p); M[p] = INQ; pgen[p] = -1; pflood[p] = 0; }
    }
  }
  // floods: stack of open floods; F[0] = top (thr 256)
  int cap = 1 << 20;
  F = malloc(sizeof(Flood) * cap);
  int* stk = malloc(sizeof(int) * 300);
  int sp = 0;
  F[0] = (Flood){256, -1, 0, 0, -1, -1};
  nf = 1;
  stk[sp++] = 0;
  // per pop: the flood it leads in, and its item id (the leader of the current flood that it
  // belongs to is itself).  For generation accounting we track, for each open flood, the current
  // (level, generation) phase and the max sub-flood depth of that generation's items.
  int32_t* leadsub = calloc(N, 4);  // flood index opened by pop x (S(x))
  int32_t* topanc = calloc(N, 4);   // for a pop inside some flood: its ancestor leader in each flood? (we store only the leader of the innermost flood)
  (void)topanc;
  long long pops = 0, maxdd = 0, ngens = 0, nfl_nonempty = 0;
  int active = 0;
  // close flood f: fold its accumulated depth into its parent's current generation
  #define FLUSH_GEN(f) do { if (F[f].cur_gen >= 0) { F[f].acc += 1 + F[f].cur_gen_max; ngens++; } } while (0)
  for (;;) {
    while (active < 256 && q[active].h == q[active].n) active++;
    if (active == 256) break;
    int v = active;
    int x = q[v].v[q[v].h++];
    pops++;
    // close sub-floods whose threshold <= v
    while (F[stk[sp - 1]].thr <= v) {
      int f = stk[--sp];
      FLUSH_GEN(f);
      int par = F[f].parent;
      if (F[f].acc > F[par].cur_gen_max) F[par].cur_gen_max = (int)F[f].acc;
      if (F[f].acc) nfl_nonempty++;
    }
    int f = stk[sp - 1];
    // generation of x within f's level-v phase: pushed by an item of the current generation at this
    // level (or inside its sub-flood) -> next generation; else generation 0 of the phase
    int g;
    if (F[f].cur_lvl != v) { FLUSH_GEN(f); F[f].cur_lvl = v; F[f].cur_gen = 0; F[f].cur_gen_max = 0; g = 0; }
    else {
      g = (pflood[x] == f && plvl[x] == v) ? pgen[x] + 1 : F[f].cur_gen;
      if (g < F[f].cur_gen) g = F[f].cur_gen;
      if (g > F[f].cur_gen) { FLUSH_GEN(f); F[f].cur_gen = g; F[f].cur_gen_max = 0; }
    }
    gen[x] = g;
    // dataflow depth
    int nb[4] = {x - 1, x + 1, x - W, x + W};
    int d = pdep[x];
    for (int k = 0; k < 4; k++) if (dd[nb[k]] > d) d = dd[nb[k]];
    d += 1;
    if (d > maxdd) maxdd = d;
    int lab = 0;
    for (int k = 0; k < 4; k++) {
      int t = M[nb[k]];
      if (t > 0) lab = lab == 0 ? t : (lab == t ? t : WSHED);
    }
    M[x] = lab;
    dd[x] = d;
    // open S(x)
    if (nf == cap) { cap *= 2; F = realloc(F, sizeof(Flood) * cap); }
    F[nf] = (Flood){v, f, 0, 0, -1, -1};
    leadsub[x] = nf;
    stk[sp++] = nf++;
    if (lab == WSHED) continue;
    // the item of flood f this pop belongs to is x itself (x leads in f); pops inside S(x) record
    // their pushes as coming from the top-level item whose generation they extend: we track that
    // by pflood/pgen/plvl of pushed pixels = (flood that receives them, generation, level)
    for (int k = 0; k < 4; k++) {
      int z = nb[k];
      if (M[z] != 0) continue;
      int t = cd(x, z);
      qpush(&q[t], z);
      if (t < active) active = t;
      M[z] = INQ;
      dd[z] = d;
      pdep[z] = d;
      // which flood will pop z: innermost open flood (incl. S(x)) with thr > t
      int s = sp - 1;
      while (F[stk[s]].thr <= t) s--;
      int fz = stk[s];
      pflood[z] = fz;
      plvl[z] = t;
      // generation of the item of fz that (transitively) made this push: if fz == the flood x leads
      // in, it is x's generation; if fz is deeper (S(x) or below) the push is at a lower level
      // (a new phase of that flood): generation 0
      if (fz == f) pgen[z] = g; else if (s + 1 < sp) {
        // fz is an ancestor-or-self flood: find the leader of fz on the stack path -- the flood
        // directly inside fz on the stack was opened by a leader of fz; use that leader's gen
        // stored in F? approximate with the fz's current generation
        pgen[z] = F[fz].cur_gen;
      } else pgen[z] = -1;
    }
  }
  while (sp > 0) {
    int f = stk[--sp];
    FLUSH_GEN(f);
    int par = F[f].parent;
    if (par >= 0 && F[f].acc > F[par].cur_gen_max) F[par].cur_gen_max = (int)F[f].acc;
  }
  fprintf(stderr, "pops %lld  dataflow depth %lld (%.0f pops/level)  nested-generation depth %lld  "
          "generations %lld  floods %d (non-empty %lld)\n",
          pops, maxdd, (double)pops / maxdd, F[0].acc, ngens, nf, nfl_nonempty);
  return 0;
}
