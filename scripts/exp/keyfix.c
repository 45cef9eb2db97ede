// Design study: cv::watershed's labels as the fixed point of LOCAL rules on "pop keys".
//
// The serial order (pop the oldest entry of the lowest non-empty of 256 FIFO buckets) is the
// lexicographic order of a nested key K(x):
//   * a pop y at level v opens the sub-flood S(y) (every later pop below v, up to the next pop at
//     >= v); a pixel pushed by p at level t is popped as a "leader" of the innermost flood, among
//     S(p), the flood p leads in, and that flood's enclosing ones, whose threshold exceeds t;
//   * leaders of one flood pop in (level, push time, direction) order, push time = the pusher's
//     own key (phase-1 entries first, in raster order), and a flood's opener precedes all of it.
// So whether a pops before b is decided by walking the pusher / opener pointers (cmp below), and
// every pixel's pusher (its earliest non-WSHED neighbour), level, flood and label (the fold of the
// neighbours popped before it) are local functions of its neighbours.  This program iterates those
// rules Jacobi-style from the phase-1 queue to the fixed point and checks it against the serial
// flood: the sweep count is the parallel depth of an engine built on the rules.
// usage: keyfix H W < (bgr H*W*3, markers H*W int32)
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define WSHED (-1)
#define INQ (-2)
static int H, W;
static const uint8_t* IMG;
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
static void serial(int32_t* M) {
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
  int active = 0;
  for (;;) {
    while (active < 256 && q[active].h == q[active].n) active++;
    if (active == 256) break;
    int x = q[active].v[q[active].h++];
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
}

// per-pixel rule state (old = read, nw = written each sweep)
typedef struct { int32_t *pi, *F, *lab; uint8_t *v, *dir, *def; uint16_t* fd; } St;
static St A, B;
static uint8_t *kind;  // 0 interior free, 1 marker, 2 border
static int32_t* M0;
static uint8_t *p1, *v1;
static long long csteps, ccalls, cfail;
#define LIMIT 1024

// does a pop before b (-1), after (+1), unknown (0)?  a, b defined, non-marker
static int cmp(const St* S, int a, int b) {
  ccalls++;
  for (int it = 0; it < LIMIT; it++) {
    csteps++;
    if (a == b) return 0;
    int fa = 0, fb = 0;
    for (int y = S->F[a]; y >= 0 && fa < 300; y = S->F[y]) fa++;
    for (int y = S->F[b]; y >= 0 && fb < 300; y = S->F[y]) fb++;
    int a0 = a, b0 = b;
    while (fa > fb) { a = S->F[a]; fa--; }
    while (fb > fa) { b = S->F[b]; fb--; }
    if (a == b) return (a == a0) ? -1 : ((b == b0) ? 1 : 0);
    int g = 0;
    while (S->F[a] != S->F[b] && g++ < 300) { a = S->F[a]; b = S->F[b]; csteps++; if (a < 0 || b < 0) return 0; }
    if (a == b) return 0;
    if (S->v[a] != S->v[b]) return S->v[a] < S->v[b] ? -1 : 1;
    int pa = S->pi[a], pb = S->pi[b];
    if (pa < 0 && pb < 0) return a < b ? -1 : 1;
    if (pa < 0) return -1;
    if (pb < 0) return 1;
    if (pa == pb) return S->dir[a] < S->dir[b] ? -1 : 1;
    if (!S->def[pa] || !S->def[pb]) return 0;
    a = pa; b = pb;
  }
  cfail++;
  return 0;
}

int main(int argc, char** argv) {
  H = atoi(argv[1]); W = atoi(argv[2]);
  size_t N = (size_t)H * W;
  uint8_t* img = malloc(N * 3);
  M0 = malloc(N * 4);
  if (fread(img, 1, N * 3, stdin) != N * 3 || fread(M0, 4, N, stdin) != N) return 2;
  IMG = img;
  int32_t* ref = malloc(N * 4);
  memcpy(ref, M0, N * 4);
  serial(ref);
  St* S[2] = {&A, &B};
  for (int s = 0; s < 2; s++) {
    S[s]->pi = malloc(N * 4); S[s]->F = malloc(N * 4); S[s]->lab = calloc(N, 4);
    S[s]->v = calloc(N, 1); S[s]->dir = calloc(N, 1); S[s]->def = calloc(N, 1); S[s]->fd = calloc(N, 2);
  }
  kind = calloc(N, 1); p1 = calloc(N, 1); v1 = calloc(N, 1);
  for (size_t p = 0; p < N; p++) {
    int r = (int)(p / W), c = (int)(p % W);
    if (r == 0 || c == 0 || r == H - 1 || c == W - 1) kind[p] = 2;
    else if (M0[p] > 0) kind[p] = 1;
  }
  for (int r = 1; r < H - 1; r++)
    for (int c = 1; c < W - 1; c++) {
      int p = r * W + c;
      if (kind[p]) continue;
      int l = 256, n[4] = {p - 1, p + 1, p - W, p + W};
      for (int k = 0; k < 4; k++) if (kind[n[k]] == 1) { int t = cd(p, n[k]); if (t < l) l = t; }
      if (l < 256) { p1[p] = 1; v1[p] = (uint8_t)l; }
    }
  const int off[4] = {-1, 1, -W, W};  // L, R, T, B: the serial push order
  int cur = 0, sweeps = 0;
  uint8_t* act = malloc(N); uint8_t* nact = calloc(N, 1);
  memset(act, 1, N);
  const int FULL = getenv("FULL") ? atoi(getenv("FULL")) : 1;
  int full_clean = 0;
  long long evals = 0;
  for (;;) {
    St* O = S[cur];
    const int rb = getenv("RB") != 0;
    St* Nw = (getenv("GS") || rb) ? O : S[cur ^ 1];
    long long changes = 0;
    for (int half = 0; half < (rb ? 2 : 1); half++)
    for (int r = 1; r < H - 1; r++)
      for (int c = 1; c < W - 1; c++) {
        int x = r * W + c;
        if (kind[x]) continue;
        if (rb && ((r + c) & 1) != half) continue;
        if (!act[x] && (sweeps % FULL) != 0) continue;
        int pi = -1, v = 0, dir = 0, F = -1, def = 0, fd = 0;
        if (p1[x]) { def = 1; v = v1[x]; }
        else {
          int best = -1, bd = 0;
          for (int d = 0; d < 4; d++) {
            int n = x - off[d];  // x = n + off[d]: n pushes x in direction d
            if (kind[n] || !O->def[n] || O->lab[n] <= 0) continue;
            if (best < 0 || cmp(O, n, best) < 0) { best = n; bd = d; }
          }
          if (best >= 0 && getenv("STRICT")) {
            // the pusher must be provably earlier than every other candidate it beat (a definite
            // comparison): a candidate set with an undecidable pair (a transient pusher cycle)
            // leaves x undefined this sweep, so cycles cannot sustain themselves
            for (int d = 0; d < 4 && best >= 0; d++) {
              int n = x - off[d];
              if (n == best || kind[n] || !O->def[n] || O->lab[n] <= 0) continue;
              if (cmp(O, best, n) >= 0) best = -1;
            }
          }
          if (best >= 0) {
            def = 1; pi = best; dir = bd; v = cd(x, best);
            if (v < O->v[best]) F = best;
            else { int y = O->F[best], g = 0; while (y >= 0 && O->v[y] <= v && g++ < 300) y = O->F[y]; F = y; }
            fd = F < 0 ? 0 : O->fd[F] + 1;
          }
        }
        int lab = 0;
        if (def) {
          // x's own new key, visible to cmp through the old arrays for this one evaluation
          int32_t spi = O->pi[x], sF = O->F[x]; uint8_t sv = O->v[x], sd = O->dir[x], sdef = O->def[x];
          uint16_t sfd = O->fd[x];
          O->pi[x] = pi; O->F[x] = F; O->v[x] = (uint8_t)v; O->dir[x] = (uint8_t)dir; O->def[x] = 1; O->fd[x] = (uint16_t)fd;
          for (int d = 0; d < 4; d++) {
            int n = x + off[d], t = 0;
            if (kind[n] == 1) t = M0[n];
            else if (kind[n] == 0 && O->def[n] && O->lab[n] > 0 && cmp(O, n, x) < 0) t = O->lab[n];
            if (t > 0) lab = lab == 0 ? t : (lab == t ? t : WSHED);
          }
          O->pi[x] = spi; O->F[x] = sF; O->v[x] = sv; O->dir[x] = sd; O->def[x] = sdef; O->fd[x] = sfd;
          if (lab == 0) lab = WSHED;  // transient: the pusher is not (yet) earlier
          evals++;
        }
        if (def != O->def[x] || pi != O->pi[x] || v != O->v[x] || lab != O->lab[x] || F != O->F[x] || dir != O->dir[x]) {
          changes++;
          if (getenv("DBG") && sweeps >= atoi(getenv("DBG")) && sweeps < atoi(getenv("DBG")) + 4)
            fprintf(stderr, "s%d x=(%d,%d) def %d->%d pi %d->%d v %d->%d lab %d->%d F %d->%d ref %d\n", sweeps, r, c,
                    O->def[x], def, O->pi[x] < 0 ? -1 : (O->pi[x] == x - 1 ? 0 : O->pi[x] == x + 1 ? 1 : O->pi[x] == x - W ? 2 : 3),
                    pi < 0 ? -1 : (pi == x - 1 ? 0 : pi == x + 1 ? 1 : pi == x - W ? 2 : 3), O->v[x], v, O->lab[x], lab,
                    O->F[x], F, ref[x]);
          nact[x] = 1;
          for (int d = 0; d < 4; d++) nact[x + off[d]] = 1;
        }
        Nw->def[x] = (uint8_t)def; Nw->pi[x] = pi; Nw->v[x] = (uint8_t)v; Nw->dir[x] = (uint8_t)dir;
        Nw->F[x] = F; Nw->lab[x] = lab; Nw->fd[x] = (uint16_t)fd;
      }
    if (!getenv("GS") && !getenv("RB")) cur ^= 1;
    { uint8_t* t = act; act = nact; nact = t; memset(nact, 0, N); }
    if ((sweeps % FULL) == 0 && changes == 0) full_clean = 1;
    sweeps++;
    if ((changes == 0 && (FULL == 1 || full_clean)) || sweeps > 30000) break;
    if (changes == 0 && FULL > 1) sweeps = (sweeps + FULL - 1) / FULL * FULL;  // next sweep: a full one
    if (sweeps % 20 == 0 || sweeps < 10) fprintf(stderr, "  sweep %d changes %lld cmp steps/call %.2f unresolved %lld\n", sweeps, changes, (double)csteps / (ccalls ? ccalls : 1), cfail);
  }
  St* R = S[cur];
  long long bad = 0;
  for (size_t p = 0; p < N; p++) {
    int got = kind[p] == 2 ? WSHED : kind[p] == 1 ? M0[p] : (R->def[p] ? R->lab[p] : 0);
    if (got != ref[p]) bad++;
  }
  fprintf(stderr, "sweeps %d  mismatches %lld  evals %lld (%.1f per px)  cmp calls %lld, steps/call %.2f, unresolved %lld\n",
          sweeps, bad, evals, (double)evals / N, ccalls, (double)csteps / (ccalls ? ccalls : 1), cfail);
  return 0;
}
