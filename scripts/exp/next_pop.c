/* Design study (round 4): could a cascade pop's neighbour loads be issued one pop early?
 * In k_spec_round a lane's next cascade pop is the smallest key of its queue AFTER the current
 * pop's pushes.  If it is usually a key that was already queued before them, the loads of the
 * queue's second-smallest key can be in flight while the current pop is decided.  Serial flood
 * (the oracle's order, oracle/ws_oracle.c), generations as in spec_kernels.hip: the lowest bucket
 * L at the generation's start; pops below L are cascade pops.  For every cascade pop: was it
 * pushed by the pop right before it (a miss for such a prefetch) or queued earlier (a hit)?
 * usage: next_pop frame.bgr frame.mk rows cols   (raw BGR u8 / int32 markers, as numpy tofile)
 * Round 4 (synth frames): cascade pops queued before the previous pop's pushes -- random 1024^2
 * 37.6%, mosaic+noise 1024^2 25.9%, random 4096^2 45.8%, mosaic+noise 4096^2 25.7%; the rest were
 * pushed by the pop right before them (first pops of cascades 8-62%, preemptions 13-46%).  The
 * kernel variant that decides the next pop before touching the queue (profiles/
 * r04n_ab_next_pop_early.log) measured slower: random 4096^2 1472 -> 1737 ms. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

static int cd(const uint8_t* a, const uint8_t* b) {
  int m = abs(a[0] - b[0]);
  if (abs(a[1] - b[1]) > m) m = abs(a[1] - b[1]);
  if (abs(a[2] - b[2]) > m) m = abs(a[2] - b[2]);
  return m;
}

int main(int argc, char** argv) {
  if (argc < 5) return 2;
  const int R = atoi(argv[3]), C = atoi(argv[4]);
  const size_t N = (size_t)R * C;
  uint8_t* img = malloc(3 * N);
  int32_t* M = malloc(4 * N);
  int32_t* who = malloc(4 * N);  /* pop index that pushed the pixel */
  FILE* f = fopen(argv[1], "rb");
  if (!f || fread(img, 1, 3 * N, f) != 3 * N) return 3;
  fclose(f);
  f = fopen(argv[2], "rb");
  if (!f || fread(M, 4, N, f) != N) return 3;
  fclose(f);
  int32_t* q[256];
  size_t qh[256] = {0}, ql[256] = {0}, qc[256];
  for (int i = 0; i < 256; i++) { qc[i] = 1024; q[i] = malloc(4 * qc[i]); }
#define PUSH(t, v) do { if (ql[t] == qc[t]) { qc[t] *= 2; q[t] = realloc(q[t], 4 * qc[t]); } q[t][ql[t]++] = (v); } while (0)
  for (int c = 0; c < C; c++) M[c] = M[(size_t)(R - 1) * C + c] = -1;
  for (int r = 1; r < R - 1; r++) {
    M[(size_t)r * C] = M[(size_t)r * C + C - 1] = -1;
    for (int c = 1; c < C - 1; c++) {
      size_t i = (size_t)r * C + c;
      if (M[i] < 0) M[i] = 0;
      if (M[i]) continue;
      int lv = 256;
      const uint8_t* p = img + 3 * i;
      if (M[i - 1] > 0 && cd(p, p - 3) < lv) lv = cd(p, p - 3);
      if (M[i + 1] > 0 && cd(p, p + 3) < lv) lv = cd(p, p + 3);
      if (M[i - C] > 0 && cd(p, p - 3 * C) < lv) lv = cd(p, p - 3 * C);
      if (M[i + C] > 0 && cd(p, p + 3 * C) < lv) lv = cd(p, p + 3 * C);
      if (lv < 256) { PUSH(lv, (int32_t)i); M[i] = -2; who[i] = -1; }
    }
  }
  long long pops = 0, cpops = 0, hit = 0, miss_first = 0, miss_prev = 0, qsz1 = 0;
  int genL = 256, active = 0;
  while (active < 256 && qh[active] == ql[active]) active++;
  long long k = 0;
  while (active < 256) {
    if (qh[active] == ql[active]) {
      while (active < 256 && qh[active] == ql[active]) active++;
      if (active == 256) break;
    }
    const int32_t i = q[active][qh[active]++];
    if (active > genL || genL == 256) genL = active;  /* the generation's bucket ran out */
    if (active < genL) {  /* a cascade pop */
      ++cpops;
      if (who[i] == k - 1) {
        /* pushed by the pop right before: the first pop after the top pop, or a preemption */
        long long before = 0;  /* keys queued below L before that pop's pushes */
        for (int t = 0; t < genL; t++) before += (long long)(ql[t] - qh[t]);
        if (before == 0) ++miss_first;
        else ++miss_prev;
      } else {
        ++hit;
      }
    }
    ++pops;
    const int r = i / C, c = i - r * C;
    int lab = 0;
    const int32_t nb[4] = {M[i - 1], M[i + 1], M[i - C], M[i + C]};
    for (int d = 0; d < 4; d++)
      if (nb[d] > 0) lab = lab == 0 ? nb[d] : (nb[d] != lab ? -1 : lab);
    M[i] = lab;
    if (lab != -1) {
      const int di[4] = {-1, 1, -C, C};
      for (int d = 0; d < 4; d++) {
        const int32_t z = i + di[d];
        if (M[z] != 0) continue;
        const int t = cd(img + 3 * (size_t)i, img + 3 * (size_t)z);
        PUSH(t, z);
        who[z] = (int32_t)k;
        M[z] = -2;
        if (t < active) active = t;
      }
    }
    ++k;
    (void)r; (void)c; (void)qsz1;
  }
  printf("%s: pops %lld, cascade pops %lld (%.1f%%): queued earlier %.1f%%, pushed by the previous pop "
         "%.1f%% (first of a cascade or after an emptied queue %.1f%%, preempting queued keys %.1f%%)\n",
         argv[1], pops, cpops, 100.0 * cpops / pops, 100.0 * hit / cpops, 100.0 * (miss_first + miss_prev) / cpops,
         100.0 * miss_first / cpops, 100.0 * miss_prev / cpops);
  return 0;
}
