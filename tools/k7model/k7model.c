// CPU model of K7's LZ77 parse and code size (hbx_deflate.hip), to compare
// compression-ratio variants without a GPU.  Not the product and not a
// checker: it estimates sizes only (dynamic Huffman code lengths by a plain
// length-limited Huffman build, header approximated), so variants are
// compared with each other and with zlib -6 on the same bytes.
//
// Variants (flags):
//   -w WAYS     candidates per hash (latest position per residue mod WAYS)
//   -b BITS     hash bits
//   -r RANGE    bytes per thread's parse range (64 in K7; 0 = whole segment,
//               i.e. matches may cross thread ranges)
//   -s SEG      segment bytes (32768 in K7)
//   -H          history: the previous segment of the block is in the window
//   -h HLEN     history of HLEN bytes before the segment (within the block)
//   -m MIN      minimum match (4 in K7; 3 allowed by deflate)
//   -l LAZY     lazy look-ahead steps (1 in K7)
//   -B BLOCK    block (chunk) bytes: segments of a block share history
//   -F          FIFO buckets (the WAYS latest positions per hash)
//   -f D4 / -g D5  length-4 / -5 matches farther than D4 / D5 are taken as literals
//   -P 1        flexible parsing: a match is cut where the next one reaches farthest
//   -S SHARE    segments that share one dynamic code and header (1 in K7)
//   -x W2       a second FIFO table of W2 ways keyed by K2 bytes (-k K2, -y BITS2)
//   cc -O2 -o k7model k7model.c -lm ; ./k7model [flags] < corpus
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

static int WAYS = 4, HBITS = 11, RANGE = 64, SEG = 32768, HIST = 0, HLEN = 0, MINM = 4, LAZY = 1, ROUND = 512;
static long BLOCK = 4 << 20;
static int W2 = 0, K2 = 8, B2 = 11, FAR4 = 0, FAR5 = 0, FLEX = 0;
static int SHARE = 1;  // -S: segments that share one dynamic code (and header)
static double hdr_total = 0;
static int FIFO = 0;  // -F: a bucket keeps its WAYS latest positions (a per-bucket counter) instead of one per residue
static uint32_t* fcnt;
static void ins(uint32_t* tab, uint32_t h, int rel) {
  if (FIFO) tab[h * WAYS + (fcnt[h]++ % WAYS)] = (uint32_t)(rel + 1);
  else tab[h * WAYS + ((unsigned)rel % WAYS)] = (uint32_t)(rel + 1);
}

static uint32_t rd4(const uint8_t* p) { uint32_t x; memcpy(&x, p, 4); return x; }
static uint32_t* fcnt2;
static uint32_t hsh2(const uint8_t* p) {
  uint32_t a = rd4(p), b = rd4(p + 4);
  if (K2 < 8) b &= (1u << (8 * (K2 - 4))) - 1u;
  return ((a * 0x9E3779B1u) ^ (b * 0x85EBCA77u)) >> (32 - B2);
}
static void ins2(uint32_t* tab, uint32_t h, int rel) { tab[h * W2 + (fcnt2[h]++ % W2)] = (uint32_t)(rel + 1); }
static uint32_t hsh(uint32_t x, int minm) {
  if (minm == 3) x &= 0xFFFFFFu;
  return (x * 0x9E3779B1u) >> (32 - HBITS);
}
static int mlen(const uint8_t* a, const uint8_t* b, int lim) {
  int n = 0;
  while (n < lim && a[n] == b[n]) n++;
  return n;
}

// length-limited Huffman code lengths (halve frequencies until depth <= 15)
typedef struct { long w; int l, r, sym; } Node;
static void depths(Node* nd, int i, int d, int* len) {
  if (nd[i].sym >= 0) { len[nd[i].sym] = d ? d : 1; return; }
  depths(nd, nd[i].l, d + 1, len);
  depths(nd, nd[i].r, d + 1, len);
}
static int cmpw(const void* a, const void* b) {
  long x = ((const Node*)a)->w, y = ((const Node*)b)->w;
  return x < y ? -1 : x > y;
}
static void huff(const long* f, int n, int lim, int* len) {
  long g[320];
  for (int i = 0; i < n; i++) g[i] = f[i];
  for (;;) {
    Node nd[700];
    int m = 0;
    for (int i = 0; i < n; i++) { len[i] = 0; if (g[i]) { nd[m].w = g[i]; nd[m].sym = i; nd[m].l = nd[m].r = -1; m++; } }
    if (m == 0) return;
    if (m == 1) { len[nd[0].sym] = 1; return; }
    qsort(nd, m, sizeof(Node), cmpw);
    // two-queue merge
    int leaf = 0, in0 = m, in1 = m;
    while ((m - leaf) + (in1 - in0) > 1) {
      int pick[2];
      for (int k = 0; k < 2; k++) {
        if (leaf < m && (in0 == in1 || nd[leaf].w <= nd[in0].w)) pick[k] = leaf++;
        else pick[k] = in0++;
      }
      nd[in1].w = nd[pick[0]].w + nd[pick[1]].w;
      nd[in1].l = pick[0]; nd[in1].r = pick[1]; nd[in1].sym = -1;
      in1++;
    }
    depths(nd, in1 - 1, 0, len);
    int mx = 0;
    for (int i = 0; i < n; i++) if (len[i] > mx) mx = len[i];
    if (mx <= lim) return;
    for (int i = 0; i < n; i++) if (g[i]) g[i] = (g[i] + 1) / 2;
  }
}
// exact dynamic header bits (RFC 1951 §3.2.7): run-length coded code lengths
// under a length-7 code-length code
static double hdr_bits(const int* ll, const int* dl, int hlit, int hdist) {
  static const int ord[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
  int seq[320], n = 0;
  for (int i = 0; i < hlit; i++) seq[n++] = ll[i];
  for (int i = 0; i < hdist; i++) seq[n++] = dl[i];
  long f[19] = {0};
  double extra = 0;
  for (int i = 0; i < n;) {
    int j = i;
    while (j < n && seq[j] == seq[i]) j++;
    int r = j - i;
    if (seq[i] == 0) {
      while (r >= 11) { int q = r > 138 ? 138 : r; f[18]++; extra += 7; r -= q; }
      if (r >= 3) { f[17]++; extra += 3; r = 0; }
      f[0] += r;
    } else {
      f[seq[i]]++; r--;
      while (r >= 3) { int q = r > 6 ? 6 : r; f[16]++; extra += 2; r -= q; }
      f[seq[i]] += r;
    }
    i = j;
  }
  int cl[19];
  huff(f, 19, 7, cl);
  int hclen = 4;
  for (int k = 0; k < 19; k++) if (cl[ord[k]]) hclen = k + 1 > hclen ? k + 1 : hclen;
  double b = 3 + 14 + 3.0 * hclen + extra;
  for (int k = 0; k < 19; k++) b += (double)f[k] * cl[k];
  return b;
}
static void lsym(int L, int* s, int* e) {
  if (L <= 10) { *s = 254 + L; *e = 0; return; }
  if (L == 258) { *s = 285; *e = 0; return; }
  int l = L - 3, ne = 31 - __builtin_clz(l) - 2;
  *s = 257 + 4 * (ne + 1) + ((l >> ne) & 3); *e = ne;
}
static void dsym(int D, int* s, int* e) {
  int d = D - 1;
  if (d < 4) { *s = d; *e = 0; return; }
  int ne = 31 - __builtin_clz(d) - 1;
  *s = 2 * (ne + 1) + ((d >> ne) & 1); *e = ne;
}

int main(int argc, char** argv) {
  int c;
  while ((c = getopt(argc, argv, "w:b:r:s:Hh:m:l:B:R:Fx:k:y:f:g:P:S:")) != -1) {
    if (c == 'P') FLEX = atoi(optarg);
    if (c == 'S') SHARE = atoi(optarg);
    if (c == 'f') FAR4 = atoi(optarg);
    if (c == 'g') FAR5 = atoi(optarg);
    if (c == 'x') W2 = atoi(optarg);
    if (c == 'k') K2 = atoi(optarg);
    if (c == 'y') B2 = atoi(optarg);
    if (c == 'h') { HIST = 1; HLEN = atoi(optarg); }
    if (c == 'F') FIFO = 1;
    if (c == 'w') WAYS = atoi(optarg);
    if (c == 'b') HBITS = atoi(optarg);
    if (c == 'r') RANGE = atoi(optarg);
    if (c == 's') SEG = atoi(optarg);
    if (c == 'H') HIST = 1;
    if (c == 'm') MINM = atoi(optarg);
    if (c == 'l') LAZY = atoi(optarg);
    if (c == 'B') BLOCK = atol(optarg);
    if (c == 'R') ROUND = atoi(optarg);
  }
  size_t cap = 1 << 26, n = 0;
  uint8_t* buf = malloc(cap + 1024);
  size_t k;
  while ((k = fread(buf + n, 1, cap - n, stdin)) > 0) { n += k; if (n == cap) { cap *= 2; buf = realloc(buf, cap + 1024); } }
  memset(buf + n, 0, 1024);
  const int nh = 1 << HBITS;
  uint32_t* tab = malloc(sizeof(uint32_t) * nh * WAYS);
  fcnt = malloc(sizeof(uint32_t) * nh);
  const int nh2 = 1 << B2;
  uint32_t* tab2 = malloc(sizeof(uint32_t) * nh2 * (W2 ? W2 : 1));
  uint32_t* snap2 = malloc(sizeof(uint32_t) * nh2 * (W2 ? W2 : 1));
  fcnt2 = malloc(sizeof(uint32_t) * nh2);
  int* cd = malloc(sizeof(int) * (SEG + 8));
  double total_bits = 0;
  long nseg = 0;
  for (size_t b0 = 0; b0 < n; b0 += BLOCK) {
    long fl[288] = {0}, fd[32] = {0};
    long extra = 0;
    int in_group = 0;
    const size_t bl = (n - b0 < (size_t)BLOCK) ? n - b0 : (size_t)BLOCK;
    const uint8_t* blk = buf + b0;
    for (size_t s0 = 0; s0 < bl; s0 += SEG) {
      const int sn = (int)((bl - s0 < (size_t)SEG) ? bl - s0 : (size_t)SEG);
      const uint8_t* sg = blk + s0;
      // window start (relative to sg): -SEG with history, else 0
      const int hl = HLEN ? HLEN : SEG;
      const int wlo = (HIST && s0 >= (size_t)hl) ? -hl : (HIST ? -(int)s0 : 0);
      memset(tab, 0, sizeof(uint32_t) * nh * WAYS);
      memset(fcnt, 0, sizeof(uint32_t) * nh);
      if (W2) {
        memset(tab2, 0, sizeof(uint32_t) * nh2 * W2);
        memset(fcnt2, 0, sizeof(uint32_t) * nh2);
      }
      // history positions inserted first (all, in order)
      for (int p = wlo; p < 0; p++) {
        if (p + 4 > 0 + sn && 0) break;
        uint32_t h = hsh(rd4(sg + p), MINM);
        ins(tab, h, p - wlo);
        if (W2 && p + K2 <= sn) ins2(tab2, hsh2(sg + p), p - wlo);
      }
      // candidates in rounds: reads see the table as of the round's start
      uint32_t* snap = malloc(sizeof(uint32_t) * nh * WAYS);
      for (int r0 = 0; r0 < sn; r0 += ROUND) {
        memcpy(snap, tab, sizeof(uint32_t) * nh * WAYS);
        if (W2) memcpy(snap2, tab2, sizeof(uint32_t) * nh2 * W2);
        for (int p = r0; p < r0 + ROUND && p < sn; p++) {
          cd[p] = 0;
          if (p + MINM > sn) continue;
          uint32_t x = rd4(sg + p);
          uint32_t h = hsh(x, MINM);
          int bestl = 0, bestd = 0;
          for (int w = 0; w < WAYS; w++) {
            uint32_t v = snap[h * WAYS + w];
            if (!v) continue;
            int q = (int)v - 1 + wlo;
            if (q >= p || p - q > 32768) continue;  // deflate's window
            int lim = sn - p < 258 ? sn - p : 258;
            int L = mlen(sg + p, sg + q, lim);
            if (L >= MINM && (L > bestl || (L == bestl && p - q < bestd))) { bestl = L; bestd = p - q; }
          }
          if (W2 && p + K2 <= sn) {
            const uint32_t h2 = hsh2(sg + p);
            for (int w = 0; w < W2; w++) {
              uint32_t v = snap2[h2 * W2 + w];
              if (!v) continue;
              int q = (int)v - 1 + wlo;
              if (q >= p || p - q > 32768) continue;
              int lim = sn - p < 258 ? sn - p : 258;
              int L = mlen(sg + p, sg + q, lim);
              if (L >= MINM && (L > bestl || (L == bestl && p - q < bestd))) { bestl = L; bestd = p - q; }
            }
          }
          cd[p] = bestd;
        }
        for (int p = r0; p < r0 + ROUND && p < sn; p++)
        {
          if (p + MINM <= sn) ins(tab, hsh(rd4(sg + p), MINM), p - wlo);
          if (W2 && p + K2 <= sn) ins2(tab2, hsh2(sg + p), p - wlo);
        }
      }
      free(snap);
      // parse
      fl[256] += 1;
      const int rng = RANGE ? RANGE : sn;
      int p = 0;
      for (int t0 = 0; t0 < sn; t0 += rng) {
        const int end = t0 + rng < sn ? t0 + rng : sn;
        if (RANGE) p = t0;  // each thread restarts at its range start
        while (p < end) {
          int lim = (RANGE ? end : sn) - p;
          if (lim > 258) lim = 258;
          int d = cd[p], L = d ? mlen(sg + p, sg + p - d, lim) : 0;
          int defer = 0;
          for (int la = 1; la <= LAZY && L >= MINM && L < 32; la++) {
            if (p + la >= (RANGE ? end : sn)) break;
            int lim1 = (RANGE ? end : sn) - p - la;
            if (lim1 > 258) lim1 = 258;
            int d1 = cd[p + la], L1 = d1 ? mlen(sg + p + la, sg + p + la - d1, lim1) : 0;
            if (L1 > L + la - 1) { defer = 1; break; }
          }
          if (L >= MINM && !defer && !(L == 3 && d > 4096) && !(FAR4 && L == 4 && d > FAR4) && !(FAR5 && L == 5 && d > FAR5)) {
            int s, e, ds, de;
            lsym(L, &s, &e);
            dsym(d, &ds, &de);
            if (FLEX && L > MINM) {
              // the cut j in [p + MINM, p + L] whose match reaches farthest
              const int E = RANGE ? end : sn;
              int bj = p + L, br = -1;
              for (int j = p + MINM; j <= p + L && j < E; j++) {
                int lj = j + 258 <= E ? 258 : E - j;
                int dj = cd[j], Lj = dj ? mlen(sg + j, sg + j - dj, lj) : 0;
                int reach = Lj >= MINM ? j + Lj : j;
                if (reach > br || (reach == br && j == p + L)) { br = reach; bj = j; }
              }
              L = bj - p;
              lsym(L, &s, &e);
            }
            fl[s]++; fd[ds]++; extra += e + de;
            p += L;
          } else {
            fl[sg[p]]++;
            p += 1;
          }
        }
      }
      nseg++;
      if (++in_group < SHARE && s0 + SEG < bl) continue;
      int ll[288], dl[32];
      huff(fl, 286, 15, ll);
      huff(fd, 30, 15, dl);
      double bits = extra;
      int hlit = 257, hdist = 1;
      for (int i = 0; i < 286; i++) { bits += (double)fl[i] * ll[i]; if (ll[i] && i >= 257) hlit = i + 1; }
      for (int i = 0; i < 30; i++) { bits += (double)fd[i] * dl[i]; if (dl[i]) hdist = i + 1; }
      const double hb = hdr_bits(ll, dl, hlit, hdist);
      hdr_total += hb;
      bits += hb;
      bits += 3 + 32 + 8;  // sync flush
      total_bits += bits;
      in_group = 0;
      extra = 0;
      memset(fl, 0, sizeof fl);
      memset(fd, 0, sizeof fd);
    }
    total_bits += 8 * 11;  // zlib header, final empty block, Adler
  }
  printf("bytes %zu  out %.0f  ratio %.4f  hdr %.2f%%  (ways %d bits %d range %d seg %d hist %d/%d min %d lazy %d block %ld)\n", n,
         total_bits / 8, total_bits / 8 / n, 100.0 * hdr_total / total_bits, WAYS, HBITS, RANGE, SEG, HIST, HLEN, MINM, LAZY, BLOCK);
  return 0;
}
