// Dev tool (CPU): compression-ratio model of LZ77 parse strategies for the GPU BGZF deflate
// kernel (dq_deflate.hip), on a decompressed BAM stream cut into htsjdk's 65280-byte blocks.
// Cost of a block = its symbols under the block's own Huffman codes (lengths <= 15, from the
// symbol histogram) + extra bits + a dynamic-header estimate; compared with zlib level 5 (htsjdk).
//   gcc -O2 -o /tmp/deflate_model tools/deflate_model.c -lz && /tmp/deflate_model STREAM
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

enum { BLK = 65280, MAXM = 258, WIN = 32768 };

typedef struct {
  const char* name;
  int seg;        // bytes per parsing lane (0 = one parse over the block)
  int cross;      // a match may run past the lane's segment end (the next lane starts after it)
  int shortd;     // distances 1..shortd always tried
  int chain;      // hash-chain links tried
  int hbits;      // hash bits
  int stripe;     // links only to positions in earlier stripes of this many positions (0 = exact)
  int lazy;       // zlib-style lazy evaluation: defer a match shorter than this
  int nice;       // stop the chain walk at a match this long
  int lazy_once;  // look one position ahead only (else defer while the next match is longer)
  int half;       // chunk size: each chunk parses on its own (its matches end inside it), with
  int xw;         // candidates from xw bytes before the chunk start on (0 = no chunks)
  int hchunk;     // one dynamic Huffman block per chunk (else one per BGZF block)
  int h4;         // bucket positions by a hash of 4 bytes (so matches are >= 4 bytes)
} Cfg;

static int lcode(int len) {  // length symbol
  if (len == 258) return 285;
  int l = len - 3;
  if (l < 8) return 257 + l;
  int b = 31 - __builtin_clz(l), nx = b - 2;
  return 257 + 4 * nx + 4 + ((l >> nx) & 3);
}
static int lextra(int s) { return (s < 265 || s == 285) ? 0 : (s - 261) >> 2; }
static int dcode(int d) {
  int v = d - 1;
  if (v < 4) return v;
  int b = 31 - __builtin_clz(v);
  return 2 * b + ((v >> (b - 1)) & 1);
}
static int dextra(int s) { return s < 4 ? 0 : (s - 2) >> 1; }

// Huffman code lengths (simple heap-free O(n^2) merge, then cap at 15 by the Kraft fix-up)
static void huff(const long* f, int n, int* len) {
  long w[600];
  int par[600], m = 0, id[600];
  for (int i = 0; i < n; i++) len[i] = 0;
  for (int i = 0; i < n; i++)
    if (f[i]) { w[m] = f[i]; id[m] = i; par[m] = -1; m++; }
  if (m == 0) return;
  if (m == 1) { len[id[0]] = 1; return; }
  int alive[600], na = m, tot = m;
  for (int i = 0; i < m; i++) alive[i] = i;
  while (na > 1) {
    int a = -1, b = -1;
    for (int k = 0; k < na; k++) {
      int x = alive[k];
      if (a < 0 || w[x] < w[a]) { b = a; a = x; }
      else if (b < 0 || w[x] < w[b]) b = x;
    }
    w[tot] = w[a] + w[b];
    par[tot] = -1;
    par[a] = tot;
    par[b] = tot;
    int na2 = 0;
    for (int k = 0; k < na; k++)
      if (alive[k] != a && alive[k] != b) alive[na2++] = alive[k];
    alive[na2++] = tot;
    na = na2;
    tot++;
  }
  int cnt[64] = {0};
  for (int i = 0; i < m; i++) {
    int d = 0;
    for (int x = i; par[x] >= 0; x = par[x]) d++;
    len[id[i]] = d;
  }
  for (int i = 0; i < n; i++) if (len[i]) cnt[len[i] > 15 ? 15 : len[i]]++;
  unsigned tot2 = 0;
  for (int l = 15; l > 0; l--) tot2 += (unsigned)cnt[l] << (15 - l);
  int over = 0;
  for (int i = 0; i < n; i++) if (len[i] > 15) over = 1;
  if (over) {  // crude cap (rare on these streams)
    while (tot2 > (1u << 15)) {
      cnt[15]--;
      for (int l = 14; l > 0; l--) if (cnt[l]) { cnt[l]--; cnt[l + 1] += 2; break; }
      tot2--;
    }
    // reassign by frequency order
    int ord[600], k = 0;
    for (int i = 0; i < n; i++) if (f[i]) ord[k++] = i;
    for (int a = 0; a < k; a++) for (int b = a + 1; b < k; b++) if (f[ord[b]] > f[ord[a]]) { int t = ord[a]; ord[a] = ord[b]; ord[b] = t; }
    int j = 0;
    for (int l = 1; l <= 15; l++) for (int c = cnt[l]; c > 0; c--) len[ord[j++]] = l;
  }
}

// exact dynamic-header bits: HLIT/HDIST/HCLEN, the code-length code, the RLE-coded lengths
static long header_bits(const int* ll, const int* dl) {
  int nlit = 286, ndist = 30;
  while (nlit > 257 && !ll[nlit - 1]) nlit--;
  while (ndist > 1 && !dl[ndist - 1]) ndist--;
  int v[320], N = nlit + ndist;
  for (int i = 0; i < nlit; i++) v[i] = ll[i];
  for (int i = 0; i < ndist; i++) v[nlit + i] = dl[i];
  int tok[400], ex[400], nt = 0;
  for (int i = 0; i < N;) {
    int run = 1;
    while (i + run < N && v[i + run] == v[i]) run++;
    int r = run;
    if (v[i] == 0) {
      while (r >= 11) { int k = r < 138 ? r : 138; tok[nt] = 18; ex[nt++] = 7; r -= k; }
      if (r >= 3) { tok[nt] = 17; ex[nt++] = 3; r = 0; }
      while (r > 0) { tok[nt] = 0; ex[nt++] = 0; r--; }
    } else {
      tok[nt] = v[i]; ex[nt++] = 0; r--;
      while (r >= 3) { int k = r < 6 ? r : 6; tok[nt] = 16; ex[nt++] = 2; r -= k; }
      while (r > 0) { tok[nt] = v[i]; ex[nt++] = 0; r--; }
    }
    i += run;
  }
  long fc[19] = {0};
  for (int k = 0; k < nt; k++) fc[tok[k]]++;
  int cl[19];
  huff(fc, 19, cl);
  for (int k = 0; k < 19; k++) if (cl[k] > 7) cl[k] = 7;  // (the cap: rare)
  static const int ord[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
  int ncl = 19;
  while (ncl > 4 && !cl[ord[ncl - 1]]) ncl--;
  long b = 3 + 5 + 5 + 4 + 3 * ncl;
  for (int k = 0; k < nt; k++) b += cl[tok[k]] + ex[k];
  return b;
}

typedef struct { int lit; int len; int dist; } Sym;

static int match_len(const uint8_t* b, int p, int q, int lim) {
  int l = 0;
  while (l < lim && b[p + l] == b[q + l]) l++;
  return l;
}

// best match at p among the tried candidates; returns len (0 if < 3), *dist
static int find(const Cfg* c, const uint8_t* b, int n, int p, int lim, const int* link, int* dist) {
  int best = 0, bd = 0;
  if (lim < 3 + (c->h4 ? 1 : 0)) return 0;
  const int qmin = c->half ? (p / c->half) * c->half - c->xw : 0;
  for (int d = 1; d <= c->shortd && d <= p; d++) {
    int l = match_len(b, p, p - d, lim);
    if (l > best) { best = l; bd = d; }
  }
  int q = link[p];
  for (int k = 0; k < c->chain && q >= qmin && p - q <= WIN; k++) {
    if (p - q > c->shortd) {
      int l = match_len(b, p, q, lim);
      if (l > best) { best = l; bd = p - q; }
      if (best >= c->nice) break;
    }
    q = link[q];
  }
  *dist = bd;
  return best >= 3 ? best : 0;
}

static long block_bits(const Cfg* c, const uint8_t* b, int n, int* link, int* head, Sym* sy) {
  // links
  int hs = 1 << c->hbits;
  for (int i = 0; i < hs; i++) head[i] = -1;
  if (c->stripe) {
    for (int r = 0; r * c->stripe < n; r++) {
      int a = r * c->stripe, e = a + c->stripe < n ? a + c->stripe : n;
      for (int p = a; p < e; p++) {
        link[p] = -1;
        if (p + 3 <= n) {
          uint32_t v = b[p] | b[p + 1] << 8 | b[p + 2] << 16;
          link[p] = head[(v * 2654435761u) >> (32 - c->hbits)];
        }
      }
      for (int p = a; p < e; p++)
        if (p + 3 <= n) {
          uint32_t v = b[p] | b[p + 1] << 8 | b[p + 2] << 16;
          head[(v * 2654435761u) >> (32 - c->hbits)] = p;
        }
    }
  } else {
    for (int p = 0; p < n; p++) {
      link[p] = -1;
      if (p + 3 + (c->h4 ? 1 : 0) <= n) {
        uint32_t v = b[p] | b[p + 1] << 8 | b[p + 2] << 16 | (c->h4 ? (uint32_t)b[p + 3] << 24 : 0u);
        uint32_t h = (v * 2654435761u) >> (32 - c->hbits);
        link[p] = head[h];
        head[h] = p;
      }
    }
  }
  // parse
  int ns = 0;
  int seg = c->seg ? c->seg : n;
  int p = 0;
  for (int s0 = 0; s0 < n; s0 += seg) {
    int s1 = s0 + seg < n ? s0 + seg : n;
    if (p < s0) p = s0;  // (never: the previous lane ended at or past s0)
    if (!c->cross) p = s0;
    int end = c->cross ? n : s1;
    if (c->half) {  // a chunk's parse ends at the chunk end
      const int ce = (s0 / c->half + 1) * c->half;
      if (end > ce) end = ce;
      if (s1 > ce) s1 = ce;
    }
    while (p < s1) {
      int lim = end - p < MAXM ? end - p : MAXM;
      int d = 0, l = find(c, b, n, p, lim, link, &d);
      while (l && c->lazy && l < c->lazy && p + 1 < end) {
        int lim2 = end - p - 1 < MAXM ? end - p - 1 : MAXM;
        int d2 = 0, l2 = find(c, b, n, p + 1, lim2, link, &d2);
        if (l2 <= l) break;
        sy[ns++] = (Sym){b[p], 0, 0}; p++; l = l2; d = d2;
        if (c->lazy_once) break;
      }
      if (l) { sy[ns++] = (Sym){0, l, d}; p += l; }
      else { sy[ns++] = (Sym){b[p], 0, 0}; p++; }
    }
  }
  // Huffman blocks: the whole parse, or one per chunk (symbols split where their bytes start)
  long total = 0;
  int s0 = 0, pos = 0;
  for (int b = 0; ; b++) {
    const int bend = c->hchunk && c->half ? (b + 1) * c->half : n;
    int s1 = s0, p1 = pos;
    while (s1 < ns && p1 < bend) { p1 += sy[s1].len ? sy[s1].len : 1; s1++; }
    long fl[286] = {0}, fd[30] = {0};
    long extra = 0;
    for (int i = s0; i < s1; i++) {
      if (sy[i].len) {
        int s = lcode(sy[i].len), d = dcode(sy[i].dist);
        fl[s]++; fd[d]++;
        extra += lextra(s) + dextra(d);
      } else fl[sy[i].lit]++;
    }
    fl[256]++;
    int ll[286], dl[30];
    huff(fl, 286, ll);
    huff(fd, 30, dl);
    long bits = extra;
    for (int i = 0; i < 286; i++) bits += fl[i] * ll[i];
    for (int i = 0; i < 30; i++) bits += fd[i] * dl[i];
    total += bits + header_bits(ll, dl);
    s0 = s1;
    pos = p1;
    if (s0 >= ns) break;
  }
  return total;
}

int main(int argc, char** argv) {
  if (argc < 2) return 1;
  FILE* f = fopen(argv[1], "rb");
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  uint8_t* u = malloc(n + 512);
  if (fread(u, 1, n, f) != (size_t)n) return 1;
  memset(u + n, 0, 512);
  long maxb = argc > 2 ? atol(argv[2]) : 200;
  int* link = malloc(sizeof(int) * BLK);
  int* head = malloc(sizeof(int) * (1 << 16));
  Sym* sy = malloc(sizeof(Sym) * (BLK + 8));
  Cfg cfgs[] = {
      {"gpu r2: seg255 greedy short8 chain6 h11 stripe256", 255, 0, 8, 6, 11, 256, 0, 258, 1},
      {"seg255 cross, exact h12 chain32 lazy16(once) nice32", 255, 1, 8, 32, 12, 0, 16, 32, 1},
      {"seg255 cross, exact h12 chain32 lazy16 nice32", 255, 1, 8, 32, 12, 0, 16, 32, 0},
      {"seg255 cross, exact h13 chain32 lazy16 nice32", 255, 1, 8, 32, 13, 0, 16, 32, 0},
      {"seg255 cross, exact h15 chain32 lazy16 nice32", 255, 1, 8, 32, 15, 0, 16, 32, 0},
      {"seg255 cross, exact h12 chain64 lazy32 nice64", 255, 1, 8, 64, 12, 0, 32, 64, 0},
      {"seg255 cross, exact h13 chain48 lazy24 nice48", 255, 1, 8, 48, 13, 0, 24, 48, 0},
      {"seg255 cross, exact h12 chain32 lazy16 nice32 short0", 255, 1, 0, 32, 12, 0, 16, 32, 0},
      {"seg255 nocross, exact h12 chain32 lazy16 nice32", 255, 0, 8, 32, 12, 0, 16, 32, 0},
      {"one parse, exact h15 chain32 lazy16 nice32 (zlib 5 like)", 0, 0, 0, 32, 15, 0, 16, 32, 0},
      {"gpu r3: seg255 cross h11 chain96 lazy32 nice96", 255, 1, 0, 96, 11, 0, 32, 96, 0},
      {"chunks: halves C=32640 X=15K seg64 (bgzf_parse_kernel)", 64, 1, 0, 96, 11, 0, 32, 96, 0, 32640, 15000, 0},
      {"  4-byte hash, 96/32/96", 64, 1, 0, 96, 11, 0, 32, 96, 0, 32640, 15000, 0, 1},
      {"  4-byte hash, 32/16/32", 64, 1, 0, 32, 11, 0, 16, 32, 0, 32640, 15000, 0, 1},
      {"  4-byte hash, 24/16/32", 64, 1, 0, 24, 11, 0, 16, 32, 0, 32640, 15000, 0, 1},
      {"  4-byte hash, 16/16/32", 64, 1, 0, 16, 11, 0, 16, 32, 0, 32640, 15000, 0, 1},
      {"  4-byte hash, 16/8/16", 64, 1, 0, 16, 11, 0, 8, 16, 0, 32640, 15000, 0, 1},
      {"  4-byte hash, 12/8/16", 64, 1, 0, 12, 11, 0, 8, 16, 0, 32640, 15000, 0, 1},
      {"  4-byte hash, 8/8/16", 64, 1, 0, 8, 11, 0, 8, 16, 0, 32640, 15000, 0, 1},
      {"  4-byte hash, 8/4/16", 64, 1, 0, 8, 11, 0, 4, 16, 0, 32640, 15000, 0, 1},
      // round 5: two parse workgroups per CU need < 80 KB of LDS each: quarter-block chunks
      {"4-byte 32/16/32 halves C=32640 X=13600 seg64 (round 4)", 64, 1, 0, 32, 11, 0, 16, 32, 0, 32640, 13600, 0, 1},
      {"4-byte 32/16/32 quarters C=16320 X=4096 seg32", 32, 1, 0, 32, 11, 0, 16, 32, 0, 16320, 4096, 0, 1},
      {"4-byte 32/16/32 quarters C=16320 X=6144 seg32", 32, 1, 0, 32, 11, 0, 16, 32, 0, 16320, 6144, 0, 1},
      {"4-byte 32/16/32 quarters C=16320 X=6896 seg32", 32, 1, 0, 32, 11, 0, 16, 32, 0, 16320, 6896, 0, 1},
      {"4-byte 32/16/32 quarters C=16320 X=8192 seg32", 32, 1, 0, 32, 11, 0, 16, 32, 0, 16320, 8192, 0, 1},
      {"4-byte 32/16/32 quarters C=16320 X=16384 seg32", 32, 1, 0, 32, 11, 0, 16, 32, 0, 16320, 16384, 0, 1},
  };
  int nc = sizeof cfgs / sizeof cfgs[0];
  long nb = (n + BLK - 1) / BLK;
  if (nb > maxb) nb = maxb;
  long in = 0, zsz = 0;
  double tot[32] = {0};
  uint8_t* zb = malloc(2 * BLK);
  for (long k = 0; k < nb; k++) {
    int m = (int)(n - k * BLK < BLK ? n - k * BLK : BLK);
    const uint8_t* b = u + k * BLK;
    in += m;
    z_stream zs;
    memset(&zs, 0, sizeof zs);
    deflateInit2(&zs, 5, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY);
    zs.next_in = (uint8_t*)b; zs.avail_in = m; zs.next_out = zb; zs.avail_out = 2 * BLK;
    deflate(&zs, Z_FINISH);
    zsz += zs.total_out + 26;
    deflateEnd(&zs);
    for (int c = 0; c < nc; c++) tot[c] += block_bits(&cfgs[c], b, m, link, head, sy) / 8.0 + 26;
  }
  printf("blocks %ld, input %ld bytes; zlib level 5 (htsjdk): ratio %.3f\n", nb, in, (double)in / zsz);
  for (int c = 0; c < nc; c++) printf("  %-58s ratio %.3f\n", cfgs[c].name, in / tot[c]);
  return 0;
}
