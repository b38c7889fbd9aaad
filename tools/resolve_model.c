// resolve_model.c -- CPU model of LZ77 match-resolve strategies for K2 (dq_inflate3.hip).
//
// Reads a BGZF file, decodes every member's DEFLATE stream into a token list (literals and
// (length, distance) matches, in output order) and reports, per BGZF block, what a parallel
// resolve would face:
//   - token counts, bytes in matches, length / distance histograms;
//   - MRR depth: rounds of "copy every match whose source bytes are final" (a match's source is
//     final when every match overlapping it was copied in an earlier round);
//   - the same after redirecting each match's source through matches that contain it whole
//     (byte x of a match equals byte x - dist, so a source range inside one match's output is
//     the same bytes dist earlier);
//   - rounds needed when the output is cut into ordered steps of S bytes (a match whose redirected
//     source lies before its step's start is final at its step).
// Development tool (not built by the product, not a test): cc -O2 -o /tmp/rm tools/resolve_model.c
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct { int32_t pos, len, dist; } Tok;  // len 0: literal
static int32_t src1[70000], nx[70000], hop[70000];  // per byte: first-hop source, jump scratch

static const uint8_t *g_in;
static size_t g_nbits, g_bp;
static uint32_t bits(int n) {
  uint32_t v = 0;
  for (int i = 0; i < n; i++, g_bp++) v |= (uint32_t)((g_in[g_bp >> 3] >> (g_bp & 7)) & 1) << i;
  return v;
}
typedef struct { uint16_t cnt[16], sym[320]; } Huff;
static void build(Huff *h, const uint8_t *len, int n) {
  memset(h, 0, sizeof *h);
  for (int i = 0; i < n; i++) h->cnt[len[i]]++;
  h->cnt[0] = 0;
  uint16_t off[16] = {0};
  for (int i = 1; i < 16; i++) off[i] = off[i - 1] + h->cnt[i - 1];
  for (int i = 0; i < n; i++)
    if (len[i]) h->sym[off[len[i]]++] = (uint16_t)i;
}
static int decode(const Huff *h) {
  int code = 0, first = 0, index = 0;
  for (int l = 1; l < 16; l++) {
    code |= (int)bits(1);
    int c = h->cnt[l];
    if (code - c < first) return h->sym[index + (code - first)];
    index += c;
    first += c;
    first <<= 1;
    code <<= 1;
  }
  return -1;
}
static const int LB[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
static const int LE[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const int DB[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
static const int DE[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

// tokens of one raw-DEFLATE stream; returns the count (-1 on error); *nblocks = deflate blocks
static int tokenize(const uint8_t *d, size_t n, Tok *tk, int cap, int *nblocks, int *outlen) {
  g_in = d;
  g_nbits = 8 * n;
  g_bp = 0;
  int nt = 0, pos = 0, last = 0;
  *nblocks = 0;
  while (!last) {
    last = (int)bits(1);
    int type = (int)bits(2);
    (*nblocks)++;
    if (type == 0) {
      g_bp = (g_bp + 7) & ~(size_t)7;
      int len = (int)bits(16);
      bits(16);
      for (int i = 0; i < len; i++) {
        bits(8);
        tk[nt++] = (Tok){pos++, 0, 0};
      }
      continue;
    }
    uint8_t ll[320];
    Huff hl, hd;
    int nlen = 288, nd = 32;
    if (type == 1) {
      for (int i = 0; i < 288; i++) ll[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : 8;
      for (int i = 0; i < 32; i++) ll[288 + i] = 5;
    } else {
      nlen = (int)bits(5) + 257;
      nd = (int)bits(5) + 1;
      int nc = (int)bits(4) + 4;
      static const int ord[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
      uint8_t cl[19] = {0};
      for (int i = 0; i < nc; i++) cl[ord[i]] = (uint8_t)bits(3);
      Huff hc;
      build(&hc, cl, 19);
      uint8_t lens[320];
      int k = 0;
      while (k < nlen + nd) {
        int s = decode(&hc);
        if (s < 0) return -1;
        if (s < 16) lens[k++] = (uint8_t)s;
        else {
          int r = s == 16 ? 3 + (int)bits(2) : s == 17 ? 3 + (int)bits(3) : 11 + (int)bits(7);
          uint8_t v = s == 16 ? lens[k - 1] : 0;
          while (r--) lens[k++] = v;
        }
      }
      memset(ll, 0, sizeof ll);
      memcpy(ll, lens, (size_t)nlen);
      memcpy(ll + 288, lens + nlen, (size_t)nd);
    }
    build(&hl, ll, 288);
    build(&hd, ll + 288, 32);
    for (;;) {
      int s = decode(&hl);
      if (s < 0) return -1;
      if (s < 256) {
        if (nt >= cap) return -1;
        tk[nt++] = (Tok){pos++, 0, 0};
      } else if (s == 256) {
        break;
      } else {
        s -= 257;
        int len = LB[s] + (int)bits(LE[s]);
        int ds = decode(&hd);
        if (ds < 0) return -1;
        int dist = DB[ds] + (int)bits(DE[ds]);
        if (nt >= cap) return -1;
        tk[nt++] = (Tok){pos, len, dist};
        pos += len;
      }
    }
  }
  *outlen = pos;
  return nt;
}

// per block statistics, summed
typedef struct {
  long blocks, toks, lits, matches, mbytes, bytes, overlap, short16;
  long lvl_sum, rlvl_sum, lvl_h[6], rlvl_h[6];  // match levels (round in which its source is final)
  long depth_sum, depth_max, rdepth_sum, rdepth_max, straddle;
  long lenh[8], disth[8];
  long step_rounds[8][2];  // steps S = 256 << i: [sum of max rounds per step over steps, steps]
  long final_at_step[8], nonfinal_at_step[8];
  long rjumps;
  long hops_lit, hops_lit_max, hops_win[8], win_rounds[8];
  long dag_steps, dag_need_prev, dag_depth_sum, dag_depth_max, dag_need_prev2;
} Stats;

int main(int argc, char **argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s file.bam [maxblocks]\n", argv[0]);
    return 2;
  }
  FILE *f = fopen(argv[1], "rb");
  if (!f) return 2;
  fseek(f, 0, SEEK_END);
  long fl = ftell(f);
  fseek(f, 0, SEEK_SET);
  uint8_t *buf = malloc((size_t)fl + 16);
  if (fread(buf, 1, (size_t)fl, f) != (size_t)fl) return 2;
  fclose(f);
  long maxb = argc > 2 ? atol(argv[2]) : 1L << 40;
  Stats S;
  memset(&S, 0, sizeof S);
  Tok *tk = malloc(sizeof(Tok) * 70000);
  int32_t *owner = malloc(sizeof(int32_t) * 70000);  // token index of each output byte
  int32_t *depth = malloc(sizeof(int32_t) * 70000), *rd = malloc(sizeof(int32_t) * 70000);
  int32_t *rs = malloc(sizeof(int32_t) * 70000);  // redirected source start
  long p = 0;
  while (p + 28 <= fl && S.blocks < maxb) {
    int bsize = buf[p + 16] | buf[p + 17] << 8;
    int cs = bsize + 1;
    int isize = buf[p + cs - 4] | buf[p + cs - 3] << 8 | buf[p + cs - 2] << 16 | buf[p + cs - 1] << 24;
    if (isize == 0) {
      p += cs;
      continue;
    }
    int nb = 0, ol = 0;
    int nt = tokenize(buf + p + 18, (size_t)cs - 26, tk, 70000, &nb, &ol);
    p += cs;
    if (nt < 0 || ol != isize) {
      fprintf(stderr, "decode error at %ld\n", p);
      return 1;
    }
    S.blocks++;
    S.toks += nt;
    S.bytes += ol;
    for (int i = 0; i < nt; i++) {
      int L = tk[i].len ? tk[i].len : 1;
      for (int k = 0; k < L; k++) owner[tk[i].pos + k] = i;
    }
    int bdepth = 0, brd = 0;
    for (int i = 0; i < nt; i++) {
      Tok t = tk[i];
      if (!t.len) {
        S.lits++;
        depth[i] = rd[i] = 0;
        rs[i] = t.pos;
        continue;
      }
      S.matches++;
      S.mbytes += t.len;
      if (t.dist < t.len) S.overlap++;
      if (t.dist < 16) S.short16++;
      int lb = t.len < 4 ? 0 : t.len < 8 ? 1 : t.len < 16 ? 2 : t.len < 32 ? 3 : t.len < 64 ? 4 : t.len < 128 ? 5 : t.len < 258 ? 6 : 7;
      S.lenh[lb]++;
      int db = t.dist < 16 ? 0 : t.dist < 64 ? 1 : t.dist < 256 ? 2 : t.dist < 1024 ? 3 : t.dist < 4096 ? 4 : t.dist < 16384 ? 5 : 6;
      S.disth[db]++;
      // MRR depth: the source bytes [s, e) (for an overlapping match, the first period)
      int s = t.pos - t.dist, e = s + (t.dist < t.len ? t.dist : t.len);
      int dm = 0;
      for (int x = s; x < e; x++) {
        int o = owner[x];
        if (depth[o] > dm) dm = depth[o];
      }
      depth[i] = dm + 1;
      if (depth[i] > bdepth) bdepth = depth[i];
      S.lvl_sum += depth[i];
      S.lvl_h[depth[i] <= 1 ? 0 : depth[i] <= 2 ? 1 : depth[i] <= 4 ? 2 : depth[i] <= 8 ? 3 : depth[i] <= 32 ? 4 : 5]++;
      // redirect: while [s, e) lies inside one match's output, move it back by that distance
      int jumps = 0;
      for (;;) {
        int o = owner[s];
        if (!tk[o].len || e > tk[o].pos + tk[o].len) break;
        s -= tk[o].dist;
        e -= tk[o].dist;
        jumps++;
      }
      S.rjumps += jumps;
      rs[i] = s;
      int rm = 0, strad = 0;
      for (int x = s; x < e; x++) {
        int o = owner[x];
        if (rd[o] > rm) rm = rd[o];
        if (x > s && o != owner[x - 1]) strad = 1;
      }
      S.straddle += strad;
      rd[i] = rm + 1;
      if (rd[i] > brd) brd = rd[i];
      S.rlvl_sum += rd[i];
      S.rlvl_h[rd[i] <= 1 ? 0 : rd[i] <= 2 ? 1 : rd[i] <= 4 ? 2 : rd[i] <= 8 ? 3 : rd[i] <= 32 ? 4 : 5]++;
    }
    // per byte: hops to a literal, and to a byte before the byte's window of W bytes; synchronous
    // pointer-jumping rounds per window (max over its bytes)
    {
      for (int i = 0; i < nt; i++) {
        Tok t = tk[i];
        if (!t.len) {
          src1[t.pos] = t.pos;
          continue;
        }
        for (int j = 0; j < t.len; j++) src1[t.pos + j] = t.pos - t.dist + (j % t.dist);
      }
      long hl = 0, hmax = 0;
      for (int x = 0; x < ol; x++) {
        int h = 0, y = x;
        while (src1[y] != y) {
          y = src1[y];
          h++;
        }
        hl += h;
        if (h > hmax) hmax = h;
      }
      S.hops_lit += hl;
      if (hmax > S.hops_lit_max) S.hops_lit_max = hmax;
      for (int wi = 0; wi < 8; wi++) {
        int W = 256 << wi;
        long hw = 0;
        for (int w0 = 0; w0 < ol; w0 += W) {
          int w1 = w0 + W < ol ? w0 + W : ol;
          for (int x = w0; x < w1; x++) {
            int h = 0, y = x;
            while (src1[y] != y && y >= w0) {
              y = src1[y];
              h++;
              if (y < w0) break;
            }
            hw += h;
            nx[x] = src1[x];
            hop[x] = 0;
          }
          // synchronous pointer jumping: p <- nx[p] while p inside the window and not a literal
          int rounds = 0;
          for (;;) {
            int ch = 0;
            for (int x = w0; x < w1; x++) {
              int p = nx[x];
              if (p >= w0 && nx[p] != p) {
                hop[x] = nx[p];
                ch = 1;
              } else
                hop[x] = p;
            }
            for (int x = w0; x < w1; x++) nx[x] = hop[x];
            if (!ch) break;
            rounds++;
          }
          S.win_rounds[wi] += rounds;
        }
        S.hops_win[wi] += hw;
      }
    }
    {  // step DAG (512-byte steps): final source of each byte after in-step resolution
      static int32_t fin[70000], sd[200];
      int ns = (ol + 511) / 512;
      for (int x = 0; x < ol; x++) {
        int s0 = x & ~511, y = x;
        // follow the byte chain while inside the step and not a literal
        while (src1[y] != y && src1[y] >= s0) y = src1[y];
        fin[x] = src1[y] == y ? y : src1[y];  // literal in step, or a byte before the step
      }
      int bmax = 0;
      for (int k = 0; k < ns; k++) {
        int need = -1;  // latest earlier step a non-literal source lies in
        for (int x = 512 * k; x < ol && x < 512 * (k + 1); x++) {
          int f = fin[x];
          if (f < 512 * k && src1[f] != f) { int st = f >> 9; if (st > need) need = st; }
        }
        int d = 1;
        for (int x = 512 * k; x < ol && x < 512 * (k + 1); x++) {
          int f = fin[x];
          if (f < 512 * k && src1[f] != f && sd[f >> 9] + 1 > d) d = sd[f >> 9] + 1;
        }
        sd[k] = d;
        if (d > bmax) bmax = d;
        S.dag_steps++;
        if (need == k - 1) S.dag_need_prev++;
        if (need >= k - 2) S.dag_need_prev2++;
      }
      S.dag_depth_sum += bmax;
      if (bmax > S.dag_depth_max) S.dag_depth_max = bmax;
    }
    S.depth_sum += bdepth;
    if (bdepth > S.depth_max) S.depth_max = bdepth;
    S.rdepth_sum += brd;
    if (brd > S.rdepth_max) S.rdepth_max = brd;
    // ordered steps: a match whose redirected source (first period) ends before its step's start is
    // final there; the others need rounds inside the step (depth among the step's own matches)
    for (int si = 0; si < 8; si++) {
      int Sz = 256 << si;
      for (int s0 = 0; s0 < ol; s0 += Sz) {
        int mx = 0;
        for (int i = 0; i < nt; i++) {
          Tok t = tk[i];
          if (t.pos < s0 || t.pos >= s0 + Sz) continue;
          if (!t.len) {
            depth[i] = 0;
            continue;
          }
          int s = rs[i], e = s + (t.dist < t.len ? t.dist : t.len);
          if (e <= s0) {
            depth[i] = 1;
            S.final_at_step[si]++;
          } else {
            S.nonfinal_at_step[si]++;
            int dm = 0;
            for (int x = s; x < e; x++) {
              int o = owner[x];
              if (tk[o].pos >= s0 && depth[o] > dm) dm = depth[o];
            }
            depth[i] = dm + 1;
          }
          if (depth[i] > mx) mx = depth[i];
        }
        S.step_rounds[si][0] += mx;
        S.step_rounds[si][1]++;
      }
    }
  }
  double B = (double)S.blocks;
  printf("blocks %ld  bytes/block %.0f  tokens/block %.0f  literals/block %.0f  matches/block %.0f\n",
         S.blocks, S.bytes / B, S.toks / B, S.lits / B, S.matches / B);
  printf("bytes in matches %.1f %%  mean match length %.2f  overlapping (dist < len) %.2f %%  dist < 16 %.2f %%\n",
         100.0 * S.mbytes / S.bytes, (double)S.mbytes / S.matches, 100.0 * S.overlap / S.matches,
         100.0 * S.short16 / S.matches);
  printf("length hist [3,4,8,16,32,64,128,258]:");
  for (int i = 0; i < 8; i++) printf(" %.1f%%", 100.0 * S.lenh[i] / S.matches);
  printf("\ndistance hist [<16,<64,<256,<1K,<4K,<16K,<32K]:");
  for (int i = 0; i < 7; i++) printf(" %.1f%%", 100.0 * S.disth[i] / S.matches);
  printf("\nMRR depth: mean %.1f max %ld;  after redirect: mean %.1f max %ld  (jumps/match %.2f, straddling %.1f %%)\n",
         S.depth_sum / B, S.depth_max, S.rdepth_sum / B, S.rdepth_max, (double)S.rjumps / S.matches,
         100.0 * S.straddle / S.matches);
  printf("match level (MRR round): mean %.2f, <=1 %.1f%% <=2 %.1f%% <=4 %.1f%% <=8 %.1f%% <=32 %.1f%% >32 %.1f%%\n",
         (double)S.lvl_sum / S.matches, 100.0 * S.lvl_h[0] / S.matches, 100.0 * S.lvl_h[1] / S.matches,
         100.0 * S.lvl_h[2] / S.matches, 100.0 * S.lvl_h[3] / S.matches, 100.0 * S.lvl_h[4] / S.matches,
         100.0 * S.lvl_h[5] / S.matches);
  printf("after redirect: mean %.2f, <=1 %.1f%% <=2 %.1f%% <=4 %.1f%% <=8 %.1f%% <=32 %.1f%% >32 %.1f%%\n",
         (double)S.rlvl_sum / S.matches, 100.0 * S.rlvl_h[0] / S.matches, 100.0 * S.rlvl_h[1] / S.matches,
         100.0 * S.rlvl_h[2] / S.matches, 100.0 * S.rlvl_h[3] / S.matches, 100.0 * S.rlvl_h[4] / S.matches,
         100.0 * S.rlvl_h[5] / S.matches);
  printf("512-byte step DAG: steps needing step k-1 %.1f %%, k-1 or k-2 %.1f %%, critical path mean %.1f max %ld steps (of %.1f)\n",
         100.0 * S.dag_need_prev / S.dag_steps, 100.0 * S.dag_need_prev2 / S.dag_steps, S.dag_depth_sum / B, S.dag_depth_max, S.dag_steps / B);
  printf("byte hops to a literal: mean %.2f max %ld\n", (double)S.hops_lit / S.bytes, S.hops_lit_max);
  for (int wi = 0; wi < 8; wi++)
    printf("window %6d: hops to before-window/literal mean %.2f, sync jump rounds per window %.2f (per block %.1f)\n",
           256 << wi, (double)S.hops_win[wi] / S.bytes, S.win_rounds[wi] / (B * (65498.0 / (256 << wi))), S.win_rounds[wi] / B);
  for (int si = 0; si < 8; si++)
    printf("steps of %6d: %5.1f steps/block, rounds per step mean %.2f (sum per block %.1f), final at step %.1f %%\n",
           256 << si, (double)S.step_rounds[si][1] / B, (double)S.step_rounds[si][0] / S.step_rounds[si][1],
           S.step_rounds[si][0] / B,
           100.0 * S.final_at_step[si] / (S.final_at_step[si] + S.nonfinal_at_step[si]));
  return 0;
}
