// dq_deflate.hip -- BGZF compression on the GPU: the write side of the BAM path (SURVEY.md
// section 8, row f3).  Replaces htsjdk's BlockCompressedOutputStream as used by
// HeaderlessBamOutputFormat.BamRecordWriter (D/impl/formats/bam/HeaderlessBamOutputFormat.java:26-50)
// and BamSink's header / terminator files (D/impl/formats/bam/BamSink.java:32-69).
//
// Block layout is htsjdk's: the byte stream is cut into blocks of 65280 uncompressed bytes
// (BlockCompressedStreamConstants.DEFAULT_UNCOMPRESSED_BLOCK_SIZE; the last one shorter), each a
// gzip member with the 'BC' extra field, BSIZE, CRC32 and ISIZE.  The DEFLATE encoder is this
// kernel's own (java.util.zip.Deflater's exact bit stream is not reproduced): the output is valid
// BGZF whose blocks inflate to exactly htsjdk's block contents.
//
// One 256-thread workgroup per block, the block's bytes in LDS (79 KB: 2 workgroups per CU).
//   1. Match finder: every position with a 3-byte suffix goes into one of 2048 hash buckets, in
//      ascending order inside its bucket (counts by LDS atomics, bucket starts by a scan, then an
//      ordered scatter in stripes of 256 positions: the lanes of a wave with equal hashes are
//      found by one ballot per hash bit, and the four waves take their bucket cursors in turn).
//      A position's candidates are the entries before it in its bucket, most recent first: a
//      contiguous run of the bucket list, so a search issues all its candidate loads at once
//      instead of chasing zlib's hash-chain links one dependent load at a time.
//   2. Parse: lane t parses from its segment start [255 t, 255 t + 255) with zlib-style lazy
//      evaluation (a match shorter than `lazy` is deferred while the next position's is longer;
//      the look-ahead search walks chain / 4 candidates once the current match is `good` long, as
//      zlib's deflate_slow), the longest match among `chain` candidates (stopping at `nice`),
//      matches running on past the segment end.  A parse step depends on its position alone, so two parses that reach the
//      same position continue identically: from its exit, each lane keeps parsing until it hits a
//      symbol boundary of a later lane's parse (usually within a few symbols) and records the
//      merge; one thread then follows the merges from lane 0, which gives every lane the part of
//      its symbols (and continuation) on the block's one parse.  No matches are cut at lane
//      boundaries.  The merged parse is valid but not always the one a single sequential pass
//      would make: a merge can land inside a lazy step of the continuing lane (after a deferred
//      literal whose look-ahead search walked chain / 4 candidates, where a sequential pass would
//      start a full search), and a continuation that finds no merge within its staging is ended
//      on the next boundary of a later lane with a shortened match.
//      (Defaults chain 96, lazy 32, nice 96, good 8: ratio 2.858 on the synthetic WGS stream, zlib
//      level 5 -- htsjdk's -- 2.857; profiles/r3as_deflate_good_sweep.txt for the frontier.)
//   3. Codes: histograms of the parse; wave 0 builds the literal/length code and wave 1 the
//      distance code (a rank sort, Moffat-Katajainen minimum-redundancy lengths, a Kraft fix-up
//      capping them at 15), the code-length sequence is run-length coded; the block is coded
//      dynamic (BTYPE 10) or fixed (01), whichever is shorter.
//   4. Emit: each lane's bit count gives its offset by an exclusive scan; every lane OR-s its bits
//      into the LDS image of the block (the input is dead by then).  A block whose code would not
//      fit BSIZE (or whose parse overflowed its staging) is stored (BTYPE 00).
// CRC32: per-lane table CRC over the segment, combined with x^(8 n) mod P multipliers.
#include "dq_internal.h"

#include <algorithm>
#include <mutex>

namespace dq {
namespace {

constexpr int DWG = 256;                 // threads per block
constexpr int BLK_U = 65280;             // htsjdk DEFAULT_UNCOMPRESSED_BLOCK_SIZE
constexpr int SEG = BLK_U / DWG;         // 255 bytes per lane
constexpr int HBITS = 11;                // hash buckets (LDS counts / offsets: 8 KB)
constexpr int MAXM = 258;
constexpr int WIN = 32768;               // DEFLATE window
constexpr int OWN_WORDS = 288;           // a lane's own symbols (<= 255 + the last step's <= 32 deferrals)
constexpr int CONT_WORDS = 224;          // its continuation past its segment end
constexpr int LANE_WORDS = OWN_WORDS + CONT_WORDS;
constexpr int MAX_DEFLATE = 65536 - 26;  // BSIZE limit: 18-byte header + payload + 8 trailer
constexpr int MAXCAND = 128;             // candidates per match search at most (cfg.chain)

__constant__ uint32_t c_dcrc[256];
__constant__ uint16_t c_lbase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                                     35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint32_t c_x2n[32];  // x^(2^k) mod P (reflected)

__device__ inline uint32_t gf2_mul(uint32_t a, uint32_t b) {  // reflected, poly 0xEDB88320
  uint32_t m = 1u << 31, p = 0;
  for (int i = 0; i < 32; i++) {
    if (a & m) p ^= b;
    m >>= 1;
    b = b & 1 ? (b >> 1) ^ 0xEDB88320u : b >> 1;
  }
  return p;
}
// x^(8 n) mod P
__device__ inline uint32_t x8n(uint32_t n) {
  uint32_t p = 1u << 31;  // x^0
  int k = 3;              // x^(2^3) = x^8
  while (n) {
    if (n & 1) p = gf2_mul(c_x2n[k & 31], p);
    n >>= 1;
    k++;
  }
  return p;
}

__device__ inline uint32_t rev(uint32_t code, int len) { return __builtin_bitreverse32(code) >> (32 - len); }

// RFC 1951 3.2.5: length symbol (257..285) and extra bits for a match length 3..258
__device__ inline void len_code(int len, int& sym, int& nx, int& xv) {
  if (len == 258) { sym = 285; nx = 0; xv = 0; return; }
  const int l = len - 3;  // 0..254
  if (l < 8) { sym = 257 + l; nx = 0; xv = 0; return; }
  const int b = 31 - __builtin_clz((uint32_t)l);  // >= 3
  nx = b - 2;
  const int hi = (l >> nx) & 3;
  sym = 257 + 4 * nx + 4 + hi;
  xv = l & ((1 << nx) - 1);
}
__device__ inline void dist_code(int d, int& sym, int& nx, int& xv) {
  const int v = d - 1;  // 0..32767
  if (v < 4) { sym = v; nx = 0; xv = 0; return; }
  const int b = 31 - __builtin_clz((uint32_t)v);  // >= 2
  nx = b - 1;
  sym = 2 * b + ((v >> nx) & 1);
  xv = v & ((1 << nx) - 1);
}
// fixed-Huffman litlen code (bit-reversed for the LSB-first stream) and its length
__device__ inline void fixed_ll(int sym, uint32_t& code, int& len) {
  if (sym < 144) { len = 8; code = rev(0x30 + sym, 8); }
  else if (sym < 256) { len = 9; code = rev(0x190 + sym - 144, 9); }
  else if (sym < 280) { len = 7; code = rev(sym - 256, 7); }
  else { len = 8; code = rev(0xC0 + sym - 280, 8); }
}

struct alignas(16) DLds {
  uint8_t in[65536 + 16];     // the block's bytes; later the deflate image (<= 65510 bytes)
  uint32_t crc_t[256];
  uint32_t lane_bits[DWG];    // the parse's exit of each lane; later its bit count, bit offset
  uint32_t lane_crc[DWG];
  uint32_t lane_mrg[DWG];     // continuation: merge lane | symbol index << 9 | count << 18 | over << 27
  uint32_t lane_eff[DWG];     // effective symbols: own start | continuation count << 9 | EFF_* flags
  uint16_t lane_nsym[DWG];    // own symbols
  int32_t head[1 << HBITS];   // bucket counts -> ends; then histograms, code tables (H_* below)
  int32_t misc[8];
};
constexpr uint32_t EFF_REACHED = 1u << 18, EFF_EOB = 1u << 19;
// word offsets inside DLds::head once the buckets are dead
enum { H_LL = 0, H_D = 288, H_CL = 320, C_LL = 352, C_D = 640, C_CL = 672, H_TOK = 704,
       H_SORT = 864, H_W = 1152, H_LEN = 1440, H_LEN_D = 1728, H_LEN_CL = 1760, H_SORT_D = 1792,
       H_W_D = 1824, H_CNT = 1856, H_CNT_D = 1890, H_BL = 1924, H_END = 1956 };
static_assert(H_END <= (1 << HBITS), "code tables fit the head table");
constexpr uint8_t c_clord[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// Code lengths (<= maxlen) of an alphabet of m <= 286 symbols from frequencies f, by one wave:
// a rank sort (frequency, symbol), then on lane 0 the in-place minimum-redundancy algorithm of
// Moffat and Katajainen and the Kraft fix-up that caps the lengths (the usual length-limiting
// heuristic: move codes from longer to shorter levels until the code is complete).  len[] is
// written for every symbol (0 = unused).  Fewer than two used symbols get lengths 1 (a complete
// code, which every inflater accepts).
__device__ void build_lengths(const int32_t* f, int m, int maxlen, int32_t* sorted, int32_t* w,
                              int32_t* len, int32_t* cnt, int lane) {
  int used = 0;
  for (int s0 = 0; s0 < m; s0 += 64) {
    const int s = s0 + lane;
    const bool u = s < m && f[s] > 0;
    used += __popcll(__ballot(u));
  }
  for (int s = lane; s < m; s += 64) {
    len[s] = 0;
    const int fs = f[s];
    if (fs <= 0) continue;
    int r = 0;
    for (int k = 0; k < m; k++) {
      const int fk = f[k];
      r += fk > 0 && (fk < fs || (fk == fs && k < s));
    }
    sorted[r] = s;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  if (lane != 0) return;
  if (used < 2) {
    // one or no used symbol: symbols 0 and 1 (or the used one and another) get length 1
    int a = used == 1 ? sorted[0] : 0;
    int c = a == 0 ? 1 : 0;
    len[a] = 1;
    len[c] = 1;
    return;
  }
  const int n = used;
  for (int i = 0; i < n; i++) w[i] = f[sorted[i]];
  // Moffat-Katajainen: w ascending -> code lengths (w[0] longest)
  w[0] += w[1];
  int root = 0, leaf = 2;
  for (int next = 1; next < n - 1; next++) {
    if (leaf >= n || w[root] < w[leaf]) { w[next] = w[root]; w[root++] = next; }
    else w[next] = w[leaf++];
    if (leaf >= n || (root < next && w[root] < w[leaf])) { w[next] += w[root]; w[root++] = next; }
    else w[next] += w[leaf++];
  }
  w[n - 2] = 0;
  for (int next = n - 3; next >= 0; next--) w[next] = w[w[next]] + 1;
  int avbl = 1, usedn = 0, dpth = 0;
  root = n - 2;
  int next = n - 1;
  while (avbl > 0) {
    while (root >= 0 && w[root] == dpth) { usedn++; root--; }
    while (avbl > usedn) { w[next--] = dpth; avbl--; }
    avbl = 2 * usedn;
    dpth++;
    usedn = 0;
  }
  // counts per length (cnt: 33 LDS words), capped at maxlen, Kraft fix-up
  for (int l = 0; l <= 32; l++) cnt[l] = 0;
  for (int i = 0; i < n; i++) cnt[min(w[i], 32)]++;
  for (int l = maxlen + 1; l <= 32; l++) { cnt[maxlen] += cnt[l]; cnt[l] = 0; }
  uint32_t total = 0;
  for (int l = maxlen; l > 0; l--) total += (uint32_t)cnt[l] << (maxlen - l);
  while (total != (1u << maxlen)) {
    cnt[maxlen]--;
    for (int l = maxlen - 1; l > 0; l--)
      if (cnt[l]) { cnt[l]--; cnt[l + 1] += 2; break; }
    total--;
  }
  // shortest codes to the most frequent symbols
  int j = n;
  for (int l = 1; l <= maxlen; l++)
    for (int c = cnt[l]; c > 0; c--) len[sorted[--j]] = l;
}

// Canonical codes (RFC 1951 3.2.2), bit-reversed for the LSB-first stream: code | len << 16.
// bl: 32 LDS words of scratch (length counts, then next codes).
__device__ void canon_codes(const int32_t* len, int m, uint32_t* code, int32_t* bl) {
  for (int l = 0; l < 32; l++) bl[l] = 0;
  for (int s = 0; s < m; s++) bl[len[s]]++;
  bl[0] = 0;
  uint32_t c = 0;
  for (int l = 1; l < 16; l++) {
    c = (c + (uint32_t)bl[l - 1]) << 1;
    bl[16 + l] = (int32_t)c;
  }
  for (int s = 0; s < m; s++) {
    const int l = len[s];
    code[s] = l ? (rev((uint32_t)bl[16 + l]++, l) | ((uint32_t)l << 16)) : 0u;
  }
}

// 4 bytes at an arbitrary LDS offset x from two aligned words
__device__ inline uint32_t ld4(const uint8_t* in, int x) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(in + (x & ~3));
  return __builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)(x & 3));  // byte shift
}

// Staged symbol word: litlen symbol | length extra << 9 | distance symbol << 14 | distance extra << 19
__device__ inline uint32_t sym_ll(uint32_t w) { return w & 511; }
__device__ inline uint32_t sym_lx(uint32_t w) { return (w >> 9) & 31; }
__device__ inline uint32_t sym_d(uint32_t w) { return (w >> 14) & 31; }
__device__ inline uint32_t sym_dx(uint32_t w) { return w >> 19; }
__device__ inline int lextra_bits(int s) { return (s < 265 || s == 285) ? 0 : (s - 261) >> 2; }
__device__ inline int dextra_bits(int d) { return d < 4 ? 0 : (d - 2) >> 1; }
__device__ inline int fixed_len_of(int s) { return s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8; }

struct ImgOut {  // LSB-first bits OR-ed into the LDS image from bit position p on
  uint32_t* img;
  uint64_t acc;
  int n;
  uint32_t w;
  __device__ ImgOut(uint32_t* im, uint32_t p) : img(im), acc(0), n((int)(p & 31)), w(p >> 5) {}
  __device__ void put(uint32_t v, int len) {
    acc |= (uint64_t)v << n;
    n += len;
    if (n >= 32) {
      atomicOr(&img[w++], (uint32_t)acc);
      acc >>= 32;
      n -= 32;
    }
  }
  __device__ void flush() {
    if (n > 0) atomicOr(&img[w], (uint32_t)acc);
  }
};

__device__ inline uint32_t hash3(const uint8_t* in, int p) {
  const uint32_t v = (uint32_t)in[p] | ((uint32_t)in[p + 1] << 8) | ((uint32_t)in[p + 2] << 16);
  return (v * 2654435761u) >> (32 - HBITS);
}

__device__ inline int sym_bytes(uint32_t w) {  // uncompressed bytes of a staged symbol
  const uint32_t ll = sym_ll(w);
  return ll < 256 ? 1 : (int)c_lbase[ll - 257] + (int)sym_lx(w);
}
__device__ inline uint64_t lanes_below(int lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }

// Match finder over the block's hash buckets: bl holds every position with a >= 3-byte suffix,
// grouped by bucket (hash3) and ascending inside a bucket; gi[p] is p's index in bl; the bucket of
// hash h ends at head[h] (it starts where bucket h - 1 ends).  The candidates of p are the
// entries before gi[p] in its bucket, most recent first -- consecutive words of bl, so all of a
// search's candidate loads are in flight together (no pointer chasing as in zlib's hash chains).
struct Finder {
  const DLds& L;
  const uint16_t* __restrict__ bl;
  const uint16_t* __restrict__ gi;
  int n, chain, nice, good;
  // longest match (>= 3, else 0) at p, at most lim bytes, among `chain` candidates; *dist its
  // distance
  __device__ int find(int p, int lim, int* dist, int chain) const {
    *dist = 0;
    if (lim < 3 || p + 3 > n) return 0;
    const uint32_t h = hash3(L.in, p);
    const int g = gi[p];
    const int lo = max(h ? L.head[h - 1] : 0, g - chain);
    const uint32_t p4 = ld4(L.in, p);
    int best = 0, bd = 0;
    const int cap = min(lim, nice);
    for (int i0 = g - 1; i0 >= lo && best < cap; i0 -= 8) {
      // a batch of 8 candidates: their positions (global) and first / scan-end words (LDS) are
      // all loaded before any is tested, so the batch costs about one load latency of each kind
      int q8[8];
#pragma unroll
      for (int k = 0; k < 8; k++) q8[k] = i0 - k >= lo ? (int)bl[i0 - k] : -1;
      // only a candidate that also matches the byte at `best` can win: the 4 bytes ending there
      // are tested first (zlib's scan_end test), with the best length at the batch start
      const bool use_e = best >= 3;
      const int be = use_e ? best - 3 : 0;
      const uint32_t pe = ld4(L.in, p + be);
      uint32_t x8[8], e8[8];
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int q = q8[k] >= 0 ? q8[k] : p;
        x8[k] = ld4(L.in, q) ^ p4;
        e8[k] = ld4(L.in, q + be) ^ pe;
      }
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int q = q8[k];
        if (q < 0 || p - q > WIN) break;
        if ((x8[k] & 0xffffffu) || (use_e && e8[k])) continue;  // a hash collision / no match at best
        // compared up to `cap` only: the first candidate that reaches it ends the search (the
        // same choice as comparing every candidate in full), and only that one is extended on
        uint32_t x = x8[k];
        int l = 0;
        while (x == 0 && l + 4 < cap) {
          l += 4;
          x = ld4(L.in, q + l) ^ ld4(L.in, p + l);
        }
        l = x ? l + (int)(__builtin_ctz(x) >> 3) : l + 4;
        l = min(l, cap);
        if (l > best) {
          best = l;
          bd = p - q;
        }
        if (best >= cap) break;
      }
    }
    if (best >= cap && cap < lim) {  // the winner, extended to the end of its match
      const int q = p - bd;
      int l = cap;
      uint32_t x = 0;
      while (x == 0 && l < lim) {
        x = ld4(L.in, q + l) ^ ld4(L.in, p + l);
        l += x ? (int)(__builtin_ctz(x) >> 3) : 4;
      }
      best = min(l, lim);
    }
    *dist = bd;
    return best >= 3 ? best : 0;
  }
};

__device__ inline uint32_t lit_word(uint32_t b) { return b; }
__device__ inline uint32_t match_word(int len, int d) {
  int sym, nx, xv, ds, dnx, dxv;
  len_code(len, sym, nx, xv);
  dist_code(d, ds, dnx, dxv);
  return (uint32_t)sym | ((uint32_t)xv << 9) | ((uint32_t)ds << 14) | ((uint32_t)dxv << 19);
}

// One parse step at p (zlib-style lazy evaluation: while the match at the next position is
// longer and the current one shorter than `lazy`, emit a literal and move on; the look-ahead
// search walks a quarter of the candidates once the current match is `good` long, as zlib's
// deflate_slow does): appends its symbols to w[*ns...] and returns the new position.  The step
// depends on p alone, so two parses that reach the same position continue identically (the
// merge rule below).
__device__ int parse_step(const Finder& F, int lazy, int p, uint32_t* w, int* ns) {
  const int n = F.n;
  int d = 0, l = F.find(p, min(MAXM, n - p), &d, F.chain);
  while (l && l < lazy && p + 1 < n) {
    int d2 = 0;
    const int ch = F.good > 0 && l >= F.good ? max(1, F.chain >> 2) : F.chain;
    const int l2 = F.find(p + 1, min(MAXM, n - p - 1), &d2, ch);
    if (l2 <= l) break;
    w[(*ns)++] = lit_word(F.L.in[p]);
    p++;
    l = l2;
    d = d2;
  }
  if (l) {
    w[(*ns)++] = match_word(l, d);
    return p + l;
  }
  w[(*ns)++] = lit_word(F.L.in[p]);
  return p + 1;
}

// Runs f(word) over lane t's effective symbols: its own from the merge index, then its
// continuation, when the parse reaches it (EFF_REACHED).
template <class Fn>
__device__ inline void for_each_sym(const DLds& L, const uint32_t* lane_w, int t, Fn f) {
  const uint32_t e = L.lane_eff[t];
  if (!(e & EFF_REACHED)) return;
  const int k0 = (int)(e & 511), nc = (int)((e >> 9) & 511), ns = L.lane_nsym[t];
  for (int k = k0; k < ns; k++) f(lane_w[k]);
  for (int k = 0; k < nc; k++) f(lane_w[OWN_WORDS + k]);
}

__global__ __launch_bounds__(DWG) void bgzf_deflate_kernel(const uint8_t* __restrict__ src,
                                                           int64_t n_in, int64_t blk0,
                                                           int64_t nblk, uint32_t* __restrict__ stage,
                                                           uint16_t* __restrict__ link,
                                                           uint8_t* __restrict__ out_slots,
                                                           int32_t* __restrict__ out_size,
                                                           uint64_t* __restrict__ tim, int chain,
                                                           int lazy, int nice, int good) {
  __shared__ DLds L;
  uint64_t tm[8];
  int ti = 0;
#define DTS()                                                            \
  do {                                                                   \
    if (tim && threadIdx.x == 0 && ti < 8) tm[ti++] = __builtin_amdgcn_s_memtime(); \
  } while (0)
  DTS();
  const int64_t b = (int64_t)blockIdx.x;  // block within this launch
  if (b >= nblk) return;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t base = (blk0 + b) * (int64_t)BLK_U;
  const int n = (int)min<int64_t>(BLK_U, n_in - base);
  // load (16-byte loads where aligned)
  for (int i = t; i < 256; i += DWG) L.crc_t[i] = c_dcrc[i];
  for (int i = t; i < (1 << HBITS); i += DWG) L.head[i] = 0;
  if (t < 8) L.misc[t] = 0;
  {
    const uint8_t* s = src + base;
    const int head = (int)((16 - (reinterpret_cast<uintptr_t>(s) & 15)) & 15);
    const int h = min(head, n);
    for (int i = t; i < h; i += DWG) L.in[i] = s[i];
    const int nv = (n - h) / 16;
    for (int i = t; i < nv; i += DWG) {
      const uint4 v = *reinterpret_cast<const uint4*>(s + h + 16 * i);
      uint8_t* d = L.in + h + 16 * i;
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 16; k++) d[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
    }
    for (int i = h + 16 * nv + t; i < n; i += DWG) L.in[i] = s[i];
    if (t < 16) L.in[n + t] = 0;  // the 4-byte compares read up to 3 bytes past the end
  }
  __syncthreads();
  DTS();
  const int s0 = min(n, t * SEG), s1 = min(n, s0 + SEG);
  // ---- CRC32 of the segment (raw register, init 0)
  {
    uint32_t c = 0;
    for (int i = s0; i < s1; i++) c = L.crc_t[(c ^ L.in[i]) & 0xff] ^ (c >> 8);
    L.lane_crc[t] = gf2_mul(x8n((uint32_t)(n - s1)), c);
  }
  // ---- hash buckets of every position with a 3-byte suffix: counts, then bucket ends by a scan
  for (int p = t; p + 3 <= n; p += DWG) atomicAdd(&L.head[hash3(L.in, p)], 1);
  __syncthreads();
  {  // exclusive scan of the 2048 counts: 8 per thread
    constexpr int PER = (1 << HBITS) / DWG;
    int v[PER], sum = 0;
#pragma unroll
    for (int k = 0; k < PER; k++) {
      v[k] = L.head[PER * t + k];
      sum += v[k];
    }
    int inc = sum;
    for (int d = 1; d < 64; d <<= 1) {
      const int y = __shfl_up(inc, d, 64);
      if (lane >= d) inc += y;
    }
    if (lane == 63) L.lane_mrg[wv] = (uint32_t)inc;
    __syncthreads();
    int off = inc - sum;
    for (int w = 0; w < wv; w++) off += (int)L.lane_mrg[w];
#pragma unroll
    for (int k = 0; k < PER; k++) {
      L.head[PER * t + k] = off;  // the bucket's cursor: its start, advanced by the scatter
      off += v[k];
    }
  }
  __syncthreads();
  // ---- ordered scatter: positions in stripes of 256, ascending inside each bucket.  Inside a
  //      wave the lanes with equal hashes are found by one ballot per hash bit; the four waves of
  //      a stripe take their cursors in turn (one barrier each).  Afterwards head[h] is the end
  //      of bucket h.
  uint16_t* bl = link + b * (2 * 65536);
  uint16_t* gi = bl + 65536;
  for (int r = 0; r * DWG < n; r++) {
    const int p = r * DWG + t;
    const bool valid = p + 3 <= n;
    const uint32_t h = valid ? hash3(L.in, p) : 0u;
    uint64_t m = __ballot(valid);
#pragma unroll
    for (int k = 0; k < HBITS; k++) {
      const bool bit = (h >> k) & 1u;
      const uint64_t bk = __ballot(bit);
      m &= bit ? bk : ~bk;
    }
    const uint64_t bel = m & lanes_below(lane);
    int rank = 0;
    for (int w = 0; w < DWG / 64; w++) {
      if (wv == w && valid) {
        rank = L.head[h] + __popcll(bel);
        if (lane == 63 || !(m >> (lane + 1))) L.head[h] = rank + 1;  // the group's last lane
      }
      __syncthreads();
    }
    if (valid) {
      bl[rank] = (uint16_t)p;
      gi[p] = (uint16_t)rank;
    }
  }
  __threadfence_block();
  __syncthreads();
  DTS();
  // ---- speculative parse: lane t from its segment start to the first symbol boundary at or past
  //      its end (a match may run on past it)
  uint32_t* lane_w = stage + ((int64_t)b * DWG + t) * LANE_WORDS;
  const Finder F{L, bl, gi, n, min(chain, MAXCAND), nice, good};
  {
    int ns = 0, p = s0;
    while (p < s1) p = parse_step(F, lazy, p, lane_w, &ns);
    L.lane_nsym[t] = (uint16_t)ns;
    L.lane_bits[t] = (uint32_t)p;  // exit
    L.lane_eff[t] = 0;
  }
  __threadfence_block();
  __syncthreads();
  // ---- continuation: from its exit, lane t parses on until it reaches a symbol boundary of a
  //      later lane's speculative parse (the same position continues identically), skipping
  //      lanes whose whole parse it overruns
  {
    int E = (int)L.lane_bits[t], u = t + 1, k = 0, nc = 0;
    int pu = min(n, u * SEG);
    bool over = false;
    for (;;) {
      if (E >= n) {
        u = DWG;
        k = 0;
        break;
      }
      if (u >= DWG || u * SEG >= n) {  // no later lane holds symbols: parse on to the end (these
        if (nc > CONT_WORDS - 40) {    // empty lanes used to be skipped as "overrun", which ended
          over = true;                 // the block one symbol short when E stopped just before n)
          break;
        }
        int nn = OWN_WORDS + nc;
        E = parse_step(F, lazy, E, lane_w, &nn);
        nc = nn - OWN_WORDS;
        continue;
      }
      const int nu = L.lane_nsym[u];
      const uint32_t* uw = stage + ((int64_t)b * DWG + u) * LANE_WORDS;
      while (k < nu && pu < E) pu += sym_bytes(uw[k++]);
      if (pu == E) break;  // merged: lane u's symbols from k on
      if (k == nu) {       // lane u's whole parse lies before E
        u++;
        k = 0;
        pu = min(n, u * SEG);
        continue;
      }
      if (nc > CONT_WORDS - 40) {  // (a step appends at most lazy + 1 <= 33 symbols)
        // no merge within the staging (e.g. one repeated byte: 258-byte matches from lane 0's
        // positions 1 + 258 k never meet another lane's 255 u + 258 k): end exactly on lane u's
        // boundary pu > E, with matches cut to fit and literals for the last < 3 bytes -- a valid
        // parse that merges, where round 3 stored the whole block
        while (E < pu && nc < CONT_WORDS) {
          int d = 0;
          const int l = F.find(E, min(MAXM, pu - E), &d, F.chain);
          lane_w[OWN_WORDS + nc++] = l ? match_word(l, d) : lit_word(F.L.in[E]);
          E += l ? l : 1;
        }
        if (E == pu) break;  // merged: lane u's symbols from k on
        over = true;         // (a gap of literals longer than the staging: stored)
        break;
      }
      int nn = OWN_WORDS + nc;
      E = parse_step(F, lazy, E, lane_w, &nn);
      nc = nn - OWN_WORDS;
    }
    L.lane_mrg[t] = (uint32_t)u | ((uint32_t)k << 9) | ((uint32_t)nc << 18) | (over ? 1u << 27 : 0u);
  }
  __threadfence_block();
  __syncthreads();
  // ---- the parse of the block: lane 0, then the lane each continuation merged into
  if (t == 0) {
    int cur = 0, k0 = 0;
    for (int it = 0; it <= DWG; it++) {
      const uint32_t m = L.lane_mrg[cur];
      if ((m >> 27) & 1u) {
        L.misc[7] = 2;  // a continuation overflowed: the block is stored
        break;
      }
      const int u = (int)(m & 511), k = (int)((m >> 9) & 511);
      L.lane_eff[cur] = (uint32_t)k0 | (m & (511u << 18)) >> 9 | EFF_REACHED | (u >= DWG ? EFF_EOB : 0u);
      if (u >= DWG) break;
      cur = u;
      k0 = k;
    }
  }
  int32_t* H = L.head;  // the buckets are dead from here
  __syncthreads();
  for (int i = t; i < H_CL + 32; i += DWG) H[i] = 0;
  __syncthreads();
  // histograms of the effective symbols
  for_each_sym(L, lane_w, t, [&](uint32_t x) {
    const uint32_t ll = sym_ll(x);
    atomicAdd(&H[H_LL + ll], 1);
    if (ll > 256) atomicAdd(&H[H_D + sym_d(x)], 1);
  });
  if (L.lane_eff[t] & EFF_EOB) atomicAdd(&H[H_LL + 256], 1);
  const bool over = L.misc[7] == 2;
  __threadfence_block();
  __syncthreads();
  DTS();
  // ---- dynamic Huffman codes: wave 0 the literal/length alphabet, wave 1 the distances
  if (wv == 0) build_lengths(H + H_LL, 286, 15, H + H_SORT, H + H_W, H + H_LEN, H + H_CNT, lane);
  if (wv == 1) build_lengths(H + H_D, 30, 15, H + H_SORT_D, H + H_W_D, H + H_LEN_D, H + H_CNT_D, lane);
  __syncthreads();
  if (t == 0) {
    canon_codes(H + H_LEN, 286, reinterpret_cast<uint32_t*>(H + C_LL), H + H_BL);
    canon_codes(H + H_LEN_D, 30, reinterpret_cast<uint32_t*>(H + C_D), H + H_BL);
    // code-length sequence, run-length coded (16: repeat 3-6, 17: 3-10 zeros, 18: 11-138 zeros)
    int nlit = 286, ndist = 30;
    while (nlit > 257 && H[H_LEN + nlit - 1] == 0) nlit--;
    while (ndist > 1 && H[H_LEN_D + ndist - 1] == 0) ndist--;
    uint16_t* tok = reinterpret_cast<uint16_t*>(H + H_TOK);
    int nt = 0;
    const int N = nlit + ndist;
    auto L_at = [&](int i) { return i < nlit ? H[H_LEN + i] : H[H_LEN_D + i - nlit]; };
    for (int i = 0; i < N;) {
      const int v = L_at(i);
      int run = 1;
      while (i + run < N && L_at(i + run) == v) run++;
      int r = run;
      if (v == 0) {
        while (r >= 11) { const int k = min(r, 138); tok[nt++] = (uint16_t)(18 | ((k - 11) << 5)); r -= k; }
        if (r >= 3) { tok[nt++] = (uint16_t)(17 | ((r - 3) << 5)); r = 0; }
        while (r > 0) { tok[nt++] = 0; r--; }
      } else {
        tok[nt++] = (uint16_t)v;
        r--;
        while (r >= 3) { const int k = min(r, 6); tok[nt++] = (uint16_t)(16 | ((k - 3) << 5)); r -= k; }
        while (r > 0) { tok[nt++] = (uint16_t)v; r--; }
      }
      i += run;
    }
    for (int k = 0; k < nt; k++) H[H_CL + (tok[k] & 31)]++;
    L.misc[2] = nlit;
    L.misc[3] = ndist;
    L.misc[4] = nt;
  }
  __syncthreads();
  if (wv == 0) build_lengths(H + H_CL, 19, 7, H + H_SORT, H + H_W, H + H_LEN_CL, H + H_CNT, lane);
  __syncthreads();
  if (t == 0) {
    canon_codes(H + H_LEN_CL, 19, reinterpret_cast<uint32_t*>(H + C_CL), H + H_BL);
    int ncl = 19;
    while (ncl > 4 && H[H_LEN_CL + c_clord[ncl - 1]] == 0) ncl--;
    L.misc[5] = ncl;
    const uint16_t* tok = reinterpret_cast<const uint16_t*>(H + H_TOK);
    uint32_t hb = 3 + 5 + 5 + 4 + 3 * (uint32_t)ncl;
    for (int k = 0; k < L.misc[4]; k++) {
      const int sy = tok[k] & 31;
      hb += (uint32_t)H[H_LEN_CL + sy] + (sy == 16 ? 2 : sy == 17 ? 3 : sy == 18 ? 7 : 0);
    }
    L.misc[6] = (int32_t)hb;  // dynamic header bits
  }
  __syncthreads();
  DTS();
  // ---- bits per lane under the dynamic and the fixed code
  {
    const uint32_t* cll = reinterpret_cast<const uint32_t*>(H + C_LL);
    const uint32_t* cd = reinterpret_cast<const uint32_t*>(H + C_D);
    uint32_t bdyn = 0, bfix = 0;
    for_each_sym(L, lane_w, t, [&](uint32_t x) {
      const int ll = (int)sym_ll(x);
      int extra = 0;
      if (ll > 256) {
        const int d = (int)sym_d(x);
        extra = lextra_bits(ll) + dextra_bits(d);
        bdyn += cd[d] >> 16;
        bfix += 5;
      }
      bdyn += (cll[ll] >> 16) + extra;
      bfix += fixed_len_of(ll) + extra;
    });
    if (L.lane_eff[t] & EFF_EOB) {
      bdyn += cll[256] >> 16;
      bfix += 7;
    }
    L.lane_bits[t] = bdyn;
    // fixed totals: the sort scratch is dead
    reinterpret_cast<uint32_t*>(H + H_SORT)[t] = bfix;
  }
  __syncthreads();
  // ---- choose dynamic or fixed; exclusive scan of the chosen lane bit counts; CRC fold
  if (t < 64) {
    uint32_t dsum = 0, fsum = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      dsum += L.lane_bits[4 * t + k];
      fsum += reinterpret_cast<uint32_t*>(H + H_SORT)[4 * t + k];
    }
    for (int o = 32; o >= 1; o >>= 1) {
      dsum += __shfl_xor(dsum, o, 64);
      fsum += __shfl_xor(fsum, o, 64);
    }
    const bool dyn = (uint32_t)L.misc[6] + dsum < 3u + fsum;
    uint32_t v[4], sm = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      v[k] = dyn ? L.lane_bits[4 * t + k] : reinterpret_cast<uint32_t*>(H + H_SORT)[4 * t + k];
      sm += v[k];
    }
    uint32_t inc = sm;
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(inc, d, 64);
      if (t >= d) inc += y;
    }
    const uint32_t hdr_bits = dyn ? (uint32_t)L.misc[6] : 3u;
    uint32_t off = hdr_bits + inc - sm;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      L.lane_bits[4 * t + k] = off;  // now: bit offset of lane 4t+k
      off += v[k];
    }
    if (t == 63) L.misc[0] = (int32_t)(hdr_bits + inc);  // total bits
    if (t == 0) L.misc[7] = dyn ? 1 : 0;
    uint32_t c = L.lane_crc[4 * t] ^ L.lane_crc[4 * t + 1] ^ L.lane_crc[4 * t + 2] ^ L.lane_crc[4 * t + 3];
    for (int o = 32; o >= 1; o >>= 1) c ^= __shfl_xor(c, o, 64);
    if (t == 0) L.misc[1] = (int32_t)(c ^ gf2_mul(x8n((uint32_t)n), 0xffffffffu) ^ 0xffffffffu);
  }
  __syncthreads();
  DTS();
  const bool dyn = L.misc[7] != 0;
  if (!dyn) {  // the fixed code into the code tables
    uint32_t* cll = reinterpret_cast<uint32_t*>(H + C_LL);
    uint32_t* cd = reinterpret_cast<uint32_t*>(H + C_D);
    for (int sy = t; sy < 286; sy += DWG) {
      uint32_t code;
      int cl;
      fixed_ll(sy, code, cl);
      cll[sy] = code | ((uint32_t)cl << 16);
    }
    if (t < 30) cd[t] = rev((uint32_t)t, 5) | (5u << 16);
  }
  const uint32_t total_bits = (uint32_t)L.misc[0];
  const int dbytes = (int)((total_bits + 7) / 8);
  uint8_t* o = out_slots + b * 65536;
  const uint32_t crc = (uint32_t)L.misc[1];
  // stored when the code is no shorter than the bytes themselves (and always when it would not fit)
  const bool stored = over || dbytes > min(MAX_DEFLATE, n + 5);
  int payload;
  if (!stored) {
    // ---- the header, then every lane's symbols, OR-ed into the LDS image (the input is dead)
    uint32_t* img = reinterpret_cast<uint32_t*>(L.in);
    for (int i = t; i < (int)(sizeof(L.in) / 4); i += DWG) img[i] = 0;
    __syncthreads();
    if (t == 0) {
      ImgOut io(img, 0);
      if (!dyn) {
        io.put(3u, 3);  // BFINAL 1, BTYPE 01
      } else {
        io.put(5u, 3);  // BFINAL 1, BTYPE 10
        io.put((uint32_t)(L.misc[2] - 257), 5);
        io.put((uint32_t)(L.misc[3] - 1), 5);
        const int ncl = L.misc[5];
        io.put((uint32_t)(ncl - 4), 4);
        for (int k = 0; k < ncl; k++) io.put((uint32_t)H[H_LEN_CL + c_clord[k]], 3);
        const uint16_t* tok = reinterpret_cast<const uint16_t*>(H + H_TOK);
        const uint32_t* ccl = reinterpret_cast<const uint32_t*>(H + C_CL);
        for (int k = 0; k < L.misc[4]; k++) {
          const int sy = tok[k] & 31, ex = tok[k] >> 5;
          io.put(ccl[sy] & 0xffff, (int)(ccl[sy] >> 16));
          if (sy == 16) io.put((uint32_t)ex, 2);
          else if (sy == 17) io.put((uint32_t)ex, 3);
          else if (sy == 18) io.put((uint32_t)ex, 7);
        }
      }
      io.flush();
    }
    {
      const uint32_t* cll = reinterpret_cast<const uint32_t*>(H + C_LL);
      const uint32_t* cd = reinterpret_cast<const uint32_t*>(H + C_D);
      ImgOut io(img, L.lane_bits[t]);
      for_each_sym(L, lane_w, t, [&](uint32_t x) {
        const int ll = (int)sym_ll(x);
        io.put(cll[ll] & 0xffff, (int)(cll[ll] >> 16));
        if (ll > 256) {
          const int lx = lextra_bits(ll);
          if (lx) io.put(sym_lx(x), lx);
          const int d = (int)sym_d(x);
          io.put(cd[d] & 0xffff, (int)(cd[d] >> 16));
          const int dx = dextra_bits(d);
          if (dx) io.put(sym_dx(x), dx);
        }
      });
      if (L.lane_eff[t] & EFF_EOB) io.put(cll[256] & 0xffff, (int)(cll[256] >> 16));
      io.flush();
    }
    __syncthreads();
    DTS();
    payload = dbytes;
    // stored 16 bytes at a time after the 18-byte header: o + 18 is 2 mod 16, so bytes
    for (int i = t; i < payload; i += DWG) o[18 + i] = L.in[i];
  } else {
    // stored block: BFINAL 1, BTYPE 00, LEN, NLEN, the bytes (from global: LDS image may be dirty)
    payload = n + 5;
    if (t == 0) {
      o[18] = 1;
      o[19] = (uint8_t)n;
      o[20] = (uint8_t)(n >> 8);
      o[21] = (uint8_t)~n;
      o[22] = (uint8_t)(~n >> 8);
    }
    for (int i = t; i < n; i += DWG) o[23 + i] = src[base + i];
  }
  if (t == 0) {
    const int bsize = 18 + payload + 8 - 1;
    const uint8_t hdr[18] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 'B', 'C', 2, 0,
                             (uint8_t)bsize, (uint8_t)(bsize >> 8)};
    for (int i = 0; i < 18; i++) o[i] = hdr[i];
    uint8_t* tr = o + 18 + payload;
    tr[0] = (uint8_t)crc; tr[1] = (uint8_t)(crc >> 8); tr[2] = (uint8_t)(crc >> 16); tr[3] = (uint8_t)(crc >> 24);
    tr[4] = (uint8_t)n; tr[5] = (uint8_t)(n >> 8); tr[6] = (uint8_t)(n >> 16); tr[7] = (uint8_t)(n >> 24);
    out_size[b] = bsize + 1;
  }
  DTS();
  if (tim && t == 0)
    for (int k = 0; k < 8; k++) tim[b * 8 + k] = k < ti ? tm[k] - tm[0] : 0;
#undef DTS
}

// Packs the fixed-stride block slots into one contiguous BGZF stream: one workgroup per block.
__global__ __launch_bounds__(256) void bgzf_pack_kernel(const uint8_t* __restrict__ slots,
                                                        const int32_t* __restrict__ size,
                                                        const int64_t* __restrict__ off, int64_t nblk,
                                                        uint8_t* __restrict__ out) {
  const int64_t b = blockIdx.x;
  if (b >= nblk) return;
  const uint8_t* s = slots + b * 65536;
  uint8_t* d = out + off[b];
  const int n = size[b];
  for (int i = threadIdx.x; i < n; i += 256) d[i] = s[i];
}

struct DefTables {
  std::once_flag once;
  bool ok = false;
};
DefTables g_def[64];

}  // namespace

int64_t bgzf_block_count(int64_t n) { return n <= 0 ? 0 : (n + BLK_U - 1) / BLK_U; }
size_t bgzf_stage_bytes(int64_t nblk) { return (size_t)nblk * DWG * LANE_WORDS * 4; }
size_t bgzf_link_bytes(int64_t nblk) { return (size_t)nblk * 2 * 65536 * sizeof(uint16_t); }

bool deflate_tables(int device) {
  if (device < 0 || device >= 64) return false;
  DefTables& D = g_def[device];
  std::call_once(D.once, [&] {
    uint32_t crc[256], x2n[32];
    for (uint32_t i = 0; i < 256; i++) {
      uint32_t c = i;
      for (int k = 0; k < 8; k++) c = c & 1 ? (c >> 1) ^ 0xEDB88320u : c >> 1;
      crc[i] = c;
    }
    auto mul = [](uint32_t a, uint32_t b) {
      uint32_t m = 1u << 31, p = 0;
      for (int i = 0; i < 32; i++) {
        if (a & m) p ^= b;
        m >>= 1;
        b = b & 1 ? (b >> 1) ^ 0xEDB88320u : b >> 1;
      }
      return p;
    };
    uint32_t p = 1u << 30;  // x^1
    for (int k = 0; k < 32; k++) {
      x2n[k] = p;
      p = mul(p, p);
    }
    int prev = -1;
    (void)hipGetDevice(&prev);
    bool ok = hipSetDevice(device) == hipSuccess;
    ok = ok && hipMemcpyToSymbol(HIP_SYMBOL(c_dcrc), crc, sizeof crc) == hipSuccess;
    ok = ok && hipMemcpyToSymbol(HIP_SYMBOL(c_x2n), x2n, sizeof x2n) == hipSuccess;
    if (prev >= 0) (void)hipSetDevice(prev);
    D.ok = ok;
  });
  return D.ok;
}

void launch_bgzf_deflate(const uint8_t* src, int64_t n_in, int64_t blk0, int64_t nblk,
                         uint32_t* stage, uint16_t* link, uint8_t* out_slots, int32_t* out_size,
                         uint64_t* tim, hipStream_t s) {
  if (nblk <= 0) return;
  // DQ_DEFLATE="chain,lazy,nice[,good]": match-search effort (default 96,32,96,8: htsjdk level 5's
  // ratio on the WGS stream; 48,24,48,8 is 40 % faster at a 1.4 % lower ratio, profiles/r3as_*;
  // zlib level 5 is 32,16,32,8 with hash chains, tools/deflate_model.c; good 0 = always the full
  // chain; read at every launch, so a test can sweep settings in one process)
  const int4 cfg = [] {
    int c = 96, l = 32, n = 96, g = 8;
    if (const char* e = getenv("DQ_DEFLATE")) sscanf(e, "%d,%d,%d,%d", &c, &l, &n, &g);
    return make_int4(std::max(1, std::min(c, MAXCAND)), std::max(0, std::min(l, 32)), std::max(3, n),
                     std::max(0, g));
  }();
  hipLaunchKernelGGL(bgzf_deflate_kernel, dim3((unsigned)nblk), dim3(DWG), 0, s, src, n_in, blk0, nblk,
                     stage, link, out_slots, out_size, tim, cfg.x, cfg.y, cfg.z, cfg.w);
}

void launch_bgzf_pack(const uint8_t* slots, const int32_t* size, const int64_t* off, int64_t nblk,
                      uint8_t* out, hipStream_t s) {
  if (nblk <= 0) return;
  hipLaunchKernelGGL(bgzf_pack_kernel, dim3((unsigned)nblk), dim3(256), 0, s, slots, size, off, nblk,
                     out);
}

DQ_CHK_UNIT(deflate)

}  // namespace dq
