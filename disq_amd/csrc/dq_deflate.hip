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
// Three kernels per batch of blocks, everything the match finder touches in LDS:
//   bgzf_parse_kernel: one 1024-thread workgroup per CHUNK, half a block (32640 bytes), holding the
//      chunk's bytes plus up to 13600 bytes before it (its window reach) and the hash-bucket lists of
//      all those positions (3 bytes of LDS per position: 160 KB, one workgroup per CU).  A chunk's
//      matches end inside it and reach back at most 13600 bytes before its start (the 32 KiB DEFLATE
//      window inside the first chunk): tools/deflate_model.c puts that at zlib level 5's ratio on
//      the WGS stream and the golden BAM / VCF streams (profiles/r4_deflate_chunk_model.txt).
//   1. Match finder: every position with a 4-byte suffix goes into one of 2048 hash buckets of its
//      first 4 bytes (a 4-byte key keeps 3-byte candidates, which rarely pay for their distance,
//      out of the chain), ascending inside its bucket: counts by LDS atomics, bucket starts by a
//      scan, then four waves scatter four position ranges in order with their own cursors (one
//      LDS atomic add per position: the lanes of one atomic that hit the same cursor get its
//      values in lane order on gfx950 -- observed, not documented -- so equal-hash positions of a
//      step get ascending slots; DQ_SCAT_ATOMIC=0, the `ballot` build, ranks them by ballots):
//      no barrier, no position hashed twice.  A position's candidates are the entries before it in
//      its bucket, most recent first (its own slot is found by a 16-way search of the bucket): a
//      contiguous run of the list, so a search loads 8 candidates and their first 16 bytes at
//      once instead of chasing zlib's hash-chain links one dependent load at a time.
//   2. Parse: the chunk is cut into 32-byte segments; thread t parses segment t from its start
//      with zlib-style lazy evaluation (a match shorter than `lazy` is deferred while the next
//      position's is longer; the look-ahead search walks chain / 4 candidates once the current
//      match is `good` long, as zlib's deflate_slow) and the longest match among `chain`
//      candidates (stopping at `nice`); nothing depends on which lane runs first, so the output
//      is a function of the input: by construction in the ballot build, and in the default
//      build while the hardware keeps the lane order above (tests/test_deflate_gpu.py compares
//      the two builds' bytes).  A parse step depends on its position alone, so two parses that reach the
//      same position continue identically: from its exit, each segment's parse is continued until
//      it hits a symbol boundary of a later segment's parse (usually within a few symbols) and the
//      merge is recorded; after `fmerge` continuation symbols without one (default 1) it is ended
//      on the next boundary of the later segment with a shortened match.  Pointer jumping over the
//      merges from segment 0 marks the segments on the chunk's one parse and the symbol each
//      starts from.  The merged parse is valid but not always the one a single sequential pass
//      would make (0.3% larger on the WGS stream; within 0.5% of zlib level 5 on every golden
//      stream, tests/test_deflate_gpu.py).  Symbols are staged per segment in HBM (one word
//      each); the chunk's literal/length and distance histograms over its parse, its CRC and a
//      word per segment (first symbol, counts) go with them.
//   bgzf_huff_kernel: one 128-thread workgroup per block (7.9 KB of LDS, many per CU).
//   3. Codes: the two chunks' histograms summed; wave 0 builds the literal/length code and wave 1
//      the distance code (a rank sort, Moffat-Katajainen minimum-redundancy lengths, a Kraft
//      fix-up capping them at 15), the code-length sequence is run-length coded; the tables go to
//      the block's record.
//   bgzf_code_kernel: one 1024-thread workgroup per block (136 KB of LDS).
//   4. Emit: the block is coded dynamic (BTYPE 10) or fixed (01), whichever is shorter -- one
//      DEFLATE block per member, as zlib writes a 64 KiB input; each thread's bit count gives its
//      offset by an exclusive scan; wave 0 writes the dynamic header (an item per lane, offsets by
//      a wave scan) while every thread OR-s its two segments' bits into the LDS image of the
//      block.  A block whose code would not fit BSIZE (or whose parse overflowed its
//      staging) is stored (BTYPE 00).
// CRC32: per-lane table CRC over the segment, combined with x^(8 n) mod P multipliers.
// (Defaults chain 32, lazy 16, nice 32, good 8: zlib level 5's.)
#include "dq_internal.h"

#include <algorithm>
#include <mutex>

namespace dq {
namespace {

constexpr int BLK_U = 65280;             // htsjdk DEFAULT_UNCOMPRESSED_BLOCK_SIZE
constexpr int NCH = 2;                   // chunks per block
constexpr int CH = BLK_U / NCH;          // 32640 bytes per chunk
constexpr int PSEG = 32;                 // bytes per parse segment
constexpr int PL = CH / PSEG;            // 1020 segments per chunk
constexpr int MSEG = 1024;               // segment slots per chunk (staging, lane words)
constexpr int PWG = 1024;                // threads per chunk workgroup: one per segment
constexpr int XW = 13600;                // window reach before the chunk start
constexpr int NPMAX = CH + XW;           // bytes (positions) a chunk workgroup holds
constexpr int HBITS = 11;                // hash buckets
constexpr int MAXM = 258;
constexpr int WIN = 32768;               // DEFLATE window
// Staged matches (literals are the input bytes between them: the code kernel reads those
// itself): a word each, gap of literals before it | (length - 3) << 9 | (distance - 1) << 17.  Up
// to MB_INL matches of a segment's own parse (or of its continuation) go to the chunk's dense
// area at an offset taken from an LDS counter when the part ends; a part with more goes whole to
// the chunk's overflow pool (OWN_CAP or CONT_CAP words taken from another counter when its ninth
// match comes; a pathological chunk that exhausts the pool has its block stored).
#ifndef DQ_MB_INL
#define DQ_MB_INL 8  // (<= 8; a build with fewer spills to the pool more often)
#endif
constexpr int MB_INL = DQ_MB_INL;
static_assert(MB_INL >= 1 && MB_INL <= 8, "register-held matches");
constexpr int CONT_WORDS = 156;          // continuation symbols at most
constexpr int OWN_CAP = 16;              // own matches (a 32-byte segment's, + one past its end)
constexpr int CONT_CAP = 160;            // continuation matches (<= CONT_WORDS)
constexpr int DENSE_WORDS = 2 * MSEG * MB_INL;  // per chunk
#ifndef DQ_SCAT_ATOMIC
#define DQ_SCAT_ATOMIC 1  // bucket scatter by LDS atomics (0: by ballot ranking, round 4)
#endif
#ifndef DQ_POOL_WORDS
#define DQ_POOL_WORDS 32768  // (a build with a small pool exercises the exhaustion path)
#endif
constexpr int POOL_WORDS = DQ_POOL_WORDS;       // per chunk
constexpr int64_t STAGE_CH_WORDS = DENSE_WORDS + POOL_WORDS;  // per chunk
constexpr int FMERGE = 1;  // continuation symbols before a forced merge (default; profiles/r4aj_*, r5zc_*)
constexpr int MAX_DEFLATE = 65536 - 26;  // BSIZE limit: 18-byte header + payload + 8 trailer
// a block's output slot: the member's 18-byte header at SLOT_HDR, the deflate payload 16-byte
// aligned at SLOT_HDR + 18, the trailer after it
constexpr int SLOT = 65600, SLOT_HDR = 14, SLOT_PAY = SLOT_HDR + 18;
static_assert(SLOT_PAY % 16 == 0 && SLOT_PAY + MAX_DEFLATE + 4 + 8 <= SLOT && SLOT % 16 == 0, "slot layout");
constexpr int MAXCAND = 128;             // candidates per match search at most (cfg.chain)
constexpr int CWG = 1024;                // threads of the code kernel
constexpr int NLANE = NCH * PL;          // 2040 segments per block; code thread i owns 2i, 2i + 1
constexpr int CSEG = 2;                  // segments per code thread
// per block in `meta`: a word per segment (NCH x MSEG), then NCH chunk records of CI_WORDS
constexpr int CI_WORDS = 320;
enum { CI_LL = 0, CI_D = 286, CI_CRC = 316, CI_OVER = 317, CI_BYTES = 318 };
// then the block's code tables (bgzf_huff_kernel -> bgzf_code_kernel): literal/length, distance
// and code-length codes, the code-length code's lengths, the run-length tokens (2 per word), misc
enum { TB_LL = 0, TB_D = 286, TB_CL = 316, TB_LENCL = 335, TB_TOK = 354, TB_MISC = 512, TB_WORDS = 520 };
// per block in `meta`: four words per segment (NCH x MSEG each), then NCH chunk records of
// CI_WORDS, then the table record.  Segment words (positions chunk-local):
//   SW_RANGE: first | end << 16 of its bytes on the chunk's parse (SW_NONE: not on it)
//   SW_OWN:   own parse start | own parse exit << 16
//   SW_OWNM, SW_CONTM: the own / continuation matches, dense offset | count << 16 | overflow << 24
enum { SW_RANGE = 0, SW_OWN = 1, SW_OWNM = 2, SW_CONTM = 3 };
constexpr uint32_t SW_NONE = 0xffffffffu;
constexpr int CI_OFF = 4 * NCH * MSEG;
constexpr int TB_OFF = CI_OFF + NCH * CI_WORDS;
constexpr int META_WORDS = TB_OFF + TB_WORDS;
static_assert(PL * PSEG == CH && PL <= MSEG && PL <= PWG && NLANE <= CSEG * CWG, "segment layout");
static_assert(CONT_WORDS < 256 && DENSE_WORDS <= 65536, "segment word fields");

__constant__ uint32_t c_dcrc[256];
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

// word offsets of the code tables in the code kernel's table area
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
#pragma unroll 8
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

// Canonical codes (RFC 1951 3.2.2), bit-reversed for the LSB-first stream: code | len << 16, by one
// wave: length counts by ballots, a symbol's code = its length's first code + its rank among the
// symbols of that length before it (ballots again), no serial loop over symbols.
__device__ void canon_codes_wave(const int32_t* len, int m, uint32_t* code, int lane) {
  int cnt[16];
#pragma unroll
  for (int l = 0; l < 16; l++) cnt[l] = 0;
  for (int s0 = 0; s0 < m; s0 += 64) {
    const int l = s0 + lane < m ? len[s0 + lane] : 0;
#pragma unroll
    for (int L = 1; L < 16; L++) cnt[L] += __popcll(__ballot(l == L));
  }
  uint32_t next[16];
  uint32_t c = 0;
  next[0] = 0;
#pragma unroll
  for (int L = 1; L < 16; L++) {
    c = (c + (uint32_t)(L > 1 ? cnt[L - 1] : 0)) << 1;
    next[L] = c;
  }
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  for (int s0 = 0; s0 < m; s0 += 64) {
    const int s = s0 + lane;
    const int l = s < m ? len[s] : 0;
    uint32_t mine = 0;
#pragma unroll
    for (int L = 1; L < 16; L++) {
      const uint64_t b = __ballot(l == L);
      if (l == L) mine = next[L] + (uint32_t)__popcll(b & below);
      next[L] += (uint32_t)__popcll(b);
    }
    if (s < m) code[s] = l ? (rev(mine, l) | ((uint32_t)l << 16)) : 0u;
  }
}

#ifndef DQ_LDS_UNALIGNED
#define DQ_LDS_UNALIGNED 1
#endif
#ifndef DQ_BATCH_REDUCE
#define DQ_BATCH_REDUCE 1  // a candidate batch without a branch per candidate (else the loop)
#endif
#if DQ_LDS_UNALIGNED
// 4 / 8 bytes at an arbitrary LDS offset x: one unaligned ds_read_b32 / ds_read_b64 (measured
// faster than aligned words + byte shifts, profiles/r4m_deflate_sweep.txt)
__device__ inline uint32_t ld4(const uint8_t* in, int x) {
  uint32_t v;
  __builtin_memcpy(&v, in + x, 4);
  return v;
}
__device__ inline uint64_t ld8(const uint8_t* in, int x) {
  uint64_t v;
  __builtin_memcpy(&v, in + x, 8);
  return v;
}
#else
// 4 / 8 bytes at an arbitrary LDS offset x from aligned words and byte shifts
__device__ inline uint32_t ld4(const uint8_t* in, int x) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(in + (x & ~3));
  return __builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)(x & 3));
}
__device__ inline uint64_t ld8(const uint8_t* in, int x) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(in + (x & ~3));
  const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], sh = (uint32_t)(x & 3);
  return (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, sh) |
         (uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32;
}
#endif

__device__ inline int fixed_len_of(int s) { return s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8; }

// LSB-first bits into the LDS image from bit position p on: the first word (when p is inside it)
// and the last are shared with the neighbouring bit ranges and OR-ed; the words between are stored
struct ImgOut {
  uint32_t* img;
  uint64_t acc;
  int n;
  uint32_t w, w0;
  __device__ ImgOut(uint32_t* im, uint32_t p)
      : img(im), acc(0), n((int)(p & 31)), w(p >> 5), w0((p & 31) ? p >> 5 : ~0u) {}
  __device__ void put(uint32_t v, int len) {
    acc |= (uint64_t)v << n;
    n += len;
    if (n >= 32) {
      DQ_CHK(w < 65536 / 4, CHK_Z_IMAGE);
      if (w == w0) atomicOr(&img[w], (uint32_t)acc);
      else img[w] = (uint32_t)acc;
      w++;
      acc >>= 32;
      n -= 32;
    }
  }
  __device__ void flush() {
    DQ_CHK(n <= 0 || w < 65536 / 4, CHK_Z_IMAGE);
    if (n > 0) atomicOr(&img[w], (uint32_t)acc);
  }
};

// bucket hash of the 4 bytes at p: candidates share 4 bytes (rarely 3 or fewer, on a collision).
// A 4-byte key keeps 3-byte matches (which rarely pay for their distance) out of the chain, so
// the same chain reaches more useful candidates: ratio 2.93 at chain 32 against 2.86 at chain 96
// with a 3-byte key on the WGS stream (tools/deflate_model.c, profiles/r4_deflate_chunk_model.txt)
__device__ inline uint32_t hash4(const uint8_t* in, int p) {
  return (ld4(in, p) * 2654435761u) >> (32 - HBITS);
}
// the same from aligned words (faster for a pass over every position: consecutive lanes' words
// coincide)
__device__ inline uint32_t hash4a(const uint8_t* in, int p) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(in + (p & ~3));
  return (__builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)(p & 3)) * 2654435761u) >> (32 - HBITS);
}

__device__ inline uint64_t lanes_below(int lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }

__device__ inline uint32_t mword(int gap, int len, int d) {
  return (uint32_t)gap | (uint32_t)(len - 3) << 9 | (uint32_t)(d - 1) << 17;
}
__device__ inline int mw_gap(uint32_t w) { return (int)(w & 511); }
__device__ inline int mw_len(uint32_t w) { return (int)((w >> 9) & 255) + 3; }
__device__ inline int mw_dist(uint32_t w) { return (int)(w >> 17) + 1; }


constexpr int SCAT_WAVES = 4;  // waves of the bucket scatter: one position range each
constexpr int NQ = (MSEG + PWG - 1) / PWG;  // segments per thread in the merge phase
constexpr int CRC_BYTES = CH / (PWG - 64 * SCAT_WAVES) + 1;  // per thread of the other waves (the CRC)
// head first, then in and bl: every array a search reads starts below 64 KiB, so its constant
// offset folds into the ds_read offset field (one VALU add fewer per access; round 5 had head past
// in and bl, at 138 KiB, as the inflate's tables were before its image moved last)
struct alignas(16) PLds {
  int32_t head[1 << HBITS];   // bucket counts -> starts (wave 0's cursors) -> ends; later the
                              // chunk's histograms
  uint8_t in[NPMAX + 16];     // bytes [r0, ce) of the block (+ zero pad for the 4/8-byte compares)
  uint16_t bl[NPMAX];         // positions grouped by hash bucket, ascending inside a bucket
  union {
    struct {
      uint32_t seg_exit[MSEG];  // the parse's exit of each segment; later jump pointers, first symbols
      uint32_t seg_mrg[MSEG];   // continuation: merge segment | symbol << 11 | count << 18 | over << 26
      uint8_t seg_mark[MSEG];   // on the chunk's parse
      uint32_t sbits[PL];       // symbol starts of each segment's own parse inside it (a deferred
                                // literal past the segment end is left out): one word each
    };
    // the bucket build (before any of the above is live): the counts of scatter waves 0..2's
    // position ranges, two 16-bit counts per word, then those waves' successors' cursors
    uint32_t cnt[SCAT_WAVES - 1][1 << (HBITS - 1)];
  };
  int32_t hist[CI_CRC];       // literal/length and distance histograms of every symbol parsed
  uint32_t wred[2 * (PWG / 64)];  // scan totals per wave, then the CRC waves' registers
  int32_t misc[8];
};
static_assert(sizeof(PLds) <= 160 * 1024, "one chunk workgroup per CU");
static_assert(offsetof(PLds, bl) < 65536 - 4096, "the search arrays' offsets fit the DS offset field");
static_assert(PSEG == 32, "a segment's symbol starts are one word of sbits");

// Match finder over the chunk's hash buckets: bl holds every local position x with a 4-byte
// suffix (x + 4 <= np), grouped by bucket (hash4) and ascending inside a bucket; the bucket of
// hash h ends at head[h] (it starts where bucket h - 1 ends).  The candidates of x are the entries
// before x's own slot in its bucket, most recent first -- consecutive words of bl, so all of a
// search's candidate loads are in flight together.
struct Finder {
  const PLds& L;
  int np, chain, nice, good;
  // the slot of x in the ascending list bl[lo, hi), which holds it: 16-way search
  __device__ __attribute__((always_inline)) int slot(int lo, int hi, int x) const {
    int a = lo, b = hi;
    while (b - a > 16) {
      const int st = (b - a) >> 4;
      int m = 0;
#pragma unroll
      for (int k = 1; k < 16; k++) m += (int)L.bl[a + k * st] <= x;
      const int na = a + m * st;
      b = m == 15 ? b : na + st;
      a = na;
    }
    // the last <= 16 entries in two 16-byte reads
    uint4 v0, v1;
    __builtin_memcpy(&v0, &L.bl[a], 16);
    __builtin_memcpy(&v1, &L.bl[a + 8], 16);
    const uint32_t w[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    int c = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) c += a + k < b && (int)((w[k >> 1] >> (16 * (k & 1))) & 0xffffu) < x;
    return a + c;
  }
  // A match search in progress: batches of 8 candidates, resumable, so the lanes of a wave run
  // one batch per step of the parse loop whichever search each is in (a lane whose search ends
  // early starts its next one instead of idling while the wave's longest search finishes).
  struct Search {
    int x, lim, i0, lo, best, bd, cap;
    uint64_t pa, pb;  // the first 16 bytes at x
    bool more;        // batches left
  };
  __device__ __attribute__((always_inline)) void begin(Search& S, int x, int lim, int ch) const {
    S.x = x;
    S.lim = lim;
    S.best = 0;
    S.bd = 0;
    S.cap = min(lim, nice);
    S.more = false;
    if (lim < 3 || x + 4 > np) return;
    const uint32_t h = hash4(L.in, x);
    const int blo = h ? L.head[h - 1] : 0;
    const int g = slot(blo, L.head[h], x);
    S.lo = max(blo, g - ch);
    S.i0 = g - 1;
    S.more = S.i0 >= S.lo;
    S.pa = ld8(L.in, x);
    S.pb = ld8(L.in, x + 8);
  }
  // one batch: 8 candidates' positions in one 16-byte read and their first 16 bytes with 16 loads
  // issued together (lengths < 16, most of them, need no further round trip)
  __device__ __attribute__((always_inline)) void batch(Search& S) const {
    const int x = S.x, i0 = S.i0, lo = S.lo, cap = S.cap;
    int best = S.best, bd = S.bd;
    bool more = true;
    int q8[8];
    uint64_t ya[8], yb[8];
#if DQ_LDS_UNALIGNED
    // entries i0 - 7 .. i0 (below lo, or before bl itself: masked)
    uint4 qq;
    __builtin_memcpy(&qq, &L.bl[i0 - 7], 16);
    const uint32_t qw[4] = {qq.x, qq.y, qq.z, qq.w};
#endif
    // (an entry below lo is the sentinel x itself: one unsigned compare, x - q - 1 < WIN, then
    // rejects it with a candidate at or past x -- which a bucket list out of order could hold --
    // and one beyond the window)
#pragma unroll
    for (int k = 0; k < 8; k++) {
#if DQ_LDS_UNALIGNED
      q8[k] = i0 - k >= lo ? (int)((qw[(7 - k) >> 1] >> (16 * ((7 - k) & 1))) & 0xffffu) : x;
#else
      q8[k] = i0 - k >= lo ? (int)L.bl[i0 - k] : x;
#endif
      ya[k] = ld8(L.in, q8[k]) ^ S.pa;
      yb[k] = ld8(L.in, q8[k] + 8) ^ S.pb;
    }
#if DQ_BATCH_REDUCE
    // the 8 lengths without a branch per candidate, the winner by one max over keys
    // length << 19 | (7 - k) << 16 | distance: the longest, the most recent among equals -- the
    // candidate the sequential loop below would pick, with the same stop at cap
    uint32_t key = 0;
    bool stop = false;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const int q = q8[k];
      const bool valid = (uint32_t)(x - q - 1) < (uint32_t)WIN;
      stop |= !valid;  // the bucket's list or the window ended (candidates: most recent first)
      int l = ya[k] ? (int)(__builtin_ctzll(ya[k]) >> 3)
                    : yb[k] ? 8 + (int)(__builtin_ctzll(yb[k]) >> 3) : 16;
      // (rare) 16 bytes equal: on up to cap, unless the 4 bytes ending at the batch's best differ
      if (valid && l == 16 && l < cap && (best <= 16 || ld4(L.in, q + best - 3) == ld4(L.in, x + best - 3))) {
        while (l < cap) {
          const uint64_t y = ld8(L.in, q + l) ^ ld8(L.in, x + l);
          if (y) {
            l += (int)(__builtin_ctzll(y) >> 3);
            break;
          }
          l += 8;
        }
      }
      l = valid ? min(l, cap) : 0;
      key = max(key, (uint32_t)l << 19 | (uint32_t)(7 - k) << 16 | (uint32_t)(valid ? x - q : 0));
    }
    const int lb = (int)(key >> 19);
    if (lb > best) {
      best = lb;
      bd = (int)(key & 0xffffu);
    }
    more = !stop && best < cap;
#else
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const int q = q8[k];
      if ((uint32_t)(x - q - 1) >= (uint32_t)WIN) {  // past the window (candidates are most recent first)
        more = false;
        break;
      }
      int l = ya[k] ? (int)(__builtin_ctzll(ya[k]) >> 3)
                    : yb[k] ? 8 + (int)(__builtin_ctzll(yb[k]) >> 3) : 16;
      // (rare) 16 bytes equal: on up to cap, unless the 4 bytes ending at `best` differ (then it
      // cannot beat best: zlib's scan_end test)
      if (l == 16 && l < cap && (best <= 16 || ld4(L.in, q + best - 3) == ld4(L.in, x + best - 3))) {
        while (l < cap) {
          const uint64_t y = ld8(L.in, q + l) ^ ld8(L.in, x + l);
          if (y) {
            l += (int)(__builtin_ctzll(y) >> 3);
            break;
          }
          l += 8;
        }
      }
      l = min(l, cap);
      if (l > best) {
        best = l;
        bd = x - q;
      }
      if (best >= cap) {  // the first candidate to reach cap wins
        more = false;
        break;
      }
    }
#endif
    S.best = best;
    S.bd = bd;
    S.i0 = i0 - 8;
    S.more = more && S.i0 >= lo;
  }
  // the search's match (>= 3, else 0), the winner extended to the end of its match; *dist
  __device__ __attribute__((always_inline)) int finish(const Search& S, int* dist) const {
    int best = S.best;
    if (best >= S.cap && S.cap < S.lim) {
      const int q = S.x - S.bd;
      int l = S.cap;
      while (l < S.lim) {
        const uint64_t y = ld8(L.in, q + l) ^ ld8(L.in, S.x + l);
        if (y) {
          l += (int)(__builtin_ctzll(y) >> 3);
          break;
        }
        l += 8;
      }
      best = min(l, S.lim);
    }
    *dist = S.bd;
    return best >= 3 ? best : 0;
  }
  // longest match (>= 3, else 0) at x, at most lim bytes, among `ch` candidates; *dist its
  // distance (the search run to its end at once)
  __device__ __attribute__((always_inline)) int find(int x, int lim, int* dist, int ch) const {
    Search S;
    begin(S, x, lim, ch);
    while (S.more) batch(S);
    return finish(S, dist);
  }
};

// The lane parse loop: zlib-style lazy evaluation (while the match at the next position is longer
// and the current one shorter than `lazy`, emit a literal and move on; the look-ahead search walks
// a quarter of the candidates once the current match is `good` long, as zlib's deflate_slow
// does), as a per-lane state machine: each pass of the loop runs one batch of each lane's current
// search, or ends it and takes the parse decision, so the wave's lanes stay busy however their
// search lengths differ (round 4: one lane in five was active per VALU instruction with the
// searches run to their ends inside each parse step).  A step depends on its position alone, so
// two parses that reach the same position continue identically (the merge rule below).  Matches
// end at the chunk end np.  emit(length, distance, position) takes a symbol (length 0: the
// literal at position); between steps next(x) says what the lane does after a step that ended at
// x (or first, at its start): the position of its next step, NX_WAIT (ask again in the next pass)
// or NX_STOP.  `lazy` and the end `n` a step's matches stop at are read at every step (next() may
// change them: a forced merge's greedy steps up to a boundary).
enum { NX_WAIT = -1, NX_STOP = -2 };
template <class Emit, class Next>
__device__ __attribute__((always_inline)) inline void parse_lanes(const Finder& F, const int& lazy,
                                                                  const int& n, int x0, Emit emit,
                                                                  Next next) {
  Finder::Search S;
  int x = x0, l = 0, d = 0;
  bool lz = false;    // the current search is the look-ahead at x + 1
  bool busy = false;  // a step is in progress
  bool done = false;
  while (__any(!done)) {
    if (!done && !busy) {  // between steps: stop, wait, or begin the next step's search
      const int r = next(x);
      done = r == NX_STOP;
      if (r >= 0) {
        x = r;
        busy = true;
        lz = false;
        F.begin(S, x, min(MAXM, n - x), F.chain);
      }
    }
    if (busy && S.more) F.batch(S);
    if (busy && !S.more) {  // the search ended: the parse decision
      int d2 = 0;
      const int r = F.finish(S, &d2);
      bool end = false;  // emit the pending symbol at x and end the step
      if (!lz) {
        l = r;
        d = d2;
        if (l && l < lazy && x + 1 < n) {
          lz = true;
          F.begin(S, x + 1, min(MAXM, n - x - 1), F.good > 0 && l >= F.good ? max(1, F.chain >> 2) : F.chain);
        } else {
          end = true;
        }
      } else if (r <= l) {
        end = true;
      } else {  // a longer match one on: a literal, and look one further
        emit(0, 0, x);
        x++;
        l = r;
        d = d2;
        if (l < lazy && x + 1 < n)
          F.begin(S, x + 1, min(MAXM, n - x - 1), F.good > 0 && l >= F.good ? max(1, F.chain >> 2) : F.chain);
        else
          end = true;
      }
      if (end) {
        emit(l, d, x);
        x += l ? l : 1;
        busy = false;
        const int r2 = next(x);  // the next step at once (no pass in between)
        done = r2 == NX_STOP;
        if (r2 >= 0) {
          x = r2;
          busy = true;
          lz = false;
          F.begin(S, x, min(MAXM, n - x), F.chain);
        }
      }
    }
  }
}

// The merge fields of seg_mrg: the segment merged into (MSEG = the chunk's end) | the merge
// position's offset from that segment's start << 11 | overflowed << 20
__device__ inline uint32_t mrg_word(int u, int off, bool over) {
  return (uint32_t)u | (uint32_t)off << 11 | (over ? 1u << 20 : 0u);
}
__device__ inline int mrg_lane(uint32_t m) { return (int)(m & 2047); }
__device__ inline int mrg_off(uint32_t m) { return (int)((m >> 11) & 511); }
__device__ inline bool mrg_over(uint32_t m) { return (m >> 20) & 1u; }

// A part's (own parse's or continuation's) match words: the first MB_INL in registers; when the
// part ends they go to the chunk's dense area at an offset from an LDS counter (the dense area is
// packed: the code kernel reads a line per few segments instead of a line per segment part).  A
// part with more is written whole to a `cap`-word area of the overflow pool instead.
struct MBuf {
  uint32_t* pool;
  int* pctr;   // the pool's LDS counter
  int* over;   // the chunk's "store the block" flag
  int cap, po;
  uint32_t p0, p1, p2, p3, p4, p5, p6, p7;
  int n;
  __device__ __attribute__((always_inline)) void put(uint32_t w) {
    p0 = n == 0 ? w : p0;
    p1 = n == 1 ? w : p1;
    p2 = n == 2 ? w : p2;
    p3 = n == 3 ? w : p3;
    p4 = n == 4 ? w : p4;
    p5 = n == 5 ? w : p5;
    p6 = n == 6 ? w : p6;
    p7 = n == 7 ? w : p7;
    if (n >= MB_INL) {
      if (n == MB_INL) {
        po = atomicAdd(pctr, cap);
        if (po + cap <= POOL_WORDS) {
          *reinterpret_cast<uint4*>(pool + po) = make_uint4(p0, p1, p2, p3);
          *reinterpret_cast<uint4*>(pool + po + 4) = make_uint4(p4, p5, p6, p7);
        } else {
          po = -1;
          *over = 1;
        }
      }
      if (po >= 0) pool[po + n] = w;
    }
    n++;
  }
  // the part's segment word (SW_OWNM / SW_CONTM): offset | count << 16 | in the pool << 24 (no
  // matches when the pool ran out: the block is stored)
  __device__ __attribute__((always_inline)) uint32_t publish(uint32_t* dense, int* ctr) {
    if (n > MB_INL) return po >= 0 ? (uint32_t)po | (uint32_t)n << 16 | 1u << 24 : 0u;
    const int o = n ? atomicAdd(ctr, n) : 0;
    uint32_t* d = dense + o;
    if (n > 0) d[0] = p0;
    if (n > 1) d[1] = p1;
    if (n > 2) d[2] = p2;
    if (n > 3) d[3] = p3;
    if (n > 4) d[4] = p4;
    if (n > 5) d[5] = p5;
    if (n > 6) d[6] = p6;
    if (n > 7) d[7] = p7;
    return (uint32_t)o | (uint32_t)n << 16;
  }
};
// the match words a segment word points at
__device__ inline const uint32_t* part_words(const uint32_t* dense, uint32_t m) {
  return dense + ((m >> 24) ? DENSE_WORDS : 0) + (m & 0xffff);
}

// The bytes of a segment on the chunk's parse, [first, end) of SW_RANGE, as literals and matches:
// its own parse's symbols from `first` on, then its continuation's.  lit(byte) for a literal (the
// chunk's bytes at `in`, LDS, read four at a time), mat(length, distance) for a match; `own` /
// `cont` its parts' match words.
template <class Lit, class Mat>
__device__ __attribute__((always_inline)) inline void walk_segment(const uint8_t* in, uint32_t range, uint32_t ownw,
                                                                    const uint32_t* __restrict__ own, int nown,
                                                                    const uint32_t* __restrict__ cont, int ncont,
                                                                    Lit lit, Mat mat) {
  auto lits = [&](int a, int e) __attribute__((always_inline)) {
    for (; a < e; a += 4) {
      const uint32_t v = ld4(in, a);
      lit(v & 255u);
      if (a + 1 < e) lit((v >> 8) & 255u);
      if (a + 2 < e) lit((v >> 16) & 255u);
      if (a + 3 < e) lit(v >> 24);
    }
  };
  const int first = (int)(range & 0xffff), end = (int)(range >> 16);
  const int eo = (int)(ownw >> 16);
  int pos = (int)(ownw & 0xffff);
  for (int k = 0; k < nown; k++) {
    const uint32_t w = own[k];
    const int ms = pos + mw_gap(w), ml = mw_len(w);
    if (ms >= first) {  // (a match before `first` ends at or before it: a boundary)
      lits(max(pos, first), ms);
      mat(ml, mw_dist(w));
    }
    pos = ms + ml;
  }
  lits(max(pos, first), eo);
  pos = eo;
  for (int k = 0; k < ncont; k++) {
    const uint32_t w = cont[k];
    const int ms = pos + mw_gap(w);
    lits(pos, ms);
    mat(mw_len(w), mw_dist(w));
    pos = ms + mw_len(w);
  }
  lits(pos, end);
}

#define DTS()                                                                      \
  do {                                                                             \
    if (tim && threadIdx.x == 0 && ti < 8) tm[ti++] = __builtin_amdgcn_s_memtime(); \
  } while (0)

__global__ __launch_bounds__(PWG) void bgzf_parse_kernel(const uint8_t* __restrict__ src,
                                                         int64_t n_in, int64_t blk0, int64_t nblk,
                                                         uint32_t* __restrict__ stage,
                                                         uint32_t* __restrict__ meta,
                                                         uint64_t* __restrict__ tim, int chain,
                                                         int lazy, int nice, int good, int fmerge) {
  __shared__ PLds L;
  uint64_t tm[8];
  int ti = 0;
  DTS();
  const int64_t b = (int64_t)blockIdx.x / NCH;  // block within this launch
  if (b >= nblk) return;
  const int c = (int)(blockIdx.x % NCH);
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t base = (blk0 + b) * (int64_t)BLK_U;
  const int n = (int)min<int64_t>(BLK_U, n_in - base);
  const int cs = c * CH;
  // this chunk's segment words: sw[k * NCH * MSEG + i] = word k of segment i
  uint32_t* sw = meta + b * META_WORDS + c * MSEG;
  int32_t* ci = reinterpret_cast<int32_t*>(meta + b * META_WORDS + CI_OFF + c * CI_WORDS);
  if (cs >= n) {  // an empty chunk (the last block is short)
    for (int i = t; i < MSEG; i += PWG) sw[SW_RANGE * NCH * MSEG + i] = SW_NONE;
    for (int i = t; i < CI_WORDS; i += PWG) ci[i] = 0;
    if (tim && t == 0)
      for (int k = 0; k < 8; k++) tim[blockIdx.x * 8 + k] = 0;
    return;
  }
  const int ce = min(n, cs + CH);
  const int r0 = max(0, cs - XW);
  const int np = ce - r0;       // bytes held: local positions [0, np)
  const int xs = cs - r0;       // the chunk's first local position
  const int npos = max(0, np - 3);  // positions with a 4-byte suffix
  const int nlc = (np - xs + PSEG - 1) / PSEG;  // segments holding bytes
  // ---- load (16-byte loads where aligned)
  for (int i = t; i < (1 << HBITS); i += PWG) L.head[i] = 0;
  for (int i = t; i < (SCAT_WAVES - 1) << (HBITS - 1); i += PWG) (&L.cnt[0][0])[i] = 0;
  if (t < 8) L.misc[t] = 0;
  // (the histogram words hold the CRC table until the bucket lists are built)
  for (int i = t; i < CI_CRC; i += PWG) L.hist[i] = i < 256 ? (int32_t)c_dcrc[i] : 0;
  {
    const uint8_t* s = src + base + r0;
    const int head = (int)((16 - (reinterpret_cast<uintptr_t>(s) & 15)) & 15);
    const int h = min(head, np);
    for (int i = t; i < h; i += PWG) L.in[i] = s[i];
    const int nv = (np - h) / 16;
    for (int i = t; i < nv; i += PWG) {
      const uint4 v = *reinterpret_cast<const uint4*>(s + h + 16 * i);
      uint8_t* d = L.in + h + 16 * i;
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 16; k++) d[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
    }
    for (int i = h + 16 * nv + t; i < np; i += PWG) L.in[i] = s[i];
    if (t < 16) L.in[np + t] = 0;  // the 4-byte compares read up to 3 bytes past the end
  }
  __syncthreads();
  DTS();
  // ---- hash buckets of every position with a 4-byte suffix.  Counts per bucket, and per bucket
  //      for each of the first three of four position ranges; bucket starts by a scan; each
  //      range's cursors = start + the earlier ranges' counts.  Then four waves scatter their
  //      ranges in order (the lanes of a 64-position step with equal hashes ranked by one ballot
  //      per hash bit, the group's last lane advancing the cursor): ascending inside each bucket,
  //      no barrier, no position hashed twice.
  const int rng = ((npos + SCAT_WAVES - 1) / SCAT_WAVES + 63) & ~63;  // positions per range
  for (int x = t; x < npos; x += PWG) {
    const uint32_t h = hash4a(L.in, x);
    atomicAdd(&L.head[h], 1);
    const int r = x / rng;
    if (r < SCAT_WAVES - 1) atomicAdd(&L.cnt[r][h >> 1], 1u << (16 * (h & 1)));
  }
  __syncthreads();
  DTS();
  {  // exclusive scan of the 2048 counts: 4 per thread
    constexpr int PER = (1 << HBITS) / PWG;
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
    if (lane == 63) L.wred[wv] = (uint32_t)inc;
    __syncthreads();
    int off = inc - sum;
    for (int w = 0; w < wv; w++) off += (int)L.wred[w];
    uint16_t* const c16 = reinterpret_cast<uint16_t*>(&L.cnt[0][0]);
#pragma unroll
    for (int k = 0; k < PER; k++) {
      const int h = PER * t + k;
      L.head[h] = off;  // range 0's cursor
      int c = off;
#pragma unroll
      for (int r = 0; r < SCAT_WAVES - 1; r++) {  // range r + 1's cursor, over range r's count
        c += c16[(r << HBITS) + h];
        c16[(r << HBITS) + h] = (uint16_t)c;
      }
      off += v[k];
    }
  }
  __syncthreads();
  DTS();
  if (wv < SCAT_WAVES) {
    const int xe = min(npos, (wv + 1) * rng);
#if DQ_SCAT_ATOMIC
    // one LDS atomic per position: the lanes of one ds_add_rtn that hit the same cursor get its
    // values in lane order on gfx950 (tools/micro/lds_atomic_order.hip: no violation in 168 M
    // atomics), so equal-hash positions of a step get ascending slots, as the ballot ranking below
    // gave them (round 4: 11 ballots per 64 positions).  Whatever the order, a candidate at or
    // past the position it is searched for is never taken (Finder::batch), so the output stays a
    // valid DEFLATE stream; its bytes are the same on every run, and equal to the ballot build's
    // (DQ_SCAT_ATOMIC=0, `make ballot`; test_atomic_scatter_equals_ballot_build), while the order
    // holds.
    uint32_t* const cur32 = wv ? reinterpret_cast<uint32_t*>(&L.cnt[wv - 1][0]) : nullptr;
    for (int x = wv * rng + lane; x < xe; x += 64) {
      const uint32_t h = hash4a(L.in, x);
      int rank;
      if (wv) {
        const uint32_t sh = 16u * (h & 1u);
        rank = (int)((atomicAdd(cur32 + (h >> 1), 1u << sh) >> sh) & 0xffffu);
      } else {
        rank = atomicAdd(&L.head[h], 1);
      }
      DQ_CHK(rank < npos, CHK_Z_BL);
      L.bl[rank] = (uint16_t)x;
    }
#else
    uint16_t* const cur16 = wv ? reinterpret_cast<uint16_t*>(&L.cnt[wv - 1][0]) : nullptr;
    for (int x0 = wv * rng; x0 < xe; x0 += 64) {
      const int x = x0 + lane;
      const bool valid = x < xe;
      const uint32_t h = valid ? hash4a(L.in, x) : 0u;
      uint64_t m = __ballot(valid);
#pragma unroll
      for (int k = 0; k < HBITS; k++) {
        const bool bit = (h >> k) & 1u;
        const uint64_t bk = __ballot(bit);
        m &= bit ? bk : ~bk;
      }
      if (valid) {
        const int cur = wv ? (int)cur16[h] : L.head[h];
        const int rank = cur + __popcll(m & lanes_below(lane));
        if (lane == 63 || !(m >> (lane + 1))) {  // the group's last lane
          if (wv) cur16[h] = (uint16_t)(rank + 1);
          else L.head[h] = rank + 1;
        }
        DQ_CHK(rank < npos, CHK_Z_BL);
        L.bl[rank] = (uint16_t)x;
      }
    }
#endif
  } else {
    // meanwhile the other waves: CRC32 of CRC_BYTES bytes per thread (raw register, init 0),
    // moved to the chunk end, XOR-ed
    const uint32_t* crc_t = reinterpret_cast<const uint32_t*>(L.hist);
    const int c0 = min(np, xs + CRC_BYTES * (t - 64 * SCAT_WAVES)), c1 = min(np, c0 + CRC_BYTES);
    uint32_t cr = 0;
    for (int i = c0; i < c1; i++) cr = crc_t[(cr ^ L.in[i]) & 0xff] ^ (cr >> 8);
    if (c1 > c0) cr = gf2_mul(x8n((uint32_t)(np - c1)), cr);
    for (int o = 32; o >= 1; o >>= 1) cr ^= __shfl_xor(cr, o, 64);
    if (lane == 0) L.wred[PWG / 64 + wv - SCAT_WAVES] = cr;
  }
  __syncthreads();
  {  // bucket ends: the last range's cursors
    const uint16_t* const c16 = reinterpret_cast<const uint16_t*>(&L.cnt[SCAT_WAVES - 2][0]);
    for (int h = t; h < (1 << HBITS); h += PWG) L.head[h] = c16[h];
  }
  for (int i = t; i < CI_CRC; i += PWG) L.hist[i] = 0;  // (the CRC table is dead)
  __syncthreads();
  DTS();
  // ---- speculative parses: thread j parses segment j (32 bytes) from its start to the first
  //      symbol boundary at or past its end (a match may run on past it).  Where a segment's parse
  //      starts never depends on another lane's progress, so the output is the same on every run.
  uint32_t* const dense = stage + (b * NCH + c) * STAGE_CH_WORDS;
  uint32_t* const pool = dense + DENSE_WORDS;
  const Finder F{L, np, min(chain, MAXCAND), nice, good};
  {
    const int j = t < nlc ? t : nlc;
    const int s0 = xs + PSEG * j, s1 = min(np, s0 + PSEG);
    int pe = s0;
    uint32_t st = 0;  // symbol starts in the segment (a deferred literal past its end: left out)
    MBuf mb{pool, &L.misc[3], &L.misc[7], OWN_CAP, 0};
    mb.n = 0;
    const int own_lazy = lazy, own_end = np;
    parse_lanes(
        F, own_lazy, own_end, s0,
        [&](int l, int d, int p) __attribute__((always_inline)) {
          if (p - s0 < PSEG) st |= 1u << (p - s0);
          if (l) {
            DQ_CHK(mb.n < OWN_CAP && p - pe < 512, CHK_Z_STAGE);
            mb.put(mword(p - pe, l, d));
            pe = p + l;
          }
        },
        [&](int x) __attribute__((always_inline)) -> int {
          if (j >= nlc) return NX_STOP;
          if (x < s1) return x;
          // segment j is parsed: publish it
          sw[SW_OWNM * NCH * MSEG + j] = mb.publish(dense, &L.misc[2]);
          sw[SW_OWN * NCH * MSEG + j] = (uint32_t)s0 | (uint32_t)x << 16;
          L.seg_exit[j] = (uint32_t)x;
          L.sbits[j] = st;
          return NX_STOP;
        });
  }
  __threadfence_block();
  __syncthreads();
  DTS();
  // ---- continuations, handed out the same way: from its exit, segment j's parse goes on until it
  //      reaches a symbol boundary of a later segment's speculative parse (the same position
  //      continues identically), skipping segments whose whole parse it overruns
  {
    int j = t < nlc ? t : nlc;
    int u = 0, pm = 0, nc = 0, pe = 0;  // merge segment, merge position, symbols, last match end
    int fpu = -1, c_lazy = lazy, c_end = np;  // forced merge: the boundary its greedy steps end on
    bool over = false;
    MBuf mb{pool, &L.misc[3], &L.misc[7], CONT_CAP, 0};
    // the merge test at E: NX_STOP (merged, the chunk's end, overflowed) or E (parse a step)
    auto check = [&](int E) __attribute__((always_inline)) -> int {
      if (fpu >= 0) {  // a forced merge's greedy steps, cut to end exactly on fpu
        DQ_CHK(E <= fpu, CHK_Z_STAGE);
        if (E >= fpu) {
          pm = fpu - (xs + PSEG * u);
          return NX_STOP;
        }
        if (nc >= CONT_WORDS) {  // (a gap of literals longer than the staging: stored)
          over = true;
          return NX_STOP;
        }
        return E;
      }
      for (;;) {
        if (E >= np) {  // the chunk's end
          u = MSEG;
          return NX_STOP;
        }
        if (u >= nlc) {  // no later segment holds symbols: parse on to the chunk end
          if (nc > CONT_WORDS - 40) {
            over = true;
            return NX_STOP;
          }
          return E;
        }
        // segment u's symbol starts ([su, su + 32)) and its exit; E >= su
        const int su = xs + PSEG * u, eu = (int)L.seg_exit[u];
        if (E > eu) {  // segment u's whole parse lies before E
          u++;
          continue;
        }
        const uint32_t ub = L.sbits[u];
        if (E == eu || (E < su + PSEG && ((ub >> (E - su)) & 1))) {  // merged: u's symbols from E on
          pm = E - su;
          return NX_STOP;
        }
        if (nc > fmerge) {  // (a step appends at most lazy + 1 <= 33 symbols: fmerge <= CONT - 40)
          // no merge within `fmerge` symbols (e.g. one repeated byte: 258-byte matches from this
          // parse's positions never meet segment u's): end exactly on segment u's next boundary
          // pu > E, with matches cut to fit and literals for the last < 3 bytes -- a valid parse
          // that merges
          const uint32_t after = E - su + 1 < PSEG ? ub >> (E - su + 1) : 0u;
          fpu = E < su + PSEG && after ? E + 1 + (int)__builtin_ctz(after) : eu;  // > E
          c_end = fpu;  // greedy steps (no lazy look-ahead) with matches cut to end on fpu
          c_lazy = 0;
          return E;
        }
        return E;
      }
    };
    // segment j's continuation from its exit: the position of its first step, or NX_STOP when it
    // ended at once (its merge word written)
    auto start = [&]() __attribute__((always_inline)) -> int {
      u = j + 1;
      pm = 0;
      nc = 0;
      over = false;
      pe = (int)L.seg_exit[j];
      mb.n = 0;
      fpu = -1;
      c_lazy = lazy;
      c_end = np;
      return check(pe);
    };
    auto finish = [&]() __attribute__((always_inline)) {
      DQ_CHK(over || u == MSEG || pm < 512, CHK_Z_STAGE);
      sw[SW_CONTM * NCH * MSEG + j] = mb.publish(dense, &L.misc[2]);
      L.seg_mrg[j] = mrg_word(over ? MSEG : u, over || u == MSEG ? 0 : pm, over);
    };
    int x0 = NX_STOP;
    while (j < nlc) {  // the first segment with a step to parse
      x0 = start();
      if (x0 >= 0) break;
      finish();
      j = PWG + atomicAdd(&L.misc[1], 1);
    }
    parse_lanes(
        F, c_lazy, c_end, x0 >= 0 ? x0 : 0,
        [&](int l, int d, int p) __attribute__((always_inline)) {
          DQ_CHK(nc < CONT_WORDS && p - pe < 512, CHK_Z_STAGE);
          nc++;
          if (l) {
            mb.put(mword(p - pe, l, d));
            pe = p + l;
          }
        },
        [&](int x) __attribute__((always_inline)) -> int {
          if (j >= nlc) return NX_STOP;
          int r = check(x);
          while (r < 0) {  // this continuation ended: the next unclaimed segment's
            finish();
            j = PWG + atomicAdd(&L.misc[1], 1);
            if (j >= nlc) return NX_STOP;
            r = start();
          }
          return r;
        });
  }
  __threadfence_block();  // staged words are read below by other threads than their writers
  if (tim) __syncthreads();  // (timing: the continuation stamp after every wave's)
  DTS();
  // ---- the chunk's parse: segment 0, then the segment each continuation merged into.  Pointer
  //      jumping: after round r every segment within 2^(r+1) - 1 merges of segment 0 is marked.
  __syncthreads();
  uint32_t* const jmp = L.seg_exit;  // the exits are dead
  for (int i = t; i < nlc; i += PWG) {
    L.seg_mark[i] = i == 0;
    jmp[i] = (uint32_t)mrg_lane(L.seg_mrg[i]);
  }
  __syncthreads();
  for (int r = 0; (1 << r) < nlc; r++) {
    uint32_t jj[NQ];
#pragma unroll
    for (int q = 0; q < NQ; q++) {
      const int i = t + q * PWG;
      const uint32_t g = i < nlc ? jmp[i] : (uint32_t)MSEG;
      if (g < (uint32_t)MSEG && L.seg_mark[i]) L.seg_mark[g] = 1;
      jj[q] = g < (uint32_t)MSEG ? jmp[g] : (uint32_t)MSEG;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NQ; q++)
      if (t + q * PWG < nlc) jmp[t + q * PWG] = jj[q];
    __syncthreads();
  }
  // the first position of each segment on the parse: set by the segment that merged into it
  bool rch[NQ];
  uint32_t mw[NQ];
#pragma unroll
  for (int q = 0; q < NQ; q++) {
    const int i = t + q * PWG;
    rch[q] = i < nlc && L.seg_mark[i];
    mw[q] = i < nlc ? L.seg_mrg[i] : 0u;
  }
  __syncthreads();
  if (t == 0) jmp[0] = (uint32_t)xs;
#pragma unroll
  for (int q = 0; q < NQ; q++) {
    const int g = mrg_lane(mw[q]);
    if (rch[q] && g < MSEG) jmp[g] = (uint32_t)(xs + PSEG * g + mrg_off(mw[q]));
    if (rch[q] && mrg_over(mw[q])) L.misc[7] = 1;
  }
  __syncthreads();
  // each segment's range on the parse, and the histograms of the parse's symbols: its literals'
  // bytes and its matches, walked as the code kernel walks them
#pragma unroll
  for (int q = 0; q < NQ; q++) {
    const int i = t + q * PWG;
    if (i >= MSEG) continue;
    if (!rch[q]) {
      sw[SW_RANGE * NCH * MSEG + i] = SW_NONE;
      continue;
    }
    const int g = mrg_lane(mw[q]);
    const int end = g < MSEG ? xs + PSEG * g + mrg_off(mw[q]) : np;
    const uint32_t range = jmp[i] | (uint32_t)end << 16;
    sw[SW_RANGE * NCH * MSEG + i] = range;
    const uint32_t ow = sw[SW_OWN * NCH * MSEG + i], om = sw[SW_OWNM * NCH * MSEG + i],
                   cm = sw[SW_CONTM * NCH * MSEG + i];
    const uint32_t* own = part_words(dense, om);
    const uint32_t* cont = part_words(dense, cm);
    walk_segment(
        L.in, range, ow, own, (int)((om >> 16) & 255), cont, (int)((cm >> 16) & 255),
        [&](uint32_t by) __attribute__((always_inline)) { atomicAdd(&L.hist[CI_LL + by], 1); },
        [&](int ml, int md) __attribute__((always_inline)) {
          int sy, nx, xv;
          len_code(ml, sy, nx, xv);
          atomicAdd(&L.hist[CI_LL + sy], 1);
          dist_code(md, sy, nx, xv);
          atomicAdd(&L.hist[CI_D + sy], 1);
        });
  }
  __syncthreads();
  for (int i = t; i < CI_CRC; i += PWG) ci[i] = L.hist[i];
  if (t == 0) {
    uint32_t cr = 0;
    for (int w = 0; w < PWG / 64 - SCAT_WAVES; w++) cr ^= L.wred[PWG / 64 + w];
    ci[CI_CRC] = (int32_t)cr;
    ci[CI_OVER] = L.misc[7];
    ci[CI_BYTES] = ce - cs;
  }
  DTS();
  if (tim && t == 0)
    for (int k = 0; k < 8; k++) tim[blockIdx.x * 8 + k] = k < ti ? tm[k] - tm[0] : 0;
}

struct alignas(16) CLds {
  uint8_t src[BLK_U + 16];  // the block's bytes (the literals)
  uint8_t img[65536];       // the deflate image (<= 65510 bytes)
  int32_t head[H_END];      // histograms and code tables (H_* offsets)
  uint32_t wsum[3 * (CWG / 64)];
  int32_t misc[8];
};

static_assert(OWN_CAP % 4 == 0 && CONT_CAP % 4 == 0 && CONT_CAP >= CONT_WORDS && STAGE_CH_WORDS % 4 == 0 &&
                  DENSE_WORDS % 4 == 0 && POOL_WORDS <= 65536,
              "16-byte aligned overflow areas");

// Huffman codes of one block per 128-thread workgroup (7.9 KB of LDS, many per CU, so the
// latency-bound serial parts -- the Moffat-Katajainen pass, the run-length coding -- of many blocks
// overlap): the two chunks' histograms summed, wave 0 the literal/length code and wave 1 the
// distance code, the code-length code; the tables and header tokens go to the block's record for
// bgzf_code_kernel.
constexpr int HWG = 128;
struct alignas(16) HLds {
  int32_t head[H_END];
  int32_t misc[8];
};
__global__ __launch_bounds__(HWG) void bgzf_huff_kernel(int64_t n_in, int64_t blk0, int64_t nblk,
                                                        uint32_t* __restrict__ meta,
                                                        uint64_t* __restrict__ tim) {
  __shared__ HLds L;
  uint64_t tm[8];
  int ti = 0;
  DTS();
  const int64_t b = (int64_t)blockIdx.x;
  if (b >= nblk) return;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t base = (blk0 + b) * (int64_t)BLK_U;
  const int n = (int)min<int64_t>(BLK_U, n_in - base);
  const int32_t* ci = reinterpret_cast<const int32_t*>(meta + b * META_WORDS + CI_OFF);
  uint32_t* tb = meta + b * META_WORDS + TB_OFF;
  int32_t* H = L.head;
  for (int i = t; i < H_CL + 32; i += HWG) H[i] = 0;
  __syncthreads();
  for (int s = t; s < CI_CRC; s += HWG) {
    int v = 0;
#pragma unroll
    for (int c = 0; c < NCH; c++) v += ci[c * CI_WORDS + s];
    H[s < CI_D ? H_LL + s : H_D + (s - CI_D)] = v;
  }
  __syncthreads();
  if (t == 0) {
    H[H_LL + 256] += 1;  // end of block
  }
  __syncthreads();
  DTS();
  // ---- dynamic Huffman codes: wave 0 the literal/length alphabet, wave 1 the distances
  if (wv == 0) build_lengths(H + H_LL, 286, 15, H + H_SORT, H + H_W, H + H_LEN, H + H_CNT, lane);
  if (wv == 1) {
    build_lengths(H + H_D, 30, 15, H + H_SORT_D, H + H_W_D, H + H_LEN_D, H + H_CNT_D, lane);
    if (lane == 0) {  // the member's CRC (while wave 0 builds the longer code)
      int over = 0;
      uint32_t cr = 0;
      for (int c = 0; c < NCH; c++) {  // raw(A B) = raw(A) x^(8 |B|) + raw(B)
        over |= ci[c * CI_WORDS + CI_OVER];
        cr = gf2_mul(x8n((uint32_t)ci[c * CI_WORDS + CI_BYTES]), cr) ^ (uint32_t)ci[c * CI_WORDS + CI_CRC];
      }
      L.misc[1] = (int32_t)(cr ^ gf2_mul(x8n((uint32_t)n), 0xffffffffu) ^ 0xffffffffu);
      L.misc[7] = over;
    }
  }
  __syncthreads();
  DTS();
  // codes by waves 0 and 1; wave 1's first lane then run-length codes the code lengths
  if (wv == 0) canon_codes_wave(H + H_LEN, 286, reinterpret_cast<uint32_t*>(H + C_LL), lane);
  if (wv == 1) canon_codes_wave(H + H_LEN_D, 30, reinterpret_cast<uint32_t*>(H + C_D), lane);
  if (t == 64) {  // (wave 1, after its distance codes)
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
  DTS();
  if (wv == 0) build_lengths(H + H_CL, 19, 7, H + H_SORT, H + H_W, H + H_LEN_CL, H + H_CNT, lane);
  __syncthreads();
  if (wv == 0) {
    canon_codes_wave(H + H_LEN_CL, 19, reinterpret_cast<uint32_t*>(H + C_CL), lane);
    int ncl = 19;
    while (ncl > 4 && H[H_LEN_CL + c_clord[ncl - 1]] == 0) ncl--;
    // dynamic header bits: the tokens' code lengths and extra bits, summed over the wave
    const uint16_t* tok = reinterpret_cast<const uint16_t*>(H + H_TOK);
    uint32_t hb = 0;
    for (int k = lane; k < L.misc[4]; k += 64) {
      const int sy = tok[k] & 31;
      hb += (uint32_t)H[H_LEN_CL + sy] + (sy == 16 ? 2 : sy == 17 ? 3 : sy == 18 ? 7 : 0);
    }
    for (int o = 32; o >= 1; o >>= 1) hb += __shfl_xor(hb, o, 64);
    if (lane == 0) {
      L.misc[5] = ncl;
      L.misc[6] = (int32_t)(hb + 3 + 5 + 5 + 4 + 3 * (uint32_t)ncl);
    }
  }
  __syncthreads();
  DTS();
  // the record
  for (int i = t; i < 286; i += HWG) tb[TB_LL + i] = (uint32_t)H[C_LL + i];
  for (int i = t; i < 30; i += HWG) tb[TB_D + i] = (uint32_t)H[C_D + i];
  for (int i = t; i < 19; i += HWG) {
    tb[TB_CL + i] = (uint32_t)H[C_CL + i];
    tb[TB_LENCL + i] = (uint32_t)H[H_LEN_CL + i];
  }
  for (int i = t; i < TB_MISC - TB_TOK; i += HWG) tb[TB_TOK + i] = (uint32_t)H[H_TOK + i];
  if (t < 8) tb[TB_MISC + t] = (uint32_t)L.misc[t];
  if (tim && t == 0)
    for (int k = 0; k < 8; k++) tim[b * 8 + k] = k < ti ? tm[k] - tm[0] : 0;
}

__global__ __launch_bounds__(CWG) void bgzf_code_kernel(const uint8_t* __restrict__ src,
                                                        int64_t n_in, int64_t blk0, int64_t nblk,
                                                        const uint32_t* __restrict__ stage,
                                                        const uint32_t* __restrict__ meta,
                                                        uint8_t* __restrict__ out_slots,
                                                        int32_t* __restrict__ out_size,
                                                        uint64_t* __restrict__ tim) {
  __shared__ CLds L;
  uint64_t tm[8];
  int ti = 0;
  DTS();
  const int64_t b = (int64_t)blockIdx.x;
  if (b >= nblk) return;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t base = (blk0 + b) * (int64_t)BLK_U;
  const int n = (int)min<int64_t>(BLK_U, n_in - base);
  const uint32_t* swb = meta + b * META_WORDS;
  int32_t* H = L.head;
  // the block's code tables from bgzf_huff_kernel
  const uint32_t* tb = meta + b * META_WORDS + TB_OFF;
  for (int i = t; i < 286; i += CWG) H[C_LL + i] = (int32_t)tb[TB_LL + i];
  for (int i = t; i < 30; i += CWG) H[C_D + i] = (int32_t)tb[TB_D + i];
  for (int i = t; i < 19; i += CWG) {
    H[C_CL + i] = (int32_t)tb[TB_CL + i];
    H[H_LEN_CL + i] = (int32_t)tb[TB_LENCL + i];
  }
  for (int i = t; i < TB_MISC - TB_TOK; i += CWG) H[H_TOK + i] = (int32_t)tb[TB_TOK + i];
  if (t < 8) L.misc[t] = (int32_t)tb[TB_MISC + t];
  {  // the block's bytes (16-byte loads where aligned)
    const uint8_t* sb = src + base;
    const int h = min(n, (int)((16 - (reinterpret_cast<uintptr_t>(sb) & 15)) & 15));
    for (int i = t; i < h; i += CWG) L.src[i] = sb[i];
    const int nv = (n - h) / 16;
    if (h == 0) {  // (the usual case: the stream 16-byte aligned)
      for (int i = t; i < nv; i += CWG)
        reinterpret_cast<uint4*>(L.src)[i] = *reinterpret_cast<const uint4*>(sb + 16 * i);
    } else {
      for (int i = t; i < nv; i += CWG) {
        const uint4 v = *reinterpret_cast<const uint4*>(sb + h + 16 * i);
        uint8_t* d = L.src + h + 16 * i;
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 16; k++) d[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
      }
    }
    for (int i = h + 16 * nv + t; i < n; i += CWG) L.src[i] = sb[i];
  }
  __syncthreads();
  const bool over = L.misc[7] != 0;
  DTS();
  // ---- bits of this thread's two segments (CSEG) under the dynamic and the fixed code
  // segment j of this thread's eight (the block's segment 8t + j) on the parse: walked with
  // lit(byte) and mat(length, distance)
  auto each_seg = [&](auto lit, auto mat) __attribute__((always_inline)) {
    for (int j = 0; j < CSEG; j++) {
      const int g = CSEG * t + j, c = g / PL, u = g - c * PL;
      if (g >= NLANE) break;
      const uint32_t* w = swb + c * MSEG + u;
      const uint32_t rg = w[SW_RANGE * NCH * MSEG];
      if (rg == SW_NONE) continue;
      const uint32_t ow = w[SW_OWN * NCH * MSEG], om = w[SW_OWNM * NCH * MSEG], cm = w[SW_CONTM * NCH * MSEG];
      const uint32_t* dense = stage + (b * NCH + c) * STAGE_CH_WORDS;
      const uint8_t* cb = L.src + max(0, c * CH - XW);  // the chunk's position 0
      walk_segment(cb, rg, ow, part_words(dense, om), (int)((om >> 16) & 255),
                   part_words(dense, cm), (int)((cm >> 16) & 255), lit, mat);
    }
  };
  const bool has_eob = CSEG * t + CSEG - 1 == NLANE - 1;  // the block's last segment ends with EOB
  uint32_t vd = 0, vf = 0;
  {
    const uint32_t* cll = reinterpret_cast<const uint32_t*>(H + C_LL);
    const uint32_t* cd = reinterpret_cast<const uint32_t*>(H + C_D);
    each_seg(
        [&](uint32_t by) __attribute__((always_inline)) {
          vd += cll[by] >> 16;
          vf += by < 144 ? 8 : 9;
        },
        [&](int ml, int md) __attribute__((always_inline)) {
          int sy, nx, xv, ds, dnx, dxv;
          len_code(ml, sy, nx, xv);
          dist_code(md, ds, dnx, dxv);
          vd += (cll[sy] >> 16) + (cd[ds] >> 16) + (uint32_t)(nx + dnx);
          vf += (uint32_t)(fixed_len_of(sy) + nx + 5 + dnx);
        });
    if (has_eob) {
      vd += cll[256] >> 16;
      vf += 7;
    }
  }
  // ---- choose dynamic or fixed; exclusive scan of the threads' chosen bit counts
  uint32_t dsum = vd, fsum = vf;
  for (int o = 32; o >= 1; o >>= 1) {
    dsum += __shfl_xor(dsum, o, 64);
    fsum += __shfl_xor(fsum, o, 64);
  }
  constexpr int NW = CWG / 64;
  if (lane == 0) {
    L.wsum[wv] = dsum;
    L.wsum[NW + wv] = fsum;
  }
  __syncthreads();
  dsum = 0;
  fsum = 0;
#pragma unroll
  for (int w = 0; w < NW; w++) {
    dsum += L.wsum[w];
    fsum += L.wsum[NW + w];
  }
  const bool dyn = (uint32_t)L.misc[6] + dsum < 3u + fsum;
  const uint32_t hdr_bits = dyn ? (uint32_t)L.misc[6] : 3u;
  const uint32_t sm = dyn ? vd : vf;
  uint32_t inc = sm;
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(inc, d, 64);
    if (lane >= d) inc += y;
  }
  if (lane == 63) L.wsum[2 * NW + wv] = inc;
  __syncthreads();
  uint32_t off = hdr_bits + inc - sm, total_bits = hdr_bits;
#pragma unroll
  for (int w = 0; w < NW; w++) {
    off += w < wv ? L.wsum[2 * NW + w] : 0u;
    total_bits += L.wsum[2 * NW + w];
  }
  DTS();
  if (!dyn) {  // the fixed code into the code tables
    uint32_t* cll = reinterpret_cast<uint32_t*>(H + C_LL);
    uint32_t* cd = reinterpret_cast<uint32_t*>(H + C_D);
    for (int sy = t; sy < 286; sy += CWG) {
      uint32_t code;
      int cl;
      fixed_ll(sy, code, cl);
      cll[sy] = code | ((uint32_t)cl << 16);
    }
    if (t < 30) cd[t] = rev((uint32_t)t, 5) | (5u << 16);
  }
  const int dbytes = (int)((total_bits + 7) / 8);
  uint8_t* o = out_slots + b * (int64_t)SLOT;
  const uint32_t crc = (uint32_t)L.misc[1];
  // stored when the code is no shorter than the bytes themselves (and always when it would not fit)
  const bool stored = over || dbytes > min(MAX_DEFLATE, n + 5);
  int payload;
  if (!stored) {
    // ---- the header, then every thread's segments, OR-ed into the LDS image; then the image
    //      to the slot in 16-byte stores (the payload is 16-byte aligned there)
    uint32_t* img = reinterpret_cast<uint32_t*>(L.img);
    const int nw = (int)(total_bits >> 5) + 1;
    for (int i = t; i < nw; i += CWG) img[i] = 0;
    __syncthreads();
    // the header, by wave 0 in parallel: item 0 the 17 bits of BFINAL, BTYPE, HLIT, HDIST, HCLEN,
    // then the HCLEN code-length code lengths, then the run-length tokens (code + extra bits), each
    // lane one item: offsets by a wave scan of the items' bit lengths, bits OR-ed into the zeroed
    // image (round 4: thread 0 put them one by one while its wave waited, ~300 dependent steps)
    if (wv == 0) {
      if (!dyn) {
        if (lane == 0) atomicOr(&img[0], 3u);  // BFINAL 1, BTYPE 01
      } else {
        const int ncl = L.misc[5], ntok = L.misc[4];
        const int nitem = 1 + ncl + ntok;
        const uint16_t* tok = reinterpret_cast<const uint16_t*>(H + H_TOK);
        const uint32_t* ccl = reinterpret_cast<const uint32_t*>(H + C_CL);
        uint32_t base = 0;
        for (int i0 = 0; i0 < nitem; i0 += 64) {
          const int i = i0 + lane;
          uint32_t v = 0;
          int len = 0;
          if (i == 0) {
            v = 5u | (uint32_t)(L.misc[2] - 257) << 3 | (uint32_t)(L.misc[3] - 1) << 8 |
                (uint32_t)(ncl - 4) << 13;
            len = 17;
          } else if (i <= ncl) {
            v = (uint32_t)H[H_LEN_CL + c_clord[i - 1]];
            len = 3;
          } else if (i < nitem) {
            const int k = i - 1 - ncl;
            const int sy = tok[k] & 31, ex = tok[k] >> 5;
            const int cl = (int)(ccl[sy] >> 16);
            const int xl = sy == 16 ? 2 : sy == 17 ? 3 : sy == 18 ? 7 : 0;
            v = (ccl[sy] & 0xffffu) | (uint32_t)ex << cl;
            len = cl + xl;
          }
          int inc = len;
          for (int d = 1; d < 64; d <<= 1) {
            const int y = __shfl_up(inc, d, 64);
            if (lane >= d) inc += y;
          }
          const uint32_t pos = base + (uint32_t)(inc - len);
          if (len) {
            const uint64_t bits = (uint64_t)v << (pos & 31);
            DQ_CHK((pos >> 5) + 1 < 65536 / 4, CHK_Z_IMAGE);
            atomicOr(&img[pos >> 5], (uint32_t)bits);
            if ((pos & 31) + (uint32_t)len > 32) atomicOr(&img[(pos >> 5) + 1], (uint32_t)(bits >> 32));
          }
          base += (uint32_t)__shfl(inc, 63, 64);
        }
      }
    }
    {
      const uint32_t* cll = reinterpret_cast<const uint32_t*>(H + C_LL);
      const uint32_t* cd = reinterpret_cast<const uint32_t*>(H + C_D);
      ImgOut io(img, off);
      each_seg(
          [&](uint32_t by) __attribute__((always_inline)) {
            const uint32_t e = cll[by];
            io.put(e & 0xffff, (int)(e >> 16));
          },
          [&](int ml, int md) __attribute__((always_inline)) {
            int sy, nx, xv, ds, dnx, dxv;
            len_code(ml, sy, nx, xv);
            dist_code(md, ds, dnx, dxv);
            io.put(cll[sy] & 0xffff, (int)(cll[sy] >> 16));
            if (nx) io.put((uint32_t)xv, nx);
            io.put(cd[ds] & 0xffff, (int)(cd[ds] >> 16));
            if (dnx) io.put((uint32_t)dxv, dnx);
          });
      if (has_eob) io.put(cll[256] & 0xffff, (int)(cll[256] >> 16));
      io.flush();
    }
    __syncthreads();
    DTS();
    payload = dbytes;
    const uint4* si = reinterpret_cast<const uint4*>(L.img);
    uint4* di = reinterpret_cast<uint4*>(o + SLOT_PAY);
    for (int i = t; i < (payload + 15) / 16; i += CWG) di[i] = si[i];
    __syncthreads();  // (the trailer over the last store's padding)
  } else {
    // stored block: BFINAL 1, BTYPE 00, LEN, NLEN, the bytes
    payload = n + 5;
    uint8_t* pb = o + SLOT_PAY;
    if (t == 0) {
      pb[0] = 1;
      pb[1] = (uint8_t)n;
      pb[2] = (uint8_t)(n >> 8);
      pb[3] = (uint8_t)~n;
      pb[4] = (uint8_t)(~n >> 8);
    }
    for (int i = t; i < n; i += CWG) pb[5 + i] = L.src[i];
  }
  if (t == 0) {
    const int bsize = 18 + payload + 8 - 1;
    uint8_t* hd = o + SLOT_HDR;
    hd[0] = 0x1f; hd[1] = 0x8b; hd[2] = 8; hd[3] = 4;
    hd[4] = 0; hd[5] = 0; hd[6] = 0; hd[7] = 0; hd[8] = 0; hd[9] = 0xff;
    hd[10] = 6; hd[11] = 0; hd[12] = 'B'; hd[13] = 'C'; hd[14] = 2; hd[15] = 0;
    hd[16] = (uint8_t)bsize; hd[17] = (uint8_t)(bsize >> 8);
    uint8_t* tr = o + SLOT_PAY + payload;
    tr[0] = (uint8_t)crc; tr[1] = (uint8_t)(crc >> 8); tr[2] = (uint8_t)(crc >> 16); tr[3] = (uint8_t)(crc >> 24);
    tr[4] = (uint8_t)n; tr[5] = (uint8_t)(n >> 8); tr[6] = (uint8_t)(n >> 16); tr[7] = (uint8_t)(n >> 24);
    out_size[b] = bsize + 1;
  }
  DTS();
  if (tim && t == 0)
    for (int k = 0; k < 8; k++) tim[b * 8 + k] = k < ti ? tm[k] - tm[0] : 0;
}
#undef DTS

// Packs the block slots (the member from SLOT_HDR on) into one contiguous BGZF stream: one
// workgroup per block.
__global__ __launch_bounds__(256) void bgzf_pack_kernel(const uint8_t* __restrict__ slots,
                                                        const int32_t* __restrict__ size,
                                                        const int64_t* __restrict__ off, int64_t nblk,
                                                        uint8_t* __restrict__ out) {
  const int64_t b = blockIdx.x;
  if (b >= nblk) return;
  const uint8_t* s = slots + b * (int64_t)SLOT + SLOT_HDR;
  uint8_t* d = out + off[b];
  const int n = size[b];
  for (int i = threadIdx.x; i < n; i += 256) d[i] = s[i];
}

// The blocks' offsets in the packed stream: an exclusive scan of their sizes on top of the running
// total at off[nblk] (one workgroup; the batch's total is added to it), so the batches need no host
// round trip.
__global__ __launch_bounds__(1024) void bgzf_offsets_kernel(const int32_t* __restrict__ size,
                                                            int64_t nblk, int64_t* __restrict__ off,
                                                            int64_t* __restrict__ total) {
  __shared__ int64_t wsum[16];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  int64_t carry = *total;
  for (int64_t b0 = 0; b0 < nblk; b0 += 1024) {
    const int64_t i = b0 + t;
    const int64_t v = i < nblk ? size[i] : 0;
    int64_t inc = v;
    for (int d = 1; d < 64; d <<= 1) {
      const int64_t y = __shfl_up(inc, d, 64);
      if (lane >= d) inc += y;
    }
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    int64_t pre = carry, all = carry;
    for (int w = 0; w < 16; w++) {
      pre += w < wv ? wsum[w] : 0;
      all += wsum[w];
    }
    if (i < nblk) off[i] = pre + inc - v;
    carry = all;
    __syncthreads();
  }
  if (t == 0) *total = carry;
}

struct DefTables {
  std::once_flag once;
  bool ok = false;
};
DefTables g_def[64];

}  // namespace

int64_t bgzf_block_count(int64_t n) { return n <= 0 ? 0 : (n + BLK_U - 1) / BLK_U; }
size_t bgzf_stage_bytes(int64_t nblk) { return (size_t)nblk * NCH * STAGE_CH_WORDS * 4; }
size_t bgzf_meta_bytes(int64_t nblk) { return (size_t)nblk * META_WORDS * 4; }
size_t bgzf_slot_bytes(int64_t nblk) { return (size_t)nblk * SLOT; }

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
                         uint32_t* stage, uint32_t* meta, uint8_t* out_slots, int32_t* out_size,
                         uint64_t* tim, hipStream_t s) {
  if (nblk <= 0) return;
  // DQ_DEFLATE="chain,lazy,nice[,good[,fmerge]]": match-search effort (default 32,16,32,8: zlib
  // level 5's own settings; with the 4-byte bucket key that is ratio 2.92 on the WGS stream against
  // htsjdk's 2.857, profiles/r4m_deflate_sweep.txt; good 0 = always the full chain) and the
  // continuation symbols before a forced merge (default 1: ratio 2.912, 14.55 GB/s, against 2.918
  // and 14.03 at 2 -- round 4's default, 2.924 at 116; 0 gives 2.902 and takes the HiSeq part past
  // zlib level 5 + 0.5 %: profiles/r4aj_deflate_fmerge.txt, r5zc_deflate_fmerge.txt); read at
  // every launch, so a test can sweep settings in one process
  int cc = 32, cl = 16, cn = 32, cg = 8, cf = FMERGE;
  if (const char* e = getenv("DQ_DEFLATE")) sscanf(e, "%d,%d,%d,%d,%d", &cc, &cl, &cn, &cg, &cf);
  cf = std::max(0, std::min(cf, CONT_WORDS - 40));
  cc = std::max(1, std::min(cc, MAXCAND));
  cl = std::max(0, std::min(cl, 32));
  cn = std::max(3, cn);
  cg = std::max(0, cg);
  hipLaunchKernelGGL(bgzf_parse_kernel, dim3((unsigned)(nblk * NCH)), dim3(PWG), 0, s, src, n_in, blk0,
                     nblk, stage, meta, tim, cc, cl, cn, cg, cf);
  hipLaunchKernelGGL(bgzf_huff_kernel, dim3((unsigned)nblk), dim3(HWG), 0, s, n_in, blk0, nblk, meta,
                     tim ? tim + nblk * NCH * 8 : nullptr);
  hipLaunchKernelGGL(bgzf_code_kernel, dim3((unsigned)nblk), dim3(CWG), 0, s, src, n_in, blk0, nblk,
                     stage, meta, out_slots, out_size, tim ? tim + nblk * (NCH + 1) * 8 : nullptr);
}

void launch_bgzf_pack(const uint8_t* slots, const int32_t* size, int64_t* off, int64_t* total,
                      int64_t nblk, uint8_t* out, hipStream_t s) {
  if (nblk <= 0) return;
  hipLaunchKernelGGL(bgzf_offsets_kernel, dim3(1), dim3(1024), 0, s, size, nblk, off, total);
  hipLaunchKernelGGL(bgzf_pack_kernel, dim3((unsigned)nblk), dim3(256), 0, s, slots, size, off, nblk,
                     out);
}

DQ_CHK_UNIT(deflate)

}  // namespace dq
