// dq_inflate.hip -- Kernel 2: BGZF block inflate + CRC32 on gfx950, as two kernels.
//
// Replaces htsjdk BlockCompressedInputStream / BlockGunzipper.unzipBlock (htsjdk 2.16.0, reached
// from D/impl/formats/bam/BamSource.java:172-175) -> java.util.zip.Inflater.
//
// K2a huff_decode_kernel -- one BGZF block per LANE (64 blocks per wave, persistent waves pulling
//   blocks from an atomic counter).  Huffman codes are decoded canonically: the 15-bit
//   bit-reversed window is compared against the per-length limits held in VGPRs, then one LDS
//   read of the per-length base and one of the sorted symbol table (~670 B of LDS per lane, so
//   three 64-lane waves fit a CU: 192 blocks in flight).  Every iteration decodes one code for
//   every lane whatever its state (literal/length or distance), so the SIMD path is uniform.
//   Dynamic headers are decoded for several waiting lanes at once (header slots) to limit
//   divergence.  Output: a u16 token stream per block (literal | 256+len-3 | 0x8000|dist-1).
// K2b lz77_resolve_kernel -- one 512-thread workgroup per block with the whole block's output
//   (<= 64 KiB) in LDS.  Tokens are consumed in chunks of <= 512 tokens / 2 KiB of output: a
//   block prefix sum places them, an owner max-scan maps every output byte to its token, and each
//   byte follows copy sources (one hop per match, modulo the distance for overlapping copies)
//   until it reaches a literal or a byte of an earlier chunk.  The CRC32 of the block is computed
//   from LDS and compared with the gzip trailer; the bytes are stored to HBM with 16-byte stores.
//
// Output stops at ISIZE (Inflater.inflate(buf, off, ISIZE) semantics); fewer bytes is an error.
#include "dq_internal.h"

namespace dq {
namespace {

constexpr int NLANE = 64;         // blocks per wave in K2a
constexpr int HDR_SLOTS = 16;     // lanes that can decode a dynamic header at once
constexpr int ITERS = 32;         // decode iterations between scheduling decisions
constexpr int STAGE = 18;         // token staging entries per lane (flush at 16)

enum : int32_t { S_IDLE = 0, S_HDR = 1, S_LIT = 2, S_DIST = 3, S_STORED = 4, S_DONE = 5, S_EXIT = 6 };

__constant__ uint16_t c_lbase[29] = {3,  4,  5,  6,  7,  8,  9,  10,  11,  13,  15,  17,  19,  23, 27,
                                     31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t c_lext[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,
                                   2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t c_dbase[30] = {1,    2,    3,    4,    5,    7,    9,    13,    17,    25,
                                     33,   49,   65,   97,   129,  193,  257,  385,   513,   769,
                                     1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t c_dext[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3,  3,  4,  4,  5,  5,  6,
                                   6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t c_clorder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

struct LaneTab {         // canonical decode tables of one lane's current deflate block (672 B)
  uint16_t lsym[288];    // litlen symbols in canonical order
  uint8_t dsym[32];      // distance symbols in canonical order
  int16_t lbase[16];     // lbase[l] = (index of first code of length l) - (first code of length l)
  int16_t dbase[16];
};

struct HdrSlot {         // scratch of one header decode (448 B)
  uint8_t lens[320];
  uint8_t clsym[20];
  int16_t clbase[16];
  uint16_t cnt[16];
  uint16_t nxt[16];
  uint8_t pad[44];
};

struct alignas(16) LdsA {
  LaneTab tab[NLANE];
  HdrSlot slot[HDR_SLOTS];
  uint16_t stage[NLANE][STAGE + 2];
  uint16_t lbase_k[29];
  uint8_t lext_k[29];
  uint16_t dbase_k[30];
  uint8_t dext_k[30];
};

__device__ inline uint32_t rev15(uint32_t w) { return __builtin_bitreverse32(w) >> 17; }

// Canonical code construction for one lane: counts, limits (left-justified to 15 bits), bases,
// sorted symbols.  Over-subscribed or incomplete codes are rejected as zlib's inflate_table does
// (a single distance code of length 1 is allowed; its missing code then decodes as invalid).
// lim[1..15] are returned; lim[15] < 32768 marks an incomplete code.
__device__ __attribute__((always_inline)) int canon_build(const uint8_t* lens, int n, uint16_t* cnt, uint16_t* nxt, int16_t* base,
                           uint8_t* sym8, uint16_t* sym16, bool allow_single, uint32_t* lim) {
  for (int i = 0; i < 16; i++) cnt[i] = 0;
  for (int s = 0; s < n; s++) cnt[lens[s]]++;
  cnt[0] = 0;
  int left = 1, maxl = 0;
#pragma unroll
  for (int l = 1; l <= 15; l++) {
    left <<= 1;
    left -= cnt[l];
    if (left < 0) return -1;
    if (cnt[l]) maxl = l;
  }
  if (maxl == 0) {  // no codes at all
#pragma unroll
    for (int l = 1; l <= 15; l++) lim[l] = 0;  // every window >= lim[15]: invalid
    return 0;
  }
  if (left > 0 && !(allow_single && maxl == 1)) return -1;
  uint32_t code = 0, off = 0;
#pragma unroll
  for (int l = 1; l <= 15; l++) {
    base[l] = (int16_t)((int32_t)off - (int32_t)code);
    nxt[l] = (uint16_t)off;
    code += cnt[l];
    off += cnt[l];
    lim[l] = code << (15 - l);
    code <<= 1;
  }
  for (int s = 0; s < n; s++) {
    int l = lens[s];
    if (l) {
      uint16_t k = nxt[l]++;
      if (sym8) sym8[k] = (uint8_t)s;
      else sym16[k] = (uint16_t)s;
    }
  }
  return 0;
}

struct Lane {
  uint64_t bb;      // bit buffer
  uint32_t bc;      // valid bits in bb
  uint32_t pf;      // prefetched next 32 bits of input
  int64_t ip;       // byte offset in C of the word held in pf
  int64_t dstart;   // first deflate byte of the block
  int32_t dbytes;
  int32_t state;
  int32_t last;
  int32_t pend;     // pending match length (S_DIST) / stored bytes left (S_STORED)
  int32_t produced;
  int32_t isize;
  int32_t ntok;     // tokens flushed so far
  int32_t sc;       // staged tokens
  int32_t blk;
  int32_t err;
  int64_t tokbase;  // byte offset of the block's token region
};

__device__ inline uint32_t load_word(const uint8_t* C, int64_t ip) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(C + (ip & ~(int64_t)3));
  const int sh = (int)(ip & 3) * 8;
  const uint32_t lo = w[0], hi = w[1];
  return sh ? (uint32_t)((((uint64_t)hi << 32) | lo) >> sh) : lo;
}

__device__ inline void refill(Lane& s, const uint8_t* C) {
  if (s.bc < 32) {
    s.bb |= (uint64_t)s.pf << s.bc;
    s.bc += 32;
    s.ip += 4;
    s.pf = load_word(C, s.ip);
  }
}
__device__ inline uint32_t take(Lane& s, uint32_t n) {
  uint32_t v = (uint32_t)(s.bb & ((1ull << n) - 1));
  s.bb >>= n;
  s.bc -= n;
  return v;
}

__device__ inline int64_t tok_region(int64_t uoff_b, int64_t b) {
  return (2 * uoff_b + 64 * b + 15) & ~(int64_t)15;
}

__device__ inline void flush16(LdsA& L, int lane, Lane& s, uint16_t* tok) {
  // stage[0..16) -> HBM (two 16-byte stores), keep the overflow entries
  uint4* dst = reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(tok) + s.tokbase + 2 * (int64_t)s.ntok);
  uint4 a, b;
  // stage rows are 40 bytes apart: read through 32-bit words (row base is 8-byte aligned)
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&L.stage[lane][0]);
  a.x = w[0]; a.y = w[1]; a.z = w[2]; a.w = w[3];
  b.x = w[4]; b.y = w[5]; b.z = w[6]; b.w = w[7];
  dst[0] = a;
  dst[1] = b;
  s.ntok += 16;
  for (int i = 16; i < s.sc; i++) L.stage[lane][i - 16] = L.stage[lane][i];
  s.sc -= 16;
}

__device__ inline void put_tok(LdsA& L, int lane, Lane& s, uint16_t t) { L.stage[lane][s.sc++] = t; }

__device__ void start_block(Lane& s, const uint8_t* C, const int64_t* blk_pos,
                            const int32_t* blk_csize, const int32_t* blk_usize,
                            const int64_t* uoff, int64_t b) {
  s.blk = (int32_t)b;
  const int64_t pos = blk_pos[b];
  s.dstart = pos + 18;
  s.dbytes = blk_csize[b] - 26;
  s.isize = blk_usize[b];
  s.tokbase = tok_region(uoff[b], b);
  s.produced = 0;
  s.ntok = 0;
  s.sc = 0;
  s.err = 0;
  s.last = 0;
  s.pend = 0;
  s.bb = 0;
  s.bc = 0;
  s.ip = s.dstart;
  s.pf = load_word(C, s.ip);
  s.state = S_HDR;
  if (s.isize < 0 || s.isize > 65536) {
    s.err = ST_ISIZE;
    s.state = S_DONE;
  } else if (s.isize == 0) {
    s.state = S_DONE;  // Inflater asked for 0 bytes: nothing to decode
  }
}

// Decode one deflate block header for this lane (slot = scratch index).
__device__ __attribute__((always_inline)) void do_header(Lane& s, LdsA& L, int lane, int slot, const uint8_t* C, uint32_t* ll,
                          uint32_t* dl) {
  refill(s, C);
  s.last = (int32_t)take(s, 1);
  const uint32_t type = take(s, 2);
  LaneTab& T = L.tab[lane];
  if (type == 0) {
    take(s, s.bc & 7);
    refill(s, C);
    const uint32_t len = take(s, 16), nlen = take(s, 16);
    if ((len ^ 0xffffu) != nlen) {
      s.err = ST_BAD_STORED;
      return;
    }
    s.pend = (int32_t)len;
    s.state = len ? S_STORED : (s.last ? S_DONE : S_HDR);
    return;
  }
  HdrSlot& H = L.slot[slot];
  if (type == 1) {  // fixed codes (RFC 1951 3.2.6); 32 distance codes, 30 and 31 invalid
    for (int i = 0; i < 144; i++) H.lens[i] = 8;
    for (int i = 144; i < 256; i++) H.lens[i] = 9;
    for (int i = 256; i < 280; i++) H.lens[i] = 7;
    for (int i = 280; i < 288; i++) H.lens[i] = 8;
    for (int i = 288; i < 320; i++) H.lens[i] = 5;
    if (canon_build(H.lens, 288, H.cnt, H.nxt, T.lbase, nullptr, T.lsym, false, ll) ||
        canon_build(H.lens + 288, 32, H.cnt, H.nxt, T.dbase, T.dsym, nullptr, false, dl)) {
      s.err = ST_BAD_TABLE;
      return;
    }
    s.state = S_LIT;
    return;
  }
  if (type != 2) {
    s.err = ST_BAD_BLOCKTYPE;
    return;
  }
  refill(s, C);
  const uint32_t nlen = take(s, 5) + 257, ndist = take(s, 5) + 1, ncode = take(s, 4) + 4;
  if (nlen > 286 || ndist > 30) {
    s.err = ST_BAD_TABLE;
    return;
  }
  uint8_t* cl = H.lens + 300;  // 19 code-length code lengths (placed past the real lens)
  for (int i = 0; i < 19; i++) cl[i] = 0;
  for (uint32_t i = 0; i < ncode; i++) {
    refill(s, C);
    cl[c_clorder[i]] = (uint8_t)take(s, 3);
  }
  uint32_t clim[16];
  if (canon_build(cl, 19, H.cnt, H.nxt, H.clbase, H.clsym, nullptr, false, clim)) {
    s.err = ST_BAD_TABLE;
    return;
  }
  uint32_t have = 0;
  const uint32_t total = nlen + ndist;
  while (have < total) {
    refill(s, C);
    const uint32_t r = __builtin_bitreverse32((uint32_t)s.bb & 0x7f) >> 25;  // 7-bit window
    int l = 1;
#pragma unroll
    for (int k = 1; k < 7; k++) l += (r >= (clim[k] >> 8));
    if (r >= (clim[7] >> 8)) {
      s.err = ST_BAD_TABLE;
      return;
    }
    const uint32_t sym = H.clsym[(r >> (7 - l)) + H.clbase[l]];
    take(s, (uint32_t)l);
    if (sym < 16) {
      H.lens[have++] = (uint8_t)sym;
    } else {
      uint32_t rep, v = 0;
      if (sym == 16) {
        if (have == 0) {
          s.err = ST_BAD_TABLE;
          return;
        }
        v = H.lens[have - 1];
        rep = 3 + take(s, 2);
      } else if (sym == 17) {
        rep = 3 + take(s, 3);
      } else {
        rep = 11 + take(s, 7);
      }
      if (have + rep > total) {
        s.err = ST_BAD_TABLE;
        return;
      }
      for (uint32_t i = 0; i < rep; i++) H.lens[have++] = (uint8_t)v;
    }
  }
  if (H.lens[256] == 0) {
    s.err = ST_BAD_TABLE;
    return;
  }
  if (canon_build(H.lens, (int)nlen, H.cnt, H.nxt, T.lbase, nullptr, T.lsym, false, ll) ||
      canon_build(H.lens + nlen, (int)ndist, H.cnt, H.nxt, T.dbase, T.dsym, nullptr, true, dl)) {
    s.err = ST_BAD_TABLE;
    return;
  }
  s.state = S_LIT;
}

__global__ __launch_bounds__(64) void huff_decode_kernel(
    const uint8_t* __restrict__ C, const int64_t* __restrict__ blk_pos,
    const int32_t* __restrict__ blk_csize, const int32_t* __restrict__ blk_usize,
    const int64_t* __restrict__ uoff, int64_t nblk, uint16_t* __restrict__ tok,
    int32_t* __restrict__ tok_count, int32_t* __restrict__ status, int32_t* __restrict__ counter) {
  __shared__ LdsA L;
  const int lane = threadIdx.x;
  for (int i = lane; i < 29; i += 64) {
    L.lbase_k[i] = c_lbase[i];
    L.lext_k[i] = c_lext[i];
  }
  for (int i = lane; i < 30; i += 64) {
    L.dbase_k[i] = c_dbase[i];
    L.dext_k[i] = c_dext[i];
  }
  __syncthreads();
  Lane s;
  s.state = S_IDLE;
  s.err = 0;
  s.blk = -1;
  uint32_t ll[16], dl[16];
#pragma unroll
  for (int k = 0; k < 16; k++) ll[k] = dl[k] = 0;

  for (;;) {
    // ---- finish blocks
    if (s.state == S_DONE || (s.state != S_IDLE && s.state != S_EXIT && s.err)) {
      if (s.err == 0) {
        // bits consumed must lie within the deflate data
        const int64_t used = 8 * (s.ip - s.dstart) - (int64_t)s.bc;
        if (used > 8 * (int64_t)s.dbytes) s.err = ST_OVERREAD;
        else if (s.produced != s.isize) s.err = ST_SHORT;
      }
      // tail of the token stream: one 32-byte store (the region has 32 bytes of slack)
      if (s.sc > 0) {
        for (int i = s.sc; i < 16; i++) L.stage[lane][i] = 0;
        const int keep = s.sc;
        s.sc = 16;
        flush16(L, lane, s, tok);
        s.ntok -= 16 - keep;
      }
      tok_count[s.blk] = s.ntok;
      status[s.blk] = s.err;
      s.state = S_IDLE;
      s.err = 0;
    }
    // ---- hand out blocks to idle lanes
    const uint64_t idle = __ballot(s.state == S_IDLE);
    if (idle) {
      int base = 0;
      if (lane == (int)__builtin_ctzll(idle))
        base = atomicAdd(counter, (int)__builtin_popcountll(idle));
      base = __shfl(base, (int)__builtin_ctzll(idle), 64);
      if (s.state == S_IDLE) {
        const int rank = (int)__builtin_popcountll(idle & ((1ull << lane) - 1));
        const int64_t b = (int64_t)base + rank;
        if (b < nblk) start_block(s, C, blk_pos, blk_csize, blk_usize, uoff, b);
        else s.state = S_EXIT;
      }
    }
    const uint64_t live = __ballot(s.state != S_EXIT);
    if (!live) break;
    // ---- headers, several lanes at a time
    const uint64_t need = __ballot(s.state == S_HDR);
    const uint64_t act = __ballot(s.state == S_LIT || s.state == S_DIST || s.state == S_STORED);
    const int nneed = (int)__builtin_popcountll(need), nact = (int)__builtin_popcountll(act);
    if (need && (nneed >= 8 || nact < 48)) {
      // the first HDR_SLOTS waiting lanes decode their headers together
      const int rank = (int)__builtin_popcountll(need & ((1ull << lane) - 1));
      if (s.state == S_HDR && rank < HDR_SLOTS) {
        do_header(s, L, lane, rank, C, ll, dl);
        if (s.err) s.state = S_DONE;
      }
    }
    // ---- decode: one code per lane per iteration
    for (int it = 0; it < ITERS; it++) {
      const bool lit = s.state == S_LIT, dist = s.state == S_DIST, stored = s.state == S_STORED;
      if (!(lit || dist || stored)) continue;
      refill(s, C);
      if (stored) {
        const uint32_t v = take(s, 8);
        put_tok(L, lane, s, (uint16_t)v);
        s.produced++;
        if (--s.pend == 0) s.state = s.last ? S_DONE : S_HDR;
        if (s.produced >= s.isize) s.state = S_DONE;
      } else {
        const uint32_t r = rev15((uint32_t)s.bb & 0x7fff);
        int l = 1;
#pragma unroll
        for (int k = 1; k < 15; k++) l += r >= (dist ? dl[k] : ll[k]);
        const uint32_t lim15 = dist ? dl[15] : ll[15];
        if (r >= lim15) {
          s.err = ST_BAD_CODE;
          s.state = S_DONE;
          continue;
        }
        const LaneTab& T = L.tab[lane];
        const int idx = (int)(r >> (15 - l)) + (dist ? T.dbase[l] : T.lbase[l]);
        const uint32_t sym = dist ? T.dsym[idx] : T.lsym[idx];
        take(s, (uint32_t)l);
        if (lit) {
          if (sym < 256) {
            put_tok(L, lane, s, (uint16_t)sym);
            s.produced++;
            if (s.produced >= s.isize) s.state = S_DONE;
          } else if (sym == 256) {
            s.state = s.last ? S_DONE : S_HDR;
          } else if (sym <= 285) {
            const int k = (int)sym - 257;
            s.pend = (int32_t)L.lbase_k[k] + (int32_t)take(s, L.lext_k[k]);
            s.state = S_DIST;
          } else {
            s.err = ST_BAD_CODE;
            s.state = S_DONE;
          }
        } else {
          if (sym >= 30) {
            s.err = ST_BAD_CODE;
            s.state = S_DONE;
            continue;
          }
          const int32_t d = (int32_t)L.dbase_k[sym] + (int32_t)take(s, L.dext_k[sym]);
          if (d > s.produced) {
            s.err = ST_BAD_DIST;
            s.state = S_DONE;
            continue;
          }
          int32_t len = s.pend;
          const int32_t room = s.isize - s.produced;
          if (len > room) len = room;  // Inflater stops at ISIZE
          put_tok(L, lane, s, (uint16_t)(255 + len));  // length token: 256..513
          put_tok(L, lane, s, (uint16_t)(0x8000u | (uint32_t)(d - 1)));
          s.produced += len;
          s.state = s.produced >= s.isize ? S_DONE : S_LIT;
        }
      }
      if (s.sc >= 16) flush16(L, lane, s, tok);
    }
  }
}

// ------------------------------------------------------------------ K2b
constexpr int RT = 512;            // threads per resolve workgroup
constexpr int CHUNK_OUT = 2048;    // output bytes per chunk (span may exceed by < 258)
constexpr int SPAN_MAX = CHUNK_OUT + 260;

struct alignas(16) LdsB {
  uint8_t out[65536 + 16];         // block output, shifted by (uoff & 15)
  uint16_t own[SPAN_MAX];          // owner token (chunk index) of each output byte of the chunk
  uint16_t tk[RT + 1];             // chunk tokens
  int32_t dst[RT + 1];             // token output offsets inside the chunk
  int32_t wsum[RT / 64 + 1];
  uint32_t crcw[RT / 64];
  int32_t misc[8];
};

__constant__ uint32_t c_crc_tab[256];
__constant__ uint32_t c_x2n[32];

__device__ inline uint32_t gf2_mulmod(uint32_t a, uint32_t b) {  // reflected, poly 0xEDB88320
  uint32_t m = 1u << 31, p = 0;
  if (a == 0) return 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    b = b & 1 ? (b >> 1) ^ 0xEDB88320u : b >> 1;
  }
  return p;
}
__device__ inline uint32_t x8nmodp(uint64_t n) {  // x^(8n) mod P
  uint32_t p = 1u << 31;
  int k = 3;
  while (n) {
    if (n & 1) p = gf2_mulmod(c_x2n[k & 31], p);
    n >>= 1;
    k++;
  }
  return p;
}

__device__ inline int tok_len(uint32_t t) {  // output bytes of a token
  if (t < 256) return 1;
  if (t < 0x8000) return (int)(t - 255);
  return 0;  // distance token
}

__global__ __launch_bounds__(RT) void lz77_resolve_kernel(
    const uint16_t* __restrict__ tok, const int32_t* __restrict__ tok_count,
    const int64_t* __restrict__ blk_pos, const int32_t* __restrict__ blk_csize,
    const int32_t* __restrict__ blk_usize, const int64_t* __restrict__ uoff, int64_t nblk,
    const uint8_t* __restrict__ C, uint8_t* __restrict__ U, int32_t* __restrict__ status,
    int32_t verify_crc) {
  __shared__ LdsB L;
  const int64_t b = blockIdx.x;
  if (b >= nblk) return;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  if (status[b] != ST_OK) return;
  const int32_t isize = blk_usize[b];
  const int64_t ub = uoff[b];
  const int sh = (int)(ub & 15);  // LDS image is aligned like U
  const int32_t ntok = tok_count[b];
  const uint16_t* T = reinterpret_cast<const uint16_t*>(reinterpret_cast<const uint8_t*>(tok) +
                                                         tok_region(ub, b));
  uint8_t* O = L.out + sh;
  int32_t produced = 0, t0 = 0;
  while (t0 < ntok) {
    // tokens of this chunk (a match's two tokens never straddle chunks)
    const int32_t i = t0 + t;
    const uint32_t tv = i < ntok ? T[i] : 0xffffu;
    L.tk[t] = (uint16_t)tv;
    if (t == 0) L.tk[RT] = t0 + RT < ntok ? T[t0 + RT] : 0xffffu;
    int len = i < ntok ? tok_len(tv) : 0;
    // block-wide exclusive scan of len
    int v = len;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      int u = __shfl_up(v, o, 64);
      if (lane >= o) v += u;
    }
    if (lane == 63) L.wsum[wv] = v;
    __syncthreads();
    int woff = 0;
    for (int w = 0; w < wv; w++) woff += L.wsum[w];
    const int d0 = woff + v - len;
    L.dst[t] = d0;
    __syncthreads();
    // chunk cut: tokens starting below CHUNK_OUT, not splitting a match pair
    if (t == 0) {
      int lo = 0, hi = RT;  // first token with dst >= CHUNK_OUT
      while (lo < hi) {
        int m = (lo + hi) >> 1;
        if (L.dst[m] >= CHUNK_OUT) hi = m;
        else lo = m + 1;
      }
      int n = lo;
      if (n > ntok - t0) n = ntok - t0;
      if (n > 0) {
        const uint32_t lt = L.tk[n - 1];
        if (lt >= 256 && lt < 0x8000) n--;  // match length token without its distance
      }
      const int span = n > 0 ? (n < RT ? L.dst[n] : L.dst[RT - 1] + tok_len(L.tk[RT - 1])) : 0;
      L.misc[0] = n;
      L.misc[1] = span;
    }
    __syncthreads();
    const int n = L.misc[0], span = L.misc[1];
    // owner map: own[byte] = last token index starting at or before it
    for (int x = t; x < span; x += RT) L.own[x] = 0;
    __syncthreads();
    if (t < n && len > 0) L.own[d0] = (uint16_t)t;
    __syncthreads();
    // inclusive max-scan over own[0..span): each thread a contiguous run
    {
      const int per = (span + RT - 1) / RT;
      const int a = t * per, e = min(span, a + per);
      int m = 0;
      for (int x = a; x < e; x++) m = max(m, (int)L.own[x]);
      int vm = m;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        int u = __shfl_up(vm, o, 64);
        if (lane >= o) vm = max(vm, u);
      }
      if (lane == 63) L.wsum[wv] = vm;
      __syncthreads();
      int carry = 0;
      for (int w = 0; w < wv; w++) carry = max(carry, L.wsum[w]);
      int excl = __shfl_up(vm, 1, 64);
      if (lane == 0) excl = 0;
      int run = max(carry, excl);
      __syncthreads();
      for (int x = a; x < e; x++) {
        run = max(run, (int)L.own[x]);
        L.own[x] = (uint16_t)run;
      }
    }
    __syncthreads();
    // resolve every byte of the chunk
    for (int x = t; x < span; x += RT) {
      int p = x;  // position relative to the chunk start
      uint8_t val = 0;
      for (int hop = 0; hop < 4096; hop++) {
        const int o = L.own[p];
        const uint32_t tv2 = L.tk[o];
        if (tv2 < 256) {
          val = (uint8_t)tv2;
          break;
        }
        const int D = (int)(L.tk[o + 1] & 0x7fff) + 1;
        const int ds = L.dst[o];
        const int j = p - ds;
        p = j < D ? p - D : ds - D + (j % D);
        if (p < 0) {
          val = O[produced + p];
          break;
        }
      }
      O[produced + x] = val;
    }
    __syncthreads();
    produced += span;
    t0 += n;
    if (n == 0) break;  // cannot happen for well-formed token streams
  }
  if (produced != isize) {
    if (t == 0) status[b] = ST_SHORT;
    return;
  }
  // CRC32 of the block: thread t hashes a contiguous run, runs combined by x^(8n) shifts
  if (verify_crc) {
    const int per = (isize + RT - 1) / RT;
    const int a = min(isize, t * per), e = min(isize, a + per);
    uint32_t c = 0;
    for (int x = a; x < e; x++) c = c_crc_tab[(c ^ O[x]) & 0xff] ^ (c >> 8);
    c = gf2_mulmod(x8nmodp((uint64_t)(isize - e)), c);
    for (int o = 32; o >= 1; o >>= 1) c ^= __shfl_xor(c, o, 64);
    if (lane == 0) L.crcw[wv] = c;
    __syncthreads();
    if (t == 0) {
      uint32_t x = 0;
      for (int w = 0; w < RT / 64; w++) x ^= L.crcw[w];
      const uint32_t init = gf2_mulmod(x8nmodp((uint64_t)isize), 0xffffffffu);
      const uint32_t crc = (x ^ init) ^ 0xffffffffu;
      const uint8_t* tr = C + blk_pos[b] + blk_csize[b] - 8;
      const uint32_t want = (uint32_t)tr[0] | ((uint32_t)tr[1] << 8) | ((uint32_t)tr[2] << 16) |
                            ((uint32_t)tr[3] << 24);
      if (crc != want) status[b] = ST_CRC;
    }
  }
  // store: 16-byte stores for the aligned interior, bytes for the edges
  uint8_t* dstU = U + ub;
  const int head = (16 - sh) & 15;  // bytes before the first 16-byte boundary
  for (int x = t; x < min(head, isize); x += RT) dstU[x] = O[x];
  const int nvec = (isize - head) / 16;
  const uint4* src4 = reinterpret_cast<const uint4*>(O + head);
  uint4* dst4 = reinterpret_cast<uint4*>(dstU + head);
  for (int k = t; k < nvec; k += RT) dst4[k] = src4[k];
  for (int x = head + 16 * nvec + t; x < isize; x += RT) dstU[x] = O[x];
}

}  // namespace

int64_t token_bytes(const int64_t uoff_total, int64_t nblk) { return 2 * uoff_total + 64 * nblk + 128; }

void launch_inflate2(const uint8_t* C, const int64_t* blk_pos, const int32_t* blk_csize,
                     const int32_t* blk_usize, const int64_t* uoff, int64_t nblk, uint16_t* tok,
                     int32_t* tok_count, int32_t* counter, uint8_t* U, int32_t* status,
                     int32_t verify_crc, int n_cu, hipEvent_t mid, hipStream_t s) {
  if (nblk <= 0) return;
  (void)hipMemsetAsync(counter, 0, sizeof(int32_t), s);
  const int waves = n_cu * 3;  // three 64-lane waves per CU (LDS ~51 KiB each)
  hipLaunchKernelGGL(huff_decode_kernel, dim3((unsigned)waves), dim3(64), 0, s, C, blk_pos,
                     blk_csize, blk_usize, uoff, nblk, tok, tok_count, status, counter);
  if (mid) (void)hipEventRecord(mid, s);
  hipLaunchKernelGGL(lz77_resolve_kernel, dim3((unsigned)nblk), dim3(RT), 0, s, tok, tok_count,
                     blk_pos, blk_csize, blk_usize, uoff, nblk, C, U, status, verify_crc);
}

void init_inflate_tables() {
  static bool done = false;
  if (done) return;
  uint32_t tab[256];
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = c & 1 ? (c >> 1) ^ 0xEDB88320u : c >> 1;
    tab[i] = c;
  }
  auto mul = [](uint32_t a, uint32_t b) {
    uint32_t m = 1u << 31, p = 0;
    for (;;) {
      if (a & m) {
        p ^= b;
        if ((a & (m - 1)) == 0) break;
      }
      m >>= 1;
      b = b & 1 ? (b >> 1) ^ 0xEDB88320u : b >> 1;
    }
    return p;
  };
  uint32_t x2n[32];
  uint32_t p = 1u << 30;  // x^1
  x2n[0] = p;
  for (int k = 1; k < 32; k++) x2n[k] = p = mul(p, p);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(c_crc_tab), tab, sizeof tab);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(c_x2n), x2n, sizeof x2n);
  done = true;
}

}  // namespace dq
