// dq_inflate3.hip -- Kernel 2 (v3): fused BGZF block inflate + CRC32, one workgroup per block.
//
// Replaces htsjdk BlockCompressedInputStream / BlockGunzipper.unzipBlock (htsjdk 2.16.0, reached
// from D/impl/formats/bam/BamSource.java:172-175) -> java.util.zip.Inflater, plus the CRC32 check
// that htsjdk leaves off by default.
//
// A BGZF block is an independent raw-DEFLATE stream of <= 64 KiB output, so blocks are decoded
// independently: one 512-thread workgroup per block, the whole output image in LDS (two
// workgroups per CU: 80 KiB of LDS each).  Per deflate block of the stream:
//   1. header   -- every thread reads BFINAL/BTYPE/HLIT/HDIST/HCLEN; 19 threads read the
//                  code-length code lengths; 128 threads fill its 7-bit decode table; the eight
//                  waves decode the code-length sequence, one 128-bit window each: every lane
//                  decodes the symbols at two offsets, the window's successor table is doubled by
//                  lane shuffles, each window's exits are chained across the windows by one
//                  thread, and runs are placed by wave scans (read_lengths).
//   2. tables   -- canonical codes are assigned in parallel (wave scans of one-hot length
//                  counters give each symbol its rank among equal lengths); 10-bit litlen / 8-bit
//                  distance root tables of 16-bit entries that carry the decoded value (literal
//                  byte, length base and extra-bit count, distance base and extra-bit count:
//                  ent_ll / ent_d) plus variable-size second-level tables for longer codes (one per
//                  root prefix, sized by its longest code), so every code decodes with at most two
//                  LDS reads and no arithmetic on the symbol number.
//   3. spec     -- the bit range is cut into NDEC segments; lane t decodes from OV bits before
//                  segment t (warm-up), counts output from its first symbol boundary at or after
//                  the segment start and stops at its EXIT, the first boundary at or after the next
//                  segment; it also records checkpoints (its first boundary past every CKI bits).
//                  Huffman codes self-synchronise, so an exit is almost always on the true path.
//   4. rounds   -- lanes whose first boundary differs from the predecessor's exit re-decode from
//                  that exit (compacted onto the first threads by an LDS counter) until they meet
//                  the speculative path at a checkpoint (same bit position = same decoder state),
//                  then take the rest of the speculative run; repeat while an exit changed.
//   5. emit     -- an exclusive scan of the per-lane byte counts gives every lane its output
//                  offset; lanes decode once more, writing literals into the LDS image and, for
//                  each match, a 3-byte descriptor (dist-1 | len-3 << 15) at its first byte plus a
//                  bit in a match-start bitmap.
// Then, for the whole BGZF block:
//   6. resolve  -- lastStart[w] = last match start at or before the end of bitmap word w (a max
//                  scan), so the owner of any byte is found in O(1).  Batches of NB chunks of 512
//                  bytes: (a) every byte's first hop (owner, descriptor, copy source start - dist +
//                  (offset mod dist)) is published as a 16-bit next pointer, then pointer jumping
//                  (barrier-free) until a literal or a byte before the byte's 512-byte step; (b)
//                  step by step, one LDS read + write per byte and one barrier; (c) the batch's
//                  16-byte lines are stored to U.  Batches are software-pipelined (batch k+1's hops
//                  and jumps run between batch k's steps).
//   7. CRC32    -- slice-by-4 per thread over a 132-byte slice, combined across threads by
//                  multiplying with x^(8n) mod P (precomputed per slice index); compared with the
//                  gzip trailer.
// Output stops at ISIZE (Inflater.inflate(buf, 0, ISIZE) semantics); fewer bytes is an error.
#include "dq_inflate_core.h"
#include "dq_internal.h"

#include <mutex>
#include <vector>

namespace dq {
namespace {

using namespace dqi;

#define DQ_HD __device__ __host__ __attribute__((always_inline)) inline

// threads per block workgroup (= speculative lanes): two workgroups per CU (the LDS image), so
// WG / 128 waves per SIMD, which bounds the VGPRs (MI355X_MICROARCH.md: 512 / waves per SIMD)
#ifndef DQ_BLK_WG
#define DQ_BLK_WG 512
#endif
constexpr int WG = DQ_BLK_WG;
static_assert(WG % 128 == 0 && WG >= 512 && WG <= 1024, "whole waves on every SIMD");
constexpr int NWV = WG / 64;      // waves per workgroup
constexpr int NDEC = WG;          // speculative decode lanes (<= WG)
constexpr uint32_t OV_DEFAULT = 96;  // speculative warm-up bits before each segment
#ifndef DQ_TAIL_OV
#define DQ_TAIL_OV OV_DEFAULT  // the tail kernel's (dev builds sweep it)
#endif
constexpr int OUTCAP = 65536 + 24;  // + alignment shift (<= 15) + descriptor overhang; bm 8-aligned
// resolve shape (tuning builds): NB chunks of G * WG bytes per batch; DQ_CSTEP = 1: one ordered
// step per chunk instead of per 512 bytes (longer in-step chains, fewer barriers; always so when
// a chunk is not a whole number of 512-byte steps)
#ifndef DQ_CSTEP
#define DQ_CSTEP 0
#endif
#ifndef DQ_RES_NB
#define DQ_RES_NB (WG == 512 ? 4 : 2)
#endif
#ifndef DQ_RES_G
#define DQ_RES_G 1
#endif
constexpr int RES_NXT = DQ_RES_NB * DQ_RES_G * WG;  // resolve batch bytes (NB * G * WG)
constexpr int NCARRY = (65536 + RES_NXT - 1) / RES_NXT + 1;  // batches of a block (carry slots)


// 16-bit decode table layout: [litlen root | litlen subtables | dist root | dist subtables]
constexpr int LR = 10, DR = 8;            // root bits
constexpr int LSB = 15 - LR, DSB = 15 - DR;  // second-level index bits
constexpr int LSLOTS = 16, DSLOTS = 4;    // second-level entries: LSLOTS * 2^LSB, DSLOTS * 2^DSB
constexpr int MAXGRP = 64;                // second-level tables (prefix groups) per alphabet
constexpr int T_LSUB = 1 << LR;
constexpr int T_DROOT = T_LSUB + LSLOTS * (1 << LSB);
constexpr int T_DSUB = T_DROOT + (1 << DR);
constexpr int T_END = T_DSUB + DSLOTS * (1 << DSB);
constexpr int HB_WORDS = 160;             // staged dynamic-header words (aliases T)
// Root entries whose code length field (bits 0-3) is 0 are not codes: 0 = no code (incomplete
// table); sb << 4 | off << 7 (sb = bits 4-6 != 0) = the second-level table of 2^sb entries at
// `off` (zlib-style: sized by the longest code under the prefix, so every alphabet fits the
// second-level area); E_SLOW = canonical decode (only past MAXGRP tables or the area).
constexpr uint16_t E_SLOW = 0x0080;
// Decoded litlen entry: code length (bits 0-3), M = length/EOB/invalid (bit 4), extra-bit count
// (bits 5-7), value (bits 8-15): the literal byte or length base - 3.  EOB and the invalid symbols
// 286/287 are M entries with 0 extra bits and values 248/249, which no length base has, so
// (e & 0xFEF0) == 0xF810 finds both.
constexpr uint32_t LL_EOB = 0xF810, LL_BAD = 0xF910;
DQ_HD uint16_t ent_ll(uint32_t sym, uint32_t len) {
  if (sym < 256) return (uint16_t)(sym << 8 | len);
  if (sym == 256) return (uint16_t)(LL_EOB | len);
  if (sym > 285) return (uint16_t)(LL_BAD | len);
  const uint32_t k = sym - 257;  // RFC 1951 3.2.5
  const uint32_t x = (k < 8 || k == 28) ? 0u : (k - 4) >> 2;
  const uint32_t base = k < 8 ? k + 3 : k == 28 ? 258u : ((4u + (k & 3u)) << ((k - 4) >> 2)) + 3u;
  return (uint16_t)((base - 3) << 8 | x << 5 | 16u | len);
}
// Decoded distance entry: code length (bits 0-3), extra-bit count (4-7), base - 1 = m << s with
// s (8-11) and m (12-13), invalid symbol 30/31 (bit 14).
DQ_HD uint16_t ent_d(uint32_t d, uint32_t len) {
  if (d >= 30) return (uint16_t)(0x4000u | len);
  const uint32_t x = d < 4 ? 0u : (d - 2) >> 1;
  const uint32_t m = d < 2 ? d : 2u + (d & 1u), sh = d < 2 ? 0u : (d >> 1) - 1u;
  return (uint16_t)(m << 12 | sh << 8 | x << 4 | len);
}

enum : int32_t { F_EXIT = 0, F_EOB = 1, F_ERR = 2, F_END = 3 };

// The tail kernel (inflate_tail_kernel): the deflate blocks of a BGZF block after its first one,
// when they are small (htsjdk's level 5 leaves ~700 symbols, ~2.9 KB of output, after a first
// block of 16,383 symbols).  The block kernel resolves, stores and checksums the bytes before the
// tail and leaves this descriptor; one wave per tail does the rest.
constexpr int TOUT = 4096;            // tail output bytes one wave holds
constexpr int TAIL_MAX_BITS = 32768;  // tail deflate bits (64 speculative lanes of <= 512 bits)
constexpr int TW = 4;                 // tails (waves) per tail-kernel workgroup
#ifndef DQ_ROOT_REG  // the tail's root-table fill with the length range ends in registers
#define DQ_ROOT_REG 1
#endif
#ifndef DQ_TAIL_HDR1  // the tail's header loads in one round trip (0: block header first)
#define DQ_TAIL_HDR1 1
#endif
constexpr int T_NCK = 4;              // checkpoints per speculative lane in the tail kernel
#ifndef DQ_TAIL_SEG
#define DQ_TAIL_SEG 96
#endif
constexpr int TAIL_SEG_MIN = DQ_TAIL_SEG;  // shortest speculative segment of a tail (bits)
constexpr int TIM_W = 32;  // DQ_TIMING words per block (dq_api.hip reads the same layout)
struct TailDesc {
  int32_t pos;       // bit position (from the block's aligned deflate base) of the tail's header
  int32_t produced;  // output bytes before the tail
  uint32_t crc_raw;  // CRC register (init 0, no final xor) of those bytes
  int32_t flag;      // 1: the tail kernel owns the rest of this block
};

struct alignas(16) LdsI {
  // decode-table layout (dsym, ll_second, d_second): the second-level tables follow each root
  static constexpr int kLSUB = T_LSUB, kDROOT = T_DROOT, kDSUB = T_DSUB;
  [[maybe_unused]] static constexpr int kTEND = T_END;  // DQ_CHK bound
  static constexpr bool kPair = true;  // literal-pair table (dsym)
  alignas(8) uint32_t bm[2048];   // match-start bitmap (read as 64-bit words in resolve)
  union {
    struct {
      uint16_t T[T_END];
      HuffCanon hl, hd;           // canonical descriptions (E_SLOW fallback)
      uint16_t lend[16], dend[16];  // left-aligned end of the length-l codes' root range (l <= R)
      uint16_t lent[288];         // decoded table entry of canonical position q
      uint16_t dent[32];
      union {
        uint16_t pair[1 << LR];   // decode: second literal of a root index (lit << 4 | len), 0 none
        struct {
          uint8_t lens[320];      // litlen lengths [0, 288), distance lengths [288, 320)
          uint8_t clen[20];
          uint16_t clt[128];      // code-length code: sym << 3 | len (len 0 = invalid)
          union {
            struct {              // build_tables
              int32_t cntw[NWV];  // per-wave counts of second-level tables
              int32_t cnts[NWV];  // per-wave second-level entries
              uint32_t ginfo[MAXGRP + 32];  // per second-level table (litlen, then distance): offset | sb << 16
              uint32_t cntp[8][8];  // per-wave counts of each code length, 16 bits per length
              uint16_t pref[320];   // root prefix of each long code, by canonical position
            };
            struct {              // read_lengths: one 128-bit window per wave
              uint8_t exitm[NWV][16];  // window w entered at offset e < 16 -> entry offset into w + 1
              int32_t ent[NWV + 1];    // true entry offset of each window (255: none)
              int32_t wt[NWV];         // lengths the window's path symbols write
              int32_t lv[NWV];         // the window's last non-repeat value (-1 none)
              int32_t endp;          // bit position after the last code-length symbol
            };
          };
        } h;
      } x;
    } d;
    struct {
      uint16_t last_start[1024];  // last match start <= end of 64-bit bitmap word (0xffff none)
      uint16_t nxt[RES_NXT];      // next pointer of each byte of the batch
      int32_t carry_ms[NCARRY];    // the match carried into batch k + 1 (start, -1 none), and its
      uint32_t carry_desc[NCARRY]; // descriptor: read before any step overwrites a descriptor
    } r;
    uint32_t crc4[4][256];
  } u;
  int32_t misc[32];
  union {
    struct {
      int32_t wsum[16];
      int32_t small[8 * 7];       // per-lane arrays when the image tail is too short
    };
    // dummy words of the branch-free stores: 16 per wave in the speculative pass (wsum is dead,
    // `small` may hold the arrays), one per lane in the emit (both dead)
    uint32_t scratch[16 + 8 * 7];
  };
  // output image: byte x at out[sh + x].  Last, so every table above sits below 64 KiB and its
  // constant offset folds into the ds_read/ds_write offset field (one VALU add fewer per lookup)
  alignas(16) uint8_t out[OUTCAP];
};
static_assert(sizeof(((LdsI*)nullptr)->scratch) >= 64 * 4, "one emit dummy word per lane");
static_assert(offsetof(LdsI, out) < 65536 - 4096, "the tables' offsets fit the DS offset field");
static_assert(2 * sizeof(LdsI) <= 160 * 1024, "two workgroups per CU");
static_assert(HB_WORDS * 4 <= T_END * 2, "header staging fits the decode table");

// emit's per-lane dummy words (one per lane of a wave): dead scratch during the emit
__device__ inline uint32_t* emit_dummy(LdsI& L) { return L.scratch; }

__constant__ uint32_t c_crc4[4][256];
__constant__ uint32_t c_x2n[32];  // x^(2^k) mod P (reflected)
__constant__ uint32_t c_x8n[TOUT + 1];  // x^(8 k) mod P, k <= TOUT: the tail kernel's CRC shifts
// CRC slices: an odd number of words (132 bytes = 33 words at 512 threads), so the 64 lanes of a
// wave read 64 different LDS banks (128-byte slices put every lane of a wave in the same bank: a
// 32-way conflict on every data read)
constexpr int CRC_SL = 4 * (((65536 / 4 + WG - 1) / WG) | 1);
static_assert(CRC_SL * WG >= 65536, "the slices cover the largest block");
__constant__ uint32_t c_slice_shift[WG];  // x^(8 * CRC_SL * k) mod P, k = 0..WG-1
__constant__ uint8_t c_clorder3[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// misc slots
enum { M_ERR = 0, M_SLOW = 1 /* an E_SLOW root entry in this deflate block's tables */, M_A = 4, M_LAST, M_MORE, M_MORE1,
       M_LQ0 = 15, M_LQN, M_DQ0, M_DQN, M_NEXT,
       M_LASTF, M_RCNT = 28 /* and 29: redo-list counters of even / odd rounds */,
       M_DIRTY = 30 /* and 31: a re-decoded exit changed, even / odd rounds */ };

template <class LT>
__device__ __attribute__((always_inline)) inline void set_err(LT& L, int32_t code) { atomicCAS(&L.misc[M_ERR], 0, code); }


#define DQ_AI __device__ __attribute__((always_inline)) inline

// The thread index behind an empty volatile asm: values derived from it cannot be hoisted out of
// the deflate-block loop.  Hoisted per-thread constants (bit-reversed indices, LDS addresses,
// lane masks) lived across the whole loop and were spilled to scratch once per workgroup --
// 48 B/thread, ~24 KiB of HBM writes per BGZF block -- while recomputing them costs a few VALU
// ops per deflate block.
DQ_AI int tid_fresh() {
  int t = (int)threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
DQ_AI void st_nt(uint4* d, uint4 v) {  // streaming store (nt): U is not re-read by this kernel
  u32x4 x = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(d));
}

// The compressed words.  (Staging a deflate block's words in the LDS image tail for the speculative
// pass and the rounds was measured: no faster, profiles/r3a_lds_bits_ab.txt -- the refill load is
// issued a half step ahead and is not the decode step's critical path.)
// A word index becomes a 32-bit byte offset from the block's (uniform) base: the load takes the
// SGPR-base + VGPR-offset form, with no 64-bit address arithmetic per refill.  (A buffer resource
// costs 4 more SGPRs, which the kernel spills: 4 v_readlane per load.)
struct GSrc {
  const uint32_t* __restrict__ p;
#ifdef DQ_CHECKED
  uint32_t lim;  // words past the member's deflate data the reader may load (refill look-ahead)
  uint32_t tag;  // the pass (1 spec, 2 redo, 3 emit) << 12, reported with the excess
#endif
  DQ_AI uint32_t operator[](uint32_t i) const {
#ifdef DQ_CHECKED
    DQ_CHKV(i < lim, CHK_K2_BITS, tag | min(i - lim + 1, 4095u));
#endif
    return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(p) + (i << 2));
  }
};

#ifndef DQ_BR64
#define DQ_BR64 0
#endif
#if DQ_BR64
// Bit reader (round 5): a 64-bit LSB-first buffer refilled 32 bits at a time from `nw`, the next
// input word, which every refill call reloads unconditionally (one global_load_dword, almost
// always an L1/L2 hit): the load lands in a loop-carried register and is first waited for at the
// next call, half a symbol later.  (A 16-byte group load needs a 4-way select of the word on every
// refill: 3 compares + 3 cndmasks + hazard nops per refill, 2 refills per symbol.)
struct BitR {
  uint64_t bb;
  uint32_t bc;
  uint32_t wp;    // word index of the next word to enter bb (br_pos = 32 * wp - bc)
  uint32_t nw;    // W[wp]
};
template <class S>
DQ_AI void br_init(BitR& r, const S& W, uint32_t bitpos) {
  const uint32_t wi = bitpos >> 5;
  const uint64_t lo = W[wi], hi = W[wi + 1];
  const uint32_t sh = bitpos & 31;
  r.bb = ((hi << 32) | lo) >> sh;
  r.bc = 64 - sh;
  r.wp = wi + 2;
  r.nw = W[r.wp];
}
template <class S>
DQ_AI void br_refill(BitR& r, const S& W) {
  const bool need = r.bc <= 32;
  r.bb |= (uint64_t)(need ? r.nw : 0u) << r.bc;  // one 32-bit select instead of a 64-bit one
  r.bc += need ? 32u : 0u;
  r.wp += need ? 1u : 0u;
  r.nw = W[r.wp];
}
DQ_AI uint32_t br_pos(const BitR& r) { return r.wp * 32 - r.bc; }
DQ_AI uint32_t br_peek(const BitR& r) { return (uint32_t)r.bb; }
template <class S>
DQ_AI void br_take(BitR& r, const S&, uint32_t n) {
  r.bb >>= n;
  r.bc -= n;
}
#else
// Bit reader: the bit position p and the two input words holding bits [32 (p >> 5), +64); a peek
// is one v_alignbit of them (32 bits from p: a litlen code + its extra bits <= 20, a distance
// code + its extra bits <= 28), an advance of n <= 28 bits crosses at most one word, which shifts
// in `nw` = W[(p >> 5) + 2].  nw is reloaded unconditionally after every advance (one
// global_load_dword, almost always an L1/L2 hit) and first waited for at the next crossing, half a
// symbol later.  No 64-bit shifts or ORs, and the position needs no arithmetic (round 5 kept a
// 64-bit buffer: a 64-bit shift and two ORs per refill, a 64-bit shift per take, and 32 wp - bc
// for every position test).
struct BitR {
  uint32_t p;       // bit position of the next bit
  uint32_t w0, w1;  // W[p >> 5], W[(p >> 5) + 1]
  uint32_t nw;      // W[(p >> 5) + 2]
};
template <class S>
DQ_AI void br_init(BitR& r, const S& W, uint32_t bitpos) {
  const uint32_t wi = bitpos >> 5;
  r.w0 = W[wi];
  r.w1 = W[wi + 1];
  r.nw = W[wi + 2];
  r.p = bitpos;
}
template <class S>
DQ_AI void br_refill(BitR&, const S&) {}
DQ_AI uint32_t br_pos(const BitR& r) { return r.p; }
DQ_AI uint32_t br_peek(const BitR& r) { return __builtin_amdgcn_alignbit(r.w1, r.w0, r.p); }
template <class S>
DQ_AI void br_take(BitR& r, const S& W, uint32_t n) {
  const uint32_t q = r.p + n;
  const bool c = (q ^ r.p) >= 32u;  // crossed into the next word
  r.w0 = c ? r.w1 : r.w0;
  r.w1 = c ? r.nw : r.w1;
  r.p = q;
  r.nw = W[(q >> 5) + 2];
}
#endif
// n (<= 25) bits at an arbitrary bit position
DQ_AI uint32_t peek_bits(const uint32_t* __restrict__ W, uint32_t pos, uint32_t n) {
  const uint32_t wi = pos >> 5;
  const uint64_t v = ((uint64_t)W[wi + 1] << 32) | W[wi];
  return (uint32_t)(v >> (pos & 31)) & ((1u << n) - 1);
}

// 3-byte match descriptor at image byte `a` via two aligned dword reads.
template <class LT>
DQ_AI uint32_t load_desc(const LT& L, int a) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(L.out + (a & ~3));
  return __builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)a & 3u) & 0xffffffu;
}

// A 16-bit table entry as a plain 32-bit value (ds_read_u16 zero-extends): behind an empty asm the
// compiler cannot narrow the entry's uses to 16-bit operations, which it then widened again with
// a v_and 0xffff per lookup (two per decode step in the ISA of round 5).
DQ_AI uint32_t zx16(uint16_t v) {
#ifndef DQ_NO_ZX16
  uint32_t x = v;
  asm("" : "+v"(x));
  return x;
#else
  return v;
#endif
}

// Second-level / canonical lookup for a root entry that is not a code.  SLOW = false (no E_SLOW
// entry in this deflate block's tables, M_SLOW): one read, with no nested branch -- a "no code"
// root entry (0: only in an incomplete code, which has no long codes) reads the first entry of the
// unused second-level area, an invalid-code sentinel (build_tables).
template <bool SLOW, class LT>
DQ_AI uint32_t ll_second(const LT& L, uint32_t e, uint32_t bb) {
  const uint32_t sb = (e >> 4) & 7;
  DQ_CHK(LT::kLSUB + (e >> 7) + ((bb >> LR) & ((1u << sb) - 1)) < (uint32_t)LT::kDROOT, CHK_K2_TABLE);
  if (!SLOW) return L.u.d.T[LT::kLSUB + (e >> 7) + ((bb >> LR) & ((1u << sb) - 1))];
  if (sb) return L.u.d.T[LT::kLSUB + (e >> 7) + ((bb >> LR) & ((1u << sb) - 1))];
  if (!(e & E_SLOW)) return 0u;
  int l = 0;
  const int k = canon_decode(bb, L.u.d.hl, LR + 1, &l);
  return k < 0 ? 0u : L.u.d.lent[k];
}
template <bool SLOW, class LT>
DQ_AI uint32_t d_second(const LT& L, uint32_t e, uint32_t bb) {
  const uint32_t sb = (e >> 4) & 7;
  DQ_CHK(LT::kDSUB + (e >> 7) + ((bb >> DR) & ((1u << sb) - 1)) < (uint32_t)LT::kTEND, CHK_K2_TABLE);
  if (!SLOW) return L.u.d.T[LT::kDSUB + (e >> 7) + ((bb >> DR) & ((1u << sb) - 1))];
  if (sb) return L.u.d.T[LT::kDSUB + (e >> 7) + ((bb >> DR) & ((1u << sb) - 1))];
  if (!(e & E_SLOW)) return 0u;
  int l = 0;
  const int k = canon_decode(bb, L.u.d.hd, DR + 1, &l);
  return k < 0 ? 0u : L.u.d.dent[k];
}


// One full symbol: a literal (value in len, is_m false) or a match (len, dist, is_m true); returns
// true instead when the symbol ends the run: EOB or an invalid code, told apart after the caller's
// loop by stop_end(e, p) from the litlen entry `e` (the bit after the EOB, or 0xffffffff) -- so
// the decode step itself carries no EOB arithmetic.  Straight-line: every lane does the litlen and the distance lookup (a
// literal lane consumes no distance bits), so a wave mixing literals and matches does not execute
// both paths one after the other.  The table entries carry the values (ent_ll / ent_d): a length
// is value + 3 + its extra bits, a distance m << s + 1 + its extra bits, each extra field one
// bit-field extract.
// Literal pairs: when the root index also holds a second whole literal (pair table) and the
// boundary between them lies before `lim` (the next bit position at which the caller looks at
// symbol boundaries: segment start/exit, checkpoint, end of data), both are taken at once and
// `lit2` is the second (else 0xffffffff) -- the boundaries the caller sees are unchanged.
template <bool SLOW, class S, class LT>
DQ_AI bool dsym(BitR& r, const S& W, const LT& L, uint32_t p, uint32_t lim,
                uint32_t& len, uint32_t& dist, uint32_t& lit2, bool& is_m, uint32_t& e) {
  br_refill(r, W);  // >= 32 bits: a litlen code + its extra bits (<= 20)
  uint32_t bb = br_peek(r);
  const uint32_t ri = bb & ((1u << LR) - 1);
  e = L.u.d.T[ri];
  uint32_t pe = 0;
  if constexpr (LT::kPair) pe = zx16(L.u.d.x.pair[ri]);
  if ((e & 15) == 0) e = ll_second<SLOW>(L, e, bb);
  const uint32_t nb = e & 15;
  const uint32_t lx = __builtin_amdgcn_ubfe(e, 5, 3);
  is_m = (e & 16) != 0;
  len = (e >> 8) + (is_m ? 3u : 0u) + __builtin_amdgcn_ubfe(bb, nb, lx);
  const bool two = pe != 0 && p + nb < lim;  // pe != 0: the root entry is a literal
  lit2 = two ? pe >> 8 : 0xffffffffu;
  br_take(r, W, nb + lx + (two ? (pe & 15) : 0u));
  br_refill(r, W);  // >= 32 bits: a distance code + its extra bits (<= 28)
  bb = br_peek(r);
  uint32_t e2 = zx16(L.u.d.T[LT::kDROOT + (bb & ((1u << DR) - 1))]);
  if (is_m && (e2 & 15) == 0) e2 = d_second<SLOW>(L, e2, bb);
  const uint32_t nb2 = e2 & 15, dx = __builtin_amdgcn_ubfe(e2, 4, 4);
  dist = (__builtin_amdgcn_ubfe(e2, 12, 2) << __builtin_amdgcn_ubfe(e2, 8, 4)) + 1u +
         __builtin_amdgcn_ubfe(bb, nb2, dx);
  br_take(r, W, is_m ? nb2 + dx : 0u);
  // SLOW = false: a code-less index reads the invalid sentinels build_tables leaves at the first
  // second-level entries, so no entry here has code length 0
  // (EOB is an M entry, so the distance bits taken above are not the stream's: the caller stops)
  return (SLOW && nb == 0) || (e & 0xFEF0u) == 0xF810u ||
         (is_m && ((SLOW && nb2 == 0) || (e2 & 0x4000u)));
}
// After dsym stopped at position p with litlen entry e: the bit after the EOB, or 0xffffffff for an
// invalid code (in the litlen or the distance alphabet)
DQ_AI uint32_t stop_end(uint32_t e, uint32_t p) {
  return (e & 15) != 0 && (e & 0xFFF0u) == LL_EOB ? p + (e & 15) : 0xffffffffu;
}

enum : int32_t { F_DEAD = 4 };  // speculative path found no boundary >= sB (garbage)

// Decode from `start`; output is counted from the first symbol boundary >= sB (*Bp) and the
// run stops at the first boundary >= sE (*Ep).  Returns F_EXIT / F_EOB (*Ep = bit after EOB) /
// F_ERR / F_END (ran off the data) / F_DEAD (no boundary >= sB before an error, EOB or the end).
constexpr int NCK_DEFAULT = 8;  // checkpoints per speculative lane
constexpr uint32_t CKI_DEFAULT = 48;  // checkpoint spacing in bits (>= the longest symbol: a symbol
                                // crosses at most one threshold; most paths re-synchronise
                                // within ~100 bits, segments are ~160-1000 bits)

// Speculative lanes also record checkpoints: the first symbol boundary at or past sB + CKI * (j+1)
// (offset from sB << 16 | bytes counted so far), j < nck, at ck[j * ckstride] (nullptr: none).
// A spacing below the longest symbol only loses merges: a merge needs equal bit positions, and
// equal positions at symbol boundaries are equal decoder states whatever the checkpoint index.
template <bool SLOW, class S, class LT>
DQ_AI int run_seg(const S& W, const LT& L, uint32_t start, uint32_t sB,
                  uint32_t sE, uint32_t endbits, int32_t* Bp, int32_t* Ep, int32_t* cntp,
                  uint32_t* ck, int ckstride, uint32_t CKI, int NCK) {
  BitR r;
  br_init(r, W, start);
  uint32_t p = br_pos(r);
  uint32_t len = 0, dist = 0, lit2, e = 0;
  bool m;
  // warm-up: to the first symbol boundary >= sB, nothing counted (one compare per step: the
  // data end is folded into the bound and tested once after the loop)
  const uint32_t sBe = min(sB, endbits);
  while (p < sBe) {
    if (dsym<SLOW>(r, W, L, p, sBe, len, dist, lit2, m, e)) {
      len = stop_end(e, p);
      *Ep = (int32_t)(len != 0xffffffffu ? len : p);
      *Bp = -1;
      *cntp = 0;
      return F_DEAD;
    }
    p = br_pos(r);
  }
  if (p < sB) {  // the data ended first
    *Ep = (int32_t)p;
    *Bp = -1;
    *cntp = 0;
    return F_DEAD;
  }
  const int32_t B = (int32_t)p;
  int32_t cnt = 0;
  int f;
  uint32_t thr = ck ? sB + CKI : 0xffffffffu;
  // a lane crosses a checkpoint every few symbols, so some lane of the wave does on most steps:
  // written branch-free, the step that crosses none stores to the lane's dummy word (wsum is
  // dead during the speculative pass; `small` may hold the per-lane arrays).  The threshold keeps
  // advancing past the last checkpoint (checkpoint j < NCK is the pointer test ckp < cke): no
  // checkpoint counter and no saturated threshold (four VALU ops per step fewer than round 5; the
  // later thresholds only bound the literal pairs, which never changes a boundary the pass sees)
  uint32_t* const dummy = const_cast<uint32_t*>(L.scratch) + (tid_fresh() & 15);
  uint32_t* ckp = ck;  // checkpoint j (advanced, not multiplied out)
  const uint32_t* const cke = ck + NCK * ckstride;
  const uint32_t sEe = min(sE, endbits);  // one compare (one branch) for both ends
  bool stopped;
  for (;;) {
    const bool cross = p >= thr;
    const bool st = cross && ckp < cke;
    *(st ? ckp : dummy) = ((p - sB) << 16) | (uint32_t)cnt;
    ckp += st ? ckstride : 0;
    thr += cross ? CKI : 0u;
    // the exits only record why they left (the exit state is computed after the loop: no
    // exit-block work and fewer loop-carried copies per step)
    stopped = false;
    if (p >= sEe) break;
    stopped = true;
    if (dsym<SLOW>(r, W, L, p, min(thr, sEe), len, dist, lit2, m, e)) break;
    cnt += m ? (int32_t)len : (lit2 != 0xffffffffu ? 2 : 1);
    p = br_pos(r);
  }
  if (stopped) {
    len = stop_end(e, p);
    *Ep = (int32_t)(len != 0xffffffffu ? len : p);
    f = len != 0xffffffffu ? F_EOB : F_ERR;
  } else {
    *Ep = (int32_t)p;
    f = p >= sE ? F_EXIT : F_END;
  }
  *Bp = B;
  *cntp = cnt;
  return f;
}

// Re-decode of lane `lt` from its verified start s0 (a boundary >= sB).  At each checkpoint
// threshold the path is compared with the speculative one: the same boundary means the same
// decoder state, so the rest of the segment is the speculative run's (exit `se` = E << 3 | flag,
// `sc` bytes from its first boundary) and the decode stops there.
template <bool SLOW, class S, class LT>
DQ_AI int run_redo(const S& W, const LT& L, uint32_t s0, uint32_t sB,
                   uint32_t sE, uint32_t endbits, const uint32_t* ck, int ckstride, int32_t se,
                   int32_t sc, int32_t* Ep, int32_t* cntp, uint32_t CKI, int NCK, int* jm = nullptr) {
  BitR r;
  br_init(r, W, s0);
  int32_t cnt = 0;
  int f;
  uint32_t thr = ck ? sB + CKI : 0xffffffffu;
  uint32_t cur = ck ? ck[0] : 0xffffffffu;
  const uint32_t* ckq = ck;  // checkpoint j (the last one once j >= NCK)
  const uint32_t* const ckl = ck + (NCK - 1) * ckstride;
  const uint32_t sEe = min(sE, endbits);
  int j = 0;
  int why;  // 0: the segment or the data ended, 1: merged, 2: dsym stopped
  uint32_t p, len = 0, e = 0;
  for (;;) {
    p = br_pos(r);
    // at a checkpoint threshold: the same boundary as the speculative run merges (one exit branch
    // for the segment end, the data end and a merge; the threshold update is branch-free, and the
    // exit state is computed after the loop)
    const bool cross = p >= thr;
    const bool merge = cross && (cur >> 16) == p - sB;
    why = merge ? 1 : 0;
    if (p >= sEe || merge) break;
    const bool more = ckq < ckl;
    if (jm) j += cross ? 1 : 0;
    ckq += cross && more ? ckstride : 0;
    const uint32_t nxt = ck ? *ckq : 0xffffffffu;
    thr += cross ? CKI : 0u;  // past the last checkpoint: cur never merges again
    cur = cross ? (more ? nxt : 0xffffffffu) : cur;
    uint32_t dist = 0, lit2;
    bool m;
    why = 2;
    if (dsym<SLOW>(r, W, L, p, min(thr, sEe), len, dist, lit2, m, e)) break;
    cnt += m ? (int32_t)len : (lit2 != 0xffffffffu ? 2 : 1);
  }
  if (why == 1) {
    *Ep = se >> 3;
    f = se & 7;
    cnt += sc - (int32_t)(cur & 0xffffu);
    if (jm) *jm = j;
  } else if (why == 2) {
    len = stop_end(e, p);
    *Ep = (int32_t)(len != 0xffffffffu ? len : p);
    f = len != 0xffffffffu ? F_EOB : F_ERR;
  } else {
    *Ep = (int32_t)p;
    f = p >= sE ? F_EXIT : F_END;
  }
  *cntp = cnt;
  return f;
}

// Emit from the verified boundary `start` to the first boundary >= target, output starting at
// absolute position p; stops at isize.  Literals, literal pairs and match descriptors are written
// by the same three byte stores: a store a symbol does not need goes to this lane's dummy word
// (wsum / small are dead during emit), so literal and match lanes do not run separate branches.
// The image and the match-start bitmap start at absolute output position ibase (0 in the block
// kernel; the tail kernel's image holds only the bytes after the first deflate block).
template <bool SLOW, class S, class LT>
DQ_AI void emit_seg(const S& W, LT& L, uint32_t start, uint32_t target,
                    uint32_t endbits, int32_t p, int32_t isize, int sh, int32_t ibase = 0) {
  typedef volatile __attribute__((address_space(3))) uint8_t lds8;
  // three ds_write_b8 (a merged unaligned b16 store stalls): volatile keeps them apart, the LDS
  // address space keeps them DS stores (a generic volatile pointer became flat stores)
  uint32_t* const dummy32 = emit_dummy(L) + (tid_fresh() & 63);
  lds8* const dummy1 = (lds8*)dummy32 - 1;  // dummy1[1], dummy2[2]: the lane's dummy word
  lds8* const dummy2 = (lds8*)dummy32 - 2;
  BitR r;
  br_init(r, W, start);
  const uint32_t te = min(target, endbits);
  // the image position of output byte p is obase + p: the base in a VGPR (laundered), since the
  // kernel's SGPRs are all taken and a uniform base was spilled -- a v_readlane per step
  int32_t obase = sh - ibase;
  asm("" : "+v"(obase));
  bool bad = false;
  for (;;) {
    const uint32_t q = br_pos(r);
    if (q >= te || p >= isize) break;
    uint32_t len = 0, dist = 0, lit2;
    bool m;
    uint32_t e;
    const bool stop = dsym<SLOW>(r, W, L, q, te, len, dist, lit2, m, e);
    const bool far = m && (int32_t)dist > p;  // a distance before the block's first byte
    bad = far && !stop;
    if (stop || far) break;  // one exit branch: EOB / bad code (accounted for by the rounds) or far
    const bool two = !m && lit2 != 0xffffffffu && p + 1 < isize;
    DQ_CHK(p >= ibase && sh + p - ibase + 2 < (int)sizeof(L.out) &&
               ((p - ibase) >> 5) < (int)(sizeof(L.bm) / 4), CHK_K2_IMAGE);
    const uint32_t desc = (dist - 1) | ((len - 3) << 15);
    lds8* const o = (lds8*)(L.out + (obase + p));
    o[0] = (uint8_t)(m ? desc : len);
    // the stores a symbol does not need go to the dummy word: the base is selected and the +1 / +2
    // stays in the DS offset field (the dummy's base is moved back by the same amount)
    (m || two ? o : dummy1)[1] = (uint8_t)(m ? desc >> 8 : lit2);
    (m ? o : dummy2)[2] = (uint8_t)(desc >> 16);
    atomicOr(m ? &L.bm[(p - ibase) >> 5] : dummy32, 1u << ((p - ibase) & 31));
    p += m ? (int32_t)len : (two ? 2 : 1);
  }
  if (bad) set_err(L, ST_BAD_DIST);
}

__device__ inline uint32_t gf2_mulmod(uint32_t a, uint32_t b) {  // reflected, poly 0xEDB88320
  // branch-free: every lane holds its own constant a, so a data-dependent loop only diverges
  uint32_t p = 0;
#pragma unroll
  for (int i = 31; i >= 0; i--) {
    p ^= ((a >> i) & 1u) ? b : 0u;
    b = (b >> 1) ^ ((b & 1u) ? 0xEDB88320u : 0u);
  }
  return p;
}

// Inclusive wave scans by DPP (row_shr 1/2/4/8 inside rows of 16, then row_bcast 15/31 across
// rows): a few cycles per step instead of a ds_bpermute round trip.  All 64 lanes must be active.
DQ_AI int wave_incl_scan(int v, int) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);
  return v;
}
DQ_AI int wave_incl_or(int v) {
  v |= __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);
  v |= __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);
  v |= __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);
  v |= __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);
  v |= __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);
  v |= __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);
  return v;
}
DQ_AI uint32_t wave_incl_xor(uint32_t v) {
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);
  return v;
}
DQ_AI int wave_incl_max(int v) {  // values >= -1
  v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x111, 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x112, 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x114, 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x118, 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x142, 0xa, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x143, 0xc, 0xf, false));
  return v;
}
DQ_AI uint64_t lanes_below(int lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }

// Canonical description of one alphabet from the per-wave length counts, by one whole wave: lane
// l (1..15) sums its length's count over the waves, and two wave scans give the sorted-list offset
// (a sum of the counts below l) and the first code, code_l = sum_{k<l} cnt_k << (l - k), as
// (sum_{k<l} cnt_k << (16 - k)) >> (16 - l) -- exact: every term is a multiple of 2^(16-l).  The
// Kraft balance left_l = 2^l - (code_l + cnt_l) is the serial recurrence left = 2 left - cnt in
// closed form.  Also stores the number of codes no longer than the root (q0) and of all codes
// (qn).  Returns (in every lane) 0, or ST_BAD_TABLE for an over-subscribed or (except a single
// code) incomplete code.
template <int W0, int NW, int R>
DQ_AI int canon_from_counts(LdsI& L, HuffCanon& h, uint16_t* end, int32_t* q0p, int32_t* qnp) {
  const int l = tid_fresh() & 63;
  const bool in = l >= 1 && l <= 15;
  uint32_t pk = 0;  // 16-bit fields: no carries (<= 320 symbols)
#pragma unroll
  for (int w = W0; w < W0 + NW; w++) pk += in ? L.u.d.x.h.cntp[w][l >> 1] : 0u;
  const int c = in ? (int)((pk >> (16 * (l & 1))) & 0xffffu) : 0;
  const int offi = wave_incl_scan(c, l);          // codes of lengths <= l
  const int tt = in ? c << (16 - l) : 0;
  const int code = in ? (int)((uint32_t)(wave_incl_scan(tt, l) - tt) >> (16 - l)) : 0;
  const int left = in ? (1 << l) - (code + c) : 0;
  const uint64_t over = __ballot(in && left < 0);
  const uint64_t used = __ballot(c > 0);
  const int maxl = used ? 63 - __clzll(used) : 0;
  const int left15 = __builtin_amdgcn_readlane(left, 15);
  if (l < 16) {
    h.first[l] = (uint16_t)code;
    h.count[l] = (uint16_t)c;
    h.offs[l] = (uint16_t)(offi - c);
    if (in && l <= R) end[l] = (uint16_t)((code + c) << (R - l));
  }
  if (l == 0) {
    *q0p = __builtin_amdgcn_readlane(offi, R);
    *qnp = __builtin_amdgcn_readlane(offi, 15);
  }
  if (over) return ST_BAD_TABLE;
  if (maxl > 0 && left15 > 0 && maxl != 1) return ST_BAD_TABLE;  // zlib inflate_table rule
  return 0;
}

// Root table entry of bit-reversed (left-aligned) index r: the canonical ranges of lengths 1..R
// are consecutive in left-aligned order, so the length is 1 + the number of range ends <= r and
// the canonical position follows from the length's first code; 0 past the short codes (a long
// code's prefix, linked below, or no code).
template <int R, class LT>
DQ_AI uint16_t root_entry(const LT& L, const HuffCanon& h, const uint16_t* end,
                          const uint16_t* ent, uint32_t r) {
  int l = 1;
#pragma unroll
  for (int k = 1; k <= R; k++) l += (uint32_t)end[k] <= r ? 1 : 0;
  if (l > R) return 0;
  const int q = (int)h.offs[l] + (int)(r >> (R - l)) - (int)h.first[l];
  return ent[q];
}
// The range ends of the lengths 1..R in registers, for a loop of root_entry_r over many indices
// (root_entry re-reads them from LDS per index: the table stores in the loop may alias them).
template <int R>
struct RootEnds {
  uint32_t e[R + 1];
};
template <int R>
DQ_AI RootEnds<R> root_ends(const uint16_t* end) {
  RootEnds<R> x;
  x.e[0] = 0;
#pragma unroll
  for (int k = 1; k <= R; k++) x.e[k] = end[k];
  return x;
}
template <int R>
DQ_AI uint16_t root_entry_r(const HuffCanon& h, const RootEnds<R>& E, const uint16_t* ent, uint32_t r) {
  int l = 1;
#pragma unroll
  for (int k = 1; k <= R; k++) l += E.e[k] <= r ? 1 : 0;
  if (l > R) return 0;
  const int q = (int)h.offs[l] + (int)(r >> (R - l)) - (int)h.first[l];
  return ent[q];
}

// Entry t (< 128) of the code-length code's 7-bit decode table from the 19 code-length code
// lengths (sym << 3 | len, 0 = no code); *ok = false for an incomplete or over-subscribed code.
DQ_AI uint16_t clt_entry(const uint8_t* clen, int t, bool* okp) {
  uint8_t cl[19];
#pragma unroll
  for (int s = 0; s < 19; s++) cl[s] = clen[s];
  // length counts packed 8 bits per length: 0-3 in pk[0], 4-7 in pk[1]
  uint32_t pk[2] = {0u, 0u};
#pragma unroll
  for (int s = 0; s < 19; s++) {
    const uint32_t inc = 1u << (8 * (cl[s] & 3));
    pk[0] += cl[s] < 4 ? inc : 0u;
    pk[1] += cl[s] >= 4 ? inc : 0u;
  }
  // the codes of lengths 1..7 occupy consecutive left-aligned ranges: the length of index
  // rv is 1 + the number of range ends at or below it (as root_entry), its rank among that
  // length's codes follows from the length's first code
  int left = 1, code = 0, len = 1, first_l = 0;
  bool ok = true;
  const int rv = (int)bitrev((uint32_t)t, 7);
#pragma unroll
  for (int l = 1; l <= 7; l++) {
    const int c = (int)((pk[l >> 2] >> (8 * (l & 3))) & 0xffu);
    left = (left << 1) - c;
    ok = ok && left >= 0;
    first_l = len == l ? code : first_l;
    code += c;
    len += (code << (7 - l)) <= rv ? 1 : 0;  // end of the length-l range
    code <<= 1;
  }
  ok = ok && left == 0;  // the code-length code must be complete
  uint16_t ent = 0;
  if (len <= 7) {  // the k-th symbol of length len (one pass, no divergence over lengths)
    int k = (rv >> (7 - len)) - first_l, s2 = 0;
#pragma unroll
    for (int s = 0; s < 19; s++) {
      const bool is = cl[s] == len;
      s2 = is && k == 0 ? s : s2;
      k -= is ? 1 : 0;
    }
    ent = (uint16_t)((s2 << 3) | len);
  }
  *okp = ok;
  return ent;
}

// Build both decode tables from L.u.d.x.h.lens (all threads; barriers inside).
// Litlen symbols are handled by threads 0..319 (waves 0-4), distance symbols by wave 5.
DQ_AI void build_tables(LdsI& L, int nlen, int ndist) {
  const int t = tid_fresh(), lane = t & 63, wv = t >> 6;
  // second-level tables (the roots are written whole); their first entries are invalid-code
  // sentinels (code length 1), which a complete code's first table overwrites: only an incomplete
  // code (no long codes) has code-less root indices, and those read them (ll_second / d_second)
  for (int i = T_LSUB + t; i < T_DROOT; i += WG) L.u.d.T[i] = i == T_LSUB ? (uint16_t)(LL_BAD | 1u) : 0;
  for (int i = T_DSUB + t; i < T_END; i += WG) L.u.d.T[i] = i == T_DSUB ? (uint16_t)0x4001u : 0;
  const bool isl = t < 320, isd = t >= 320 && t < 352;
  const int sym = isl ? t : t - 320;
  const int len = isl ? (sym < nlen ? L.u.d.x.h.lens[sym] : 0)
                      : (isd && sym < ndist ? L.u.d.x.h.lens[288 + sym] : 0);
  // rank among equal lengths inside the wave: a wave scan of one-hot length counters packed
  // 8 bits per length in 4 registers (<= 64 per wave: no carries)
  int rank = 0;
  if (wv < 6) {
    uint32_t c[4];
#pragma unroll
    for (int j = 0; j < 4; j++)
      c[j] = (len >> 2) == j ? 1u << (8 * (len & 3)) : 0u;
#pragma unroll
    for (int j = 0; j < 4; j++) c[j] = (uint32_t)wave_incl_scan((int)c[j], lane);
    const uint32_t mine = (len >> 2) == 0 ? c[0] : (len >> 2) == 1 ? c[1] : (len >> 2) == 2 ? c[2] : c[3];
    rank = (int)((mine >> (8 * (len & 3))) & 0xffu) - 1;
    if (lane == 63)
#pragma unroll
      for (int j = 0; j < 8; j++)  // widened to 16 bits per length for the cross-wave sums
        L.u.d.x.h.cntp[wv][j] = ((c[j >> 1] >> (16 * (j & 1))) & 0xffu) |
                                (((c[j >> 1] >> (16 * (j & 1) + 8)) & 0xffu) << 16);
  }
  __syncthreads();
  if (wv == 0) {  // whole waves (DPP scans)
    const int e = canon_from_counts<0, 5, LR>(L, L.u.d.hl, L.u.d.lend, &L.misc[M_LQ0], &L.misc[M_LQN]);
    if (e && lane == 0) set_err(L, e);
  }
  if (wv == 5) {
    const int e = canon_from_counts<5, 1, DR>(L, L.u.d.hd, L.u.d.dend, &L.misc[M_DQ0], &L.misc[M_DQN]);
    if (e && lane == 0) set_err(L, e);
  }
  __syncthreads();
  if (L.misc[M_ERR]) return;
  const HuffCanon& H = isl ? L.u.d.hl : L.u.d.hd;
  const int R = isl ? LR : DR;
  int q = -1;  // canonical position
  uint32_t code = 0;
  if (len) {
    if (isl)
      for (int w = 0; w < wv; w++) rank += (int)((L.u.d.x.h.cntp[w][len >> 1] >> (16 * (len & 1))) & 0xffffu);
    code = H.first[len] + (uint32_t)rank;
    q = H.offs[len] + rank;
    const uint16_t ent = isl ? ent_ll((uint32_t)sym, (uint32_t)len) : ent_d((uint32_t)sym, (uint32_t)len);
    if (isl) L.u.d.lent[q] = ent;
    else L.u.d.dent[q] = ent;
    if (len > R) L.u.d.x.h.pref[(isl ? 0 : 288) + q] = (uint16_t)(code >> (len - R));
  }
  __syncthreads();
  // root tables, one entry per thread and index (no per-code replica loops)
  for (int i = t; i < (1 << LR); i += WG)
    L.u.d.T[i] = root_entry<LR>(L, L.u.d.hl, L.u.d.lend, L.u.d.lent, bitrev((uint32_t)i, LR));
  if (t < (1 << DR))
    L.u.d.T[T_DROOT + t] = root_entry<DR>(L, L.u.d.hd, L.u.d.dend, L.u.d.dent, bitrev((uint32_t)t, DR));
  // second-level tables: thread t handles canonical position t of each alphabet.  The long codes
  // under one root prefix are consecutive canonical positions (a group); a group's table has
  // 2^(longest length - R) entries, placed by a scan of the sizes (the link entries are written
  // after the barrier below, over the root entries above)
  {
    const int q0 = isl ? L.misc[M_LQ0] : L.misc[M_DQ0];
    const int qn = isl ? L.misc[M_LQN] : L.misc[M_DQN];
    const int base = isl ? 0 : 288;
    const bool lng = (isl || isd) && sym >= q0 && sym < qn;  // here `sym` = canonical position
    const uint16_t pf = lng ? L.u.d.x.h.pref[base + sym] : 0;
    const bool start = lng && (sym == q0 || L.u.d.x.h.pref[base + sym - 1] != pf);
    const bool gend = lng && (sym == qn - 1 || L.u.d.x.h.pref[base + sym + 1] != pf);
    const uint16_t ent = lng ? (isl ? L.u.d.lent[sym] : L.u.d.dent[sym]) : (uint16_t)0;
    const int cl = ent & 15;
    const int gsz = gend ? 1 << (cl - R) : 0;
    const uint64_t sm = __ballot(start);
    int slot = __popcll(sm & lanes_below(lane)) + (start ? 1 : 0);  // inclusive
    int osz = wave_incl_scan(gsz, lane);                              // inclusive
    if (lane == 63) {
      L.u.d.x.h.cntw[wv] = __popcll(sm);
      L.u.d.x.h.cnts[wv] = osz;
    }
    __syncthreads();
    if (isl)
      for (int w = 0; w < wv; w++) {
        slot += L.u.d.x.h.cntw[w];
        osz += L.u.d.x.h.cnts[w];
      }
    slot -= 1;
    const int R2 = isl ? LR : DR;
    const int area = isl ? LSLOTS << LSB : DSLOTS << DSB;
    const int gmax = isl ? MAXGRP : 32;
    uint32_t* const ginfo = L.u.d.x.h.ginfo + (isl ? 0 : MAXGRP);
    if (gend && slot < gmax) ginfo[slot] = (uint32_t)(osz - gsz) | (uint32_t)(cl - R2) << 16;
    __syncthreads();
    if (lng) {
      const uint32_t gi = slot < gmax ? ginfo[slot] : 0u;
      const int off = (int)(gi & 0xffffu), sb = (int)(gi >> 16);
      const bool fits = slot < gmax && off + (1 << sb) <= area;
      if (start) {
        const uint32_t ridx = bitrev(pf, R2) + (isl ? 0 : T_DROOT);
        L.u.d.T[ridx] = fits ? (uint16_t)(sb << 4 | off << 7) : E_SLOW;
        if (!fits) L.misc[M_SLOW] = 1;  // the decode passes take the canonical fallback
      }
      if (fits) {  // this canonical position's code into its group's table
        const uint32_t c = H.first[cl] + (uint32_t)(sym - H.offs[cl]);
        const int m = cl - R2;
        const uint32_t tail = bitrev(c & ((1u << m) - 1), m);
        uint16_t* sub = L.u.d.T + (isl ? T_LSUB : T_DSUB) + off;
        for (uint32_t k = 0; k < (1u << (sb - m)); k++) sub[tail | (k << m)] = ent;
      }
    }
  }
  __syncthreads();
}

// Dynamic header: decode the code-length sequence into L.u.d.x.h.lens, all eight waves at once.
// Returns the bit position after the header, or sets M_ERR.
// Wave w takes the 128-bit window w of a (128 * NWV)-bit pass: lane l decodes the symbol at offsets l and
// 64 + l of its window (entries e = l and 64 + l) and the window's successor table is doubled
// (successor^(2^b), b < 7, by lane shuffles of both halves).  A window's true path enters at one of
// its first 14 offsets (a code-length symbol is at most 7 + 7 bits), so each wave first maps every
// such entry to its exit into the next window; one thread chains the eight maps from the pass's
// start, and every wave then takes the path from its true entry: entry k of the window takes the
// k-th symbol of the path.  Repeat values are forward-filled by max-scans and runs placed by
// sum-scans, across windows through per-window totals (zero runs need no stores: the lengths are
// zero-filled).  Round 2 ran this serially over the windows in wave 0 (~25k cycles per header).
DQ_AI uint32_t read_lengths(LdsI& L, uint32_t P, int nlen, int ndist, uint32_t endbits, uint32_t hbase) {
  // the header's compressed words were staged in the (not yet built) decode table: HB_WORDS
  // words cover the longest possible header (17 + 57 + 320 * 14 bits)
  const uint32_t* hb = reinterpret_cast<const uint32_t*>(L.u.d.T);
  auto word = [&](uint32_t i) -> uint32_t { return hb[min(i - hbase, (uint32_t)HB_WORDS - 1)]; };
  auto& H = L.u.d.x.h;
  const int t = tid_fresh(), lane = t & 63, w = t >> 6;
  const int total = nlen + ndist;
  int have = 0, prev = -1;  // workgroup-uniform
  // successor^(2^b) of entry h * 64 + lane, 128 = past the window; a lookup of entry y
  auto look = [&](int v0, int v1, int y) -> int {
    const int a = __shfl(v0, y & 63, 64), c = __shfl(v1, y & 63, 64);
    return y >= 128 ? 128 : (y >= 64 ? c : a);
  };
  for (int pass = 0; pass < 8 && have < total; pass++) {
    if (P > endbits) {
      set_err(L, ST_OVERREAD);
      return P;
    }
    const uint32_t Wb = P + 128u * (uint32_t)w;
    const uint32_t wi = Wb >> 5, off = Wb & 31;
    const uint32_t k0 = (off + (uint32_t)lane) >> 5, sh = (off + (uint32_t)lane) & 31;
    uint32_t bits[2];
    bits[0] = __builtin_amdgcn_alignbit(word(wi + k0 + 1), word(wi + k0), sh);
    bits[1] = __builtin_amdgcn_alignbit(word(wi + k0 + 3), word(wi + k0 + 2), sh);
    int s[2], rep[2], adv[2], J[7][2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const uint32_t ent = H.clt[bits[h] & 127];
      const uint32_t cl = ent & 7, sy = ent >> 3;
      const uint32_t ex = sy == 16 ? 2u : sy == 17 ? 3u : sy == 18 ? 7u : 0u;
      const uint32_t xv = (bits[h] >> cl) & ((1u << ex) - 1);
      s[h] = (int)sy;
      rep[h] = sy < 16 ? 1 : sy == 16 ? 3 + (int)xv : sy == 17 ? 3 + (int)xv : 11 + (int)xv;
      adv[h] = cl ? (int)(cl + ex) : 0;
      const int e = lane + 64 * h;
      J[0][h] = adv[h] ? min(e + adv[h], 128) : e;  // an invalid code is a self-loop
    }
#pragma unroll
    for (int b = 1; b < 7; b++)
#pragma unroll
      for (int h = 0; h < 2; h++) J[b][h] = look(J[b - 1][0], J[b - 1][1], J[b - 1][h]);
    {  // exit of the path entered at offset `lane` (< 16): its last position inside the window
       // (largest jumps that stay inside), then that symbol's successor
      int x = lane & 15;
#pragma unroll
      for (int b = 6; b >= 0; b--) {
        const int y = look(J[b][0], J[b][1], x);
        x = y < 128 ? y : x;
      }
      const int ax = look(adv[0], adv[1], x);
      const int ex = ax ? x + ax - 128 : 255;  // 255: the path meets an invalid code
      if (lane < 16) H.exitm[w][lane] = (uint8_t)(ex >= 0 && ex < 16 ? ex : 255);
    }
    __syncthreads();
    if (t == 0) {
      int e = 0;
      for (int v = 0; v < NWV; v++) {
        H.ent[v] = e;
        e = e < 16 ? H.exitm[v][e] : 255;
      }
      H.ent[NWV] = e;
    }
    __syncthreads();
    const int entry = H.ent[w];
    // entry k = h * 64 + lane takes the k-th symbol of the path from `entry`
    uint32_t pm[4] = {0, 0, 0, 0};  // the path as a 128-bit mask
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int k = lane + 64 * h;
      int pk = entry < 128 ? entry : 128;
#pragma unroll
      for (int b = 0; b < 7; b++) {
        const int y = look(J[b][0], J[b][1], pk);
        if ((k >> b) & 1) pk = pk >= 128 ? 128 : y;
      }
#pragma unroll
      for (int q = 0; q < 4; q++) pm[q] |= (pk >> 5) == q ? 1u << (pk & 31) : 0u;
    }
#pragma unroll
    for (int q = 0; q < 4; q++) pm[q] = (uint32_t)__builtin_amdgcn_readlane(wave_incl_or((int)pm[q]), 63);
    bool onp[2];
    onp[0] = (lane < 32 ? pm[0] >> lane : pm[1] >> (lane - 32)) & 1;
    onp[1] = (lane < 32 ? pm[2] >> lane : pm[3] >> (lane - 32)) & 1;
    // lengths written by the path symbols before each entry; the last non-repeat value
    int rp[2], rinc[2];
    rp[0] = onp[0] ? rep[0] : 0;
    rp[1] = onp[1] ? rep[1] : 0;
    rinc[0] = wave_incl_scan(rp[0], lane);
    rinc[1] = wave_incl_scan(rp[1], lane) + __builtin_amdgcn_readlane(rinc[0], 63);
    const int v00 = s[0] < 16 ? s[0] : 0, v01 = s[1] < 16 ? s[1] : 0;
    const int key0 = wave_incl_max(onp[0] && s[0] != 16 ? ((lane + 1) << 5) | v00 : 0);
    const int key1 = max(wave_incl_max(onp[1] && s[1] != 16 ? ((lane + 65) << 5) | v01 : 0),
                         __builtin_amdgcn_readlane(key0, 63));
    if (lane == 63) {
      H.wt[w] = rinc[1];
      H.lv[w] = key1 > 0 ? (key1 & 31) : -1;
    }
    __syncthreads();
    int have_w = have, prev_w = prev, wsum = 0, lvall = prev;
    for (int v = 0; v < NWV; v++) {
      const int wt = H.wt[v], lv = H.lv[v];
      if (v < w) {
        have_w += wt;
        prev_w = lv >= 0 ? lv : prev_w;
      }
      wsum += wt;
      lvall = lv >= 0 ? lv : lvall;
    }
    // take path symbols while the lengths read so far are < total
    bool take[2];
    take[0] = onp[0] && have_w + rinc[0] - rp[0] < total;
    take[1] = onp[1] && have_w + rinc[1] - rp[1] < total;
    int val[2];
    val[0] = (take[0] && s[0] == 16) ? (key0 > 0 ? (key0 & 31) : prev_w) : v00;
    val[1] = (take[1] && s[1] == 16) ? (key1 > 0 ? (key1 & 31) : prev_w) : v01;
    if ((take[0] && (adv[0] == 0 || (s[0] == 16 && val[0] < 0))) ||
        (take[1] && (adv[1] == 0 || (s[1] == 16 && val[1] < 0))))
      set_err(L, ST_BAD_TABLE);
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int r = take[h] ? rep[h] : 0;
      if (take[h] && val[h] != 0) {  // lens is zero-filled: zero runs (up to 138) need no stores
        for (int i = have_w + rinc[h] - r; i < have_w + rinc[h] && i < total; i++)
          H.lens[i < nlen ? i : 288 + i - nlen] = (uint8_t)val[h];
      }
    }
    // the window where the lengths reach total publishes the header's end (and checks the last
    // symbol does not run past total)
    if (have_w < total && have_w + H.wt[w] >= total) {
      const uint64_t mark0 = __ballot(take[0]), mark1 = __ballot(take[1]);
      const int lastl = mark1 ? 64 + 63 - __clzll(mark1) : 63 - __clzll(mark0);
      const int ll = lastl & 63;
      const int cum = have_w + (lastl >= 64 ? __builtin_amdgcn_readlane(rinc[1], ll) : __builtin_amdgcn_readlane(rinc[0], ll));
      const int j = lastl + (lastl >= 64 ? __builtin_amdgcn_readlane(adv[1], ll) : __builtin_amdgcn_readlane(adv[0], ll));
      if (lane == 0) {
        if (cum > total) set_err(L, ST_BAD_TABLE);
        H.endp = (int32_t)(Wb + (uint32_t)j);
      }
    }
    have += wsum;
    prev = lvall;
    const uint32_t nextP = P + 128u * NWV + (uint32_t)H.ent[NWV];
    if (have < total && H.ent[NWV] >= 16) {  // the path met an invalid code before total
      set_err(L, ST_BAD_TABLE);
      return P;
    }
    __syncthreads();  // H.endp / lens visible; ent, wt, lv reused by the next pass
    if (L.misc[M_ERR]) return P;
    P = nextP;
  }
  if (have < total) {
    set_err(L, ST_BAD_TABLE);
    return P;
  }
  return (uint32_t)H.endp;
}

template <bool TIMING, int NB, int G>
__global__ __launch_bounds__(WG, WG / 128) void inflate_block_kernel(
    const uint8_t* __restrict__ C, const int64_t* __restrict__ blk_pos,
    const int32_t* __restrict__ blk_csize, const int32_t* __restrict__ blk_usize,
    const int64_t* __restrict__ uoff, int64_t nblk, uint8_t* __restrict__ U,
    int32_t* __restrict__ status, int32_t verify_crc, const uint32_t* __restrict__ crc_init,
    uint64_t* __restrict__ tim, uint32_t OV, uint32_t sflags, const int32_t* __restrict__ sel,
    TailDesc* __restrict__ tails) {
  // compile-time checkpoints (the spacing/count sweep's choice, profiles/r3ij_*): the decode loops
  // fold the threshold updates and hold fewer SGPRs (spec + rounds -8 k cycles per block, r3y)
  constexpr uint32_t CKI = CKI_DEFAULT;
  constexpr int NCK = NCK_DEFAULT;
  __shared__ LdsI L;
  // DQ_TIMING: thread 0 accumulates s_memtime cycles per phase (tim != nullptr only then)
  // [0..15] phases over the BGZF block; [16..21] phases 0-5 of its first deflate block; [22] the
  // number of deflate blocks
  uint64_t tacc[24] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t tlast = TIMING ? __builtin_amdgcn_s_memtime() : 0;
#define TST(i)                                            \
  do {                                                    \
    if (TIMING && threadIdx.x == 0) {                     \
      const uint64_t now_ = __builtin_amdgcn_s_memtime(); \
      tacc[i] += now_ - tlast;                            \
      tlast = now_;                                       \
    }                                                     \
  } while (0)
#define TCOUNT(i) do { if (TIMING && threadIdx.x == 0) tacc[i] += 1; } while (0)
  if ((int64_t)blockIdx.x >= nblk) return;
  // sel: the blocks to inflate (sparse runs: only the blocks an interval traversal needs)
  const int64_t b = sel ? (int64_t)sel[blockIdx.x] : (int64_t)blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t cpos = blk_pos[b];
  const int32_t csize = blk_csize[b];
  const int32_t isize = blk_usize[b];
  const int64_t ub = uoff[b];
  const int sh = (int)(ub & 15);
  // deflate data: bytes [cpos + 18, cpos + csize - 8); bit positions relative to the aligned base
  // (pointer arithmetic on C keeps the global address space: an integer round trip would turn
  // every load into a FLAT load, which the compiler must wait for with vmcnt(0) lgkmcnt(0))
  const uint8_t* dp = C + cpos + 18;
  const int mis = (int)(reinterpret_cast<uintptr_t>(dp) & 15);
  const uint32_t* W =
      reinterpret_cast<const uint32_t*>(__builtin_assume_aligned(dp - mis, 16));
  const uint32_t a0 = 8u * (uint32_t)mis;
  const int32_t dbytes = csize - 26;
  const uint32_t endbits = a0 + 8u * (uint32_t)max(dbytes, 0);

  // DQ_WARM (sflags bit 4): one load per 128-byte line of the deflate data, issued first and
  // waited for at the barrier below, so the speculative lanes' first reads hit L2 instead of each
  // taking an HBM round trip after the header
  uint32_t warm = 0;
  if ((sflags & 16) && 128u * (uint32_t)t < (uint32_t)(mis + max(dbytes, 0))) warm = W[32 * t];
  for (int i = t; i < 2048; i += WG) L.bm[i] = 0;
  if (t < 32) L.misc[t] = 0;
  if (t == 0) {
    if (isize < 0 || isize > 65536) L.misc[M_ERR] = ST_ISIZE;
    else if (dbytes < 0) L.misc[M_ERR] = ST_OVERREAD;
  }
  asm volatile("" ::"v"(warm));
  __syncthreads();
  int32_t produced = 0;
  uint32_t pos = a0;  // bit position of the next deflate block's header
  bool deferred = false;  // the rest of the block goes to the tail kernel
  while (L.misc[M_ERR] == 0 && produced < isize) {
    const int t = tid_fresh(), lane = t & 63, wv = t >> 6;
    // ---- 1. block header: every thread reads it (the branches below are uniform, no barrier).
    //      The dynamic header's staged words and code-length code lengths are loaded with it
    //      (their position follows from pos alone; C is padded, so a stored or fixed block near
    //      the end reads pad bytes it never uses).
    if (t == 0) L.misc[M_SLOW] = 0;  // read after build_tables' barriers; the last read of the
                                     // previous deflate block's flag precedes the emit barrier
    const uint32_t clpos = pos + 17;
    const uint32_t hbase = clpos >> 5;
    const uint32_t hw = t < HB_WORDS ? W[hbase + t] : 0u;
    const uint32_t hcl = t < 19 ? peek_bits(W, clpos + 3 * t, 3) : 0u;
    const uint32_t h = peek_bits(W, pos, 17);
    const int32_t bfinal = (int32_t)(h & 1), btype = (int32_t)((h >> 1) & 3);
    const int32_t herr = pos + 3 > endbits ? ST_OVERREAD : btype == 3 ? ST_BAD_BLOCKTYPE : 0;
    if (herr) {
      if (t == 0) L.misc[M_ERR] = herr;
      break;
    }
    if (btype == 0) {  // stored block: copy
      const uint32_t q = (pos + 3 + 7) & ~7u;  // byte boundary
      const uint8_t* bp = reinterpret_cast<const uint8_t*>(W) + q / 8;
      const uint32_t len = bp[0] | ((uint32_t)bp[1] << 8), nl = bp[2] | ((uint32_t)bp[3] << 8);
      const int32_t serr = (len ^ 0xffffu) != nl ? ST_BAD_STORED : q + 32 + 8 * len > endbits ? ST_OVERREAD : 0;
      if (serr) {
        if (t == 0) L.misc[M_ERR] = serr;
        break;
      }
      const uint8_t* sp = bp + 4;
      const int32_t n = min((int32_t)len, isize - produced);
      DQ_CHK(sh + produced + n <= OUTCAP, CHK_K2_IMAGE);
      for (int i = t; i < n; i += WG) L.out[sh + produced + i] = sp[i];
      produced += n;
      pos = q + 32 + 8 * len;
      __syncthreads();
      if (bfinal) break;
      continue;
    }
    const int nlen = btype == 1 ? 288 : (int)((h >> 3) & 31) + 257;
    const int ndist = btype == 1 ? 32 : (int)((h >> 8) & 31) + 1;
    if (btype == 2 && (nlen > 286 || ndist > 30)) {
      if (t == 0) L.misc[M_ERR] = ST_BAD_TABLE;
      break;
    }
    if (btype == 1) {
      for (int i = t; i < 320; i += WG) L.u.d.x.h.lens[i] = fixed_len(i);
      if (t == 0) L.misc[M_A] = (int32_t)(pos + 3);
      __syncthreads();
    } else {
      const int ncode = (int)((h >> 13) & 15) + 4;
      for (int i = t; i < 320; i += WG) L.u.d.x.h.lens[i] = 0;
      if (t < HB_WORDS) reinterpret_cast<uint32_t*>(L.u.d.T)[t] = hw;
      if (t < 19) L.u.d.x.h.clen[c_clorder3[t]] = t < ncode ? (uint8_t)hcl : 0;
      __syncthreads();
      // code-length code: 7-bit table, one entry per thread (canonical decode over 19 lengths)
      if (t < 128) {
        bool ok = true;
        L.u.d.x.h.clt[t] = clt_entry(L.u.d.x.h.clen, t, &ok);
        if (t == 0 && !ok) set_err(L, ST_BAD_TABLE);
      }
      __syncthreads();
      if (L.misc[M_ERR]) break;
      {
        const uint64_t tr0 = TIMING ? __builtin_amdgcn_s_memtime() : 0;
        const uint32_t a = read_lengths(L, clpos + 3 * (uint32_t)ncode, nlen, ndist, endbits, hbase);
        if (t == 0) L.misc[M_A] = (int32_t)a;
        if (TIMING && t == 0) tacc[8] += __builtin_amdgcn_s_memtime() - tr0;
      }
      __syncthreads();
      if (L.misc[M_ERR]) break;
      // an EOB code is required
      if (L.u.d.x.h.lens[256] == 0) {
        if (t == 0) L.misc[M_ERR] = ST_BAD_TABLE;
        break;
      }
    }
    TST(0);
    // ---- 2. tables
    build_tables(L, nlen, ndist);
    if (TIMING && t == 0) tacc[11] += __builtin_amdgcn_s_memtime() - tlast;  // without the pair table
    if (L.misc[M_ERR]) break;
    // pair table (the header scratch is dead): root index i whose literal leaves room for a
    // second whole literal code in the remaining root bits -- the root entry of i >> l1 (its
    // upper bits zero) is that literal iff its code fits them
    for (int i = t; i < (1 << LR); i += WG) {
      const uint32_t e1 = L.u.d.T[i];
      const uint32_t l1 = e1 & 15;
      uint16_t v = 0;
      if (l1 > 0 && !(e1 & 16) && l1 < (uint32_t)LR) {  // a literal code
        const uint32_t e2 = L.u.d.T[(uint32_t)i >> l1];
        const uint32_t l2 = e2 & 15;
        if (l2 > 0 && !(e2 & 16) && l1 + l2 <= (uint32_t)LR)
          v = (uint16_t)e2;
      }
      L.u.d.x.pair[i] = v;
    }
    __syncthreads();
    TST(1);
    const uint32_t a = (uint32_t)L.misc[M_A];
    const bool slow = L.misc[M_SLOW] != 0;  // uniform: the canonical fallback is rare
    if (a > endbits) {
      if (t == 0) L.misc[M_ERR] = ST_OVERREAD;
      break;
    }
    const uint32_t span = endbits - a;
    // per-lane arrays live in the not-yet-written tail of the output image
    const int ob = (sh + produced + 3) & ~3;
    const int cap = (sh + isize - ob) / (4 * (7 + NCK));  // NCK: this launch's checkpoints
    int32_t* AB;  // verified start (first boundary >= segment start), -1 none
    int32_t* AE;  // exit << 3 | flag
    int32_t* AC;  // output bytes in [B, E)
    int32_t* LS;  // redo list: lane
    int32_t* ST;  // redo list: start
    int32_t* SE;  // speculative exit << 3 | flag
    int32_t* SC;  // speculative byte count
    uint32_t* CK = nullptr;  // checkpoints, [j * nl + lane]
    // lanes: one per >= 128 bits, at most NDEC (tuning: sflags bits 8-17 cap the lanes, bits
    // 20-29 set the minimum segment bits)
    const uint32_t maxl = (sflags >> 8) & 1023u, minseg = (sflags >> 20) & 1023u;
    int nl = (int)max(1u, min(maxl ? maxl : (uint32_t)NDEC, span / (minseg ? minseg : 128u)));
    nl = cap >= 8 ? min(nl, cap) : min(nl, 8);  // a short image tail: at most 8 lanes, no checkpoints
    // segments of ceil(span / nl) bits; lanes whose segment would start past the data end (up to
    // nl - seg bits of rounding: their warm-up read words past the member) are not started
    const uint32_t seg = (span + nl - 1) / nl;
    if (seg) nl = (int)((span + seg - 1) / seg);
    AB = cap >= 8 ? reinterpret_cast<int32_t*>(L.out + ob) : L.small;
    AE = AB + nl;
    AC = AE + nl;
    LS = AC + nl;
    ST = LS + nl;
    SE = ST + nl;
    SC = SE + nl;
    if (cap >= 8) CK = reinterpret_cast<uint32_t*>(SC + nl);
    DQ_CHK(cap < 8 || (ob >= sh + produced && ob + 4 * nl * (7 + NCK) <= OUTCAP), CHK_K2_LANES);
#ifdef DQ_CHECKED
    GSrc gsrc{W, (endbits >> 5) + 8, 1u << 12};
#else
    const GSrc gsrc{W};
#endif
    // ---- 3. speculative pass: from OV bits before the segment, counting from its first boundary
    if (t == 0) {  // published by the barrier below
      L.misc[M_RCNT] = 0;       // round 0's redo-list counter
      L.misc[M_LAST] = nl - 1;  // the first lane that does not exit normally (atomicMin)
    }
    if (t < nl) {
      const uint32_t sB = a + (uint32_t)t * seg;
      const uint32_t start = t == 0 ? a : (sB > a + OV ? sB - OV : a);
      const uint32_t sE = t == nl - 1 ? 0xffffffffu : a + (uint32_t)(t + 1) * seg;
      int32_t B = -1, E = 0, c = 0;
      if (CK)
        for (int j = 0; j < NCK; j++) CK[j * nl + t] = 0xffffffffu;
      const int f = slow ? run_seg<true>(gsrc, L, start, sB, sE, endbits, &B, &E, &c,
                                         CK ? CK + t : nullptr, nl, CKI, NCK)
                         : run_seg<false>(gsrc, L, start, sB, sE, endbits, &B, &E, &c,
                                          CK ? CK + t : nullptr, nl, CKI, NCK);
      AB[t] = B;
      AE[t] = (E << 3) | f;
      AC[t] = c;
      SE[t] = (E << 3) | f;
      SC[t] = c;
    }
    __syncthreads();
    TST(2);
#ifdef DQ_CHECKED
    gsrc.tag = 2u << 12;
#endif
    // ---- 4. rounds: lanes whose first boundary differs from the predecessor's exit re-decode
    //      from that exit (compacted onto the first threads by an LDS counter, one barrier per
    //      round besides the re-decode's); repeat until consistent
    for (int round = 0; round <= nl; round++) {
      bool need = false;
      int32_t st = 0;
      if (t > 0 && t < nl) {
        const int32_t pe = AE[t - 1];
        st = pe >> 3;
        need = (pe & 7) == F_EXIT && AB[t] != st;
      }
      int32_t* rc = &L.misc[M_RCNT + (round & 1)];
      if (need) {
        const int r = atomicAdd(rc, 1);
        DQ_CHK(r < nl, CHK_K2_LANES);
        LS[r] = t;
        ST[r] = st;
      }
      if (t == 0) {  // the next round's counter; this round's changed-exit flag
        L.misc[M_RCNT + ((round + 1) & 1)] = 0;
        L.misc[M_DIRTY + (round & 1)] = 0;
      }
      __syncthreads();
      const int nneed = *rc;
      if (nneed == 0) break;
      TCOUNT(10);
      const bool hi = __builtin_amdgcn_readfirstlane(t) < __builtin_amdgcn_readfirstlane(nneed);  // the few waves re-decoding
      if (hi) __builtin_amdgcn_s_setprio(3);
      if (t < nneed) {
        const int lt = LS[t];
        const uint32_t s0 = (uint32_t)ST[t];
        const uint32_t sE = lt == nl - 1 ? 0xffffffffu : a + (uint32_t)(lt + 1) * seg;
        int32_t E = 0, c = 0;
        int jmerge = -1;
        const uint32_t sB = a + (uint32_t)lt * seg;
        // a speculative lane that found no boundary (F_DEAD) recorded no checkpoints
        const int f = slow ? run_redo<true>(gsrc, L, s0, sB, sE, endbits, CK ? CK + lt : nullptr,
                                            nl, SE[lt], SC[lt], &E, &c, CKI, NCK,
                                            TIMING ? &jmerge : nullptr)
                           : run_redo<false>(gsrc, L, s0, sB, sE, endbits, CK ? CK + lt : nullptr,
                                             nl, SE[lt], SC[lt], &E, &c, CKI, NCK,
                                             TIMING ? &jmerge : nullptr);
        const int32_t ae = (E << 3) | f;
        if (ae != AE[lt]) L.misc[M_DIRTY + (round & 1)] = 1;  // the successor's start moved
        AB[lt] = (int32_t)s0;
        AE[lt] = ae;
        AC[lt] = c;
        if (TIMING) {
          atomicAdd(&L.misc[21], 1);
          if (jmerge >= 0) {
            atomicAdd(&L.misc[23], 1);
            atomicAdd(&L.misc[24], jmerge);
          } else {
            const int sf = SE[lt] & 7;
            atomicAdd(&L.misc[sf == F_ERR || sf == F_EOB ? 25 : sf == F_EXIT ? 26 : 27], 1);
          }
        }
      }
      if (hi) __builtin_amdgcn_s_setprio(0);
      __syncthreads();
      // no re-decoded lane changed its exit: every successor's start still holds, so the
      // check of another round would find nothing to do (the slot is cleared again two rounds on)
      if (L.misc[M_DIRTY + (round & 1)] == 0) break;
    }
    TST(3);

    // ---- 5. counts -> offsets (the first non-exit lane ends the deflate block)
    int32_t myB = 0, myE = 0, myF = F_DEAD, myC = 0;
    if (t < nl) {
      myB = AB[t];
      myE = AE[t] >> 3;
      myF = AE[t] & 7;
      myC = AC[t];
    }
    if (t < nl && myF != F_EXIT) atomicMin(&L.misc[M_LAST], t);  // initialised with the spec pass
    __syncthreads();
    const int last = L.misc[M_LAST];
    const int32_t cv = t <= last ? myC : 0;
    const int32_t incl = wave_incl_scan(cv, lane);
    if (lane == 63) L.wsum[wv] = incl;
    if (t == last) {
      L.misc[M_NEXT] = myE;
      L.misc[M_LASTF] = myF;
    }
    __syncthreads();
    int32_t woff = 0;
    for (int w = 0; w < wv; w++) woff += L.wsum[w];
    const int32_t myoff = produced + woff + incl - cv;  // absolute output offset of lane t
    int32_t total = 0;
    for (int w = 0; w < WG / 64; w++) total += L.wsum[w];
    // ISIZE: the lane that reaches isize ends the stream (Inflater stops filling its buffer)
    const bool full = produced + total >= isize;
    const int32_t fl = L.misc[M_LASTF];
    if (!full && fl != F_EOB && t == 0) L.misc[M_ERR] = fl == F_ERR ? ST_BAD_CODE : ST_SHORT;
    __syncthreads();  // the arrays are dead from here: emit overwrites them
    TST(4);
    if (L.misc[M_ERR]) break;
    // ---- emit
#ifdef DQ_CHECKED
    gsrc.tag = 3u << 12;
#endif
    if (t <= last && myoff < isize) {
      const uint32_t sE = t == nl - 1 ? 0xffffffffu : a + (uint32_t)(t + 1) * seg;
      if (slow) emit_seg<true>(gsrc, L, (uint32_t)myB, sE, endbits, myoff, isize, sh);
      else emit_seg<false>(gsrc, L, (uint32_t)myB, sE, endbits, myoff, isize, sh);
    }
    const int32_t nextpos = L.misc[M_NEXT];
    __syncthreads();
    TST(5);
    produced = min(isize, produced + total);
    if (TIMING && t == 0) {
      if (tacc[22] == 0)
        for (int i = 0; i < 6; i++) tacc[16 + i] = tacc[i];
      tacc[22] += 1;
    }
    if (full || bfinal) break;
    pos = (uint32_t)nextpos;
    // the rest of the BGZF block is a small deflate block (htsjdk's level 5 closes one every 16,383
    // symbols: ~700 symbols left of a 65,498-byte block): hand it to the tail kernel, which decodes
    // many such tails per CU, one wave each, instead of running its fixed-latency phases here with
    // one wave busy (~23 % of this kernel's cycles for ~4 % of the symbols, round 3)
    if (tails && isize - produced <= TOUT && endbits - pos <= (uint32_t)TAIL_MAX_BITS) {
      deferred = true;
      break;
    }
  }
  __syncthreads();
  int32_t err = L.misc[M_ERR];
  if (!err && !deferred && produced != isize) err = ST_SHORT;
  // the bytes this workgroup resolves, stores and checksums: the whole block, or those before the
  // deferred tail
  const int32_t rsize = deferred ? produced : isize;
  if (deferred && t == 0) {
    TailDesc td;
    td.pos = (int32_t)pos;
    td.produced = produced;
    td.crc_raw = 0;
    td.flag = 1;
    tails[blockIdx.x] = td;
  }
  if (err) {
    if (t == 0) status[b] = err;
    return;
  }
  // ---- 6. resolve matches, chunk by chunk
  const uint64_t* bm64 = reinterpret_cast<const uint64_t*>(L.bm);
  {  // last_start: max-scan over 64-bit bitmap words (2 words per thread, threads >= 512 none)
    int ls[2];
    int run = -1;
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const uint64_t m = 2 * t + k < 1024 ? bm64[min(2 * t + k, 1023)] : 0ull;
      if (m) run = 64 * (2 * t + k) + 63 - __clzll(m);
      ls[k] = run;
    }
    const int wm = wave_incl_max(run);  // wave inclusive max-scan of the thread's last value
    if (lane == 63) L.wsum[wv] = wm;
    int ex = __shfl_up(wm, 1, 64);
    if (lane == 0) ex = -1;
    __syncthreads();
    for (int w = 0; w < wv; w++) ex = max(ex, L.wsum[w]);
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const int v = max(ex, ls[k]);
      if (WG == 512 || 2 * t + k < 1024) L.u.r.last_start[2 * t + k] = v < 0 ? (uint16_t)0xffff : (uint16_t)v;
    }
    __syncthreads();
  }
  uint8_t* dstU = U + ub;
  const uint8_t* O = L.out + sh;
  const int head = min((16 - sh) & 15, rsize);  // bytes before the first 16-byte U boundary
  int32_t lines_done = 0;                       // 16-byte lines [head + 16k, +16) stored
  // chunks of CH = G * WG bytes, thread t owns bytes [G t, G t + G) of each; NB chunks per batch;
  // a byte's chain may stop at any byte before its 512-byte step (the unit of the barriers in (b))
  constexpr int CH = G * WG;
  constexpr int BATCH = NB * CH;
  constexpr int NE = NB * G;
  // DQ_CSTEP: one step (and one barrier) per chunk of G * 512 bytes instead of per 512 bytes
  constexpr bool CSTEP = (DQ_CSTEP != 0 && G > 1) || CH % 512 != 0;
  static_assert(BATCH <= RES_NXT, "the batch's next-pointers fit the resolve scratch");
  static_assert((65536 + BATCH - 1) / BATCH <= NCARRY, "one carry slot per batch");
  uint16_t* nxt = L.u.r.nxt;
  // (a) sources of batch `b0`.  First hop, every byte: its owner (one 64-bit bitmap word, one
  //     last_start) and the owner's descriptor give the copy source (G <= 4 bytes have at most
  //     two owners: matches are >= 3 bytes long).  A source before the byte's 512-byte step is
  //     final (that step is complete when (b) reaches this one); so is a literal.  Every byte
  //     publishes its source in nxt.  The match straddling the batch start is the carry (cms,
  //     cdesc): its descriptor lies before the batch.
  auto first_hop = [&](int32_t b0, int32_t cms, uint32_t cdesc, int32_t* fr, int32_t* xs,
                       bool& pending) {
    pending = false;
    uint64_t mw[NB];
    int32_t lsv[NB];
#pragma unroll
    for (int k = 0; k < NB; k++) {
      const int32_t g0 = b0 + k * CH + G * t;
      const int w = min(g0 >> 6, 1023);  // bytes past rsize: read anything, copy = false
      DQ_CHK(w >= 0 && w - 1 < 1024, CHK_K2_LAST);
      mw[k] = bm64[w];
      lsv[k] = w ? (int32_t)zx16(L.u.r.last_start[w - 1]) : 0xffff;
    }
    int32_t msv[NE];
    uint32_t da[NB], db[NB];
#pragma unroll
    for (int k = 0; k < NB; k++) {
      const int32_t g0 = b0 + k * CH + G * t;
#pragma unroll
      for (int i = 0; i < G; i++) {
        const uint64_t mi = mw[k] & (~0ull >> (63 - ((g0 + i) & 63)));
        msv[k * G + i] = mi ? (g0 | 63) - (int32_t)__clzll(mi) : lsv[k];
      }
      // (an owner before the batch reads a stale descriptor, in range and unused: the carry's is
      // taken instead)
      da[k] = load_desc(L, sh + min(msv[k * G], 65535));
      db[k] = G > 1 ? load_desc(L, sh + min(msv[k * G + G - 1], 65535)) : da[k];
    }
#pragma unroll
    for (int k = 0; k < NB; k++) {
      const int32_t g0 = b0 + k * CH + G * t;
      const int32_t sbk = b0 + k * CH + (CSTEP ? 0 : ((G * t) & ~511));
#pragma unroll
      for (int i = 0; i < G; i++) {
        const int e = k * G + i;
        const int32_t x = g0 + i, ms = msv[e];
        const bool before = ms < b0;  // descriptors before the batch are overwritten: the carry
        const uint32_t desc = before ? cdesc : (ms == msv[k * G + G - 1] ? db[k] : da[k]);
        const int32_t len = (int32_t)(desc >> 15) + 3, D1 = (int32_t)(desc & 0x7fff);  // D - 1
        const bool copy = x < rsize && ms != 0xffff && (!before || ms == cms) && x < ms + len;
        // src = ms - D + (x - ms) mod D; x - ms <= 257: a float reciprocal + one fix-up is exact,
        // needed only by bytes past the first period of an overlapping match (skipped per wave);
        // otherwise src = x - D = (D1 ^ ~0) + x, one v_xad
        const int32_t jj = x - ms;
        int32_t src = (int32_t)((uint32_t)D1 ^ ~0u) + x;
        if (__builtin_expect(__any(copy && jj > D1), 0)) {
          const int32_t D = D1 + 1;
          const int32_t q = (int32_t)((float)jj * __builtin_amdgcn_rcpf((float)D));
          int32_t r = jj - q * D;
          r = r >= D ? r - D : r;
          src = ms - D + r;
        }
        DQ_CHK(!copy || (src >= 0 && src < x), CHK_K2_SRC);
        const bool done = !copy || src < sbk;
        fr[e] = copy ? src : x;
        xs[e] = done ? x : src;  // a final entry points at its own byte (see jump_round)
        pending = pending || !done;
        nxt[x - b0] = (uint16_t)(copy ? src : x);  // a final source (or the literal), else in-step
      }
    }
  };
  // Pointer jumping inside the byte's step: a pending byte reads nxt at its current source and
  // publishes how far it got, so a byte that reads an advanced pointer skips that byte's chain.
  // Every value read is a byte of the same chain, so no barrier orders the rounds and each read
  // advances at least one hop; it ends at a literal (nxt[p] == p) or a byte before the step.
  auto jump_round = [&](int32_t b0, int32_t* fr, int32_t* xs, bool& pending) {
    // branch-free over the entries: a final entry points at its own byte (xs == own), so it
    // re-reads and re-writes its own next pointer, which holds its final source already -- the
    // pending state is the pointer itself (round 5 kept a bit per entry: an extract, a select of
    // the read address and a bit update per entry and round)
    int32_t qv[NE];
#pragma unroll
    for (int e = 0; e < NE; e++) {
      DQ_CHK(xs[e] - b0 >= 0 && xs[e] - b0 < BATCH, CHK_K2_NXT);
      qv[e] = (int32_t)zx16(nxt[xs[e] - b0]);
    }
    bool any = false;
#pragma unroll
    for (int e = 0; e < NE; e++) {
      const int32_t own = (e / G) * CH + G * t + e % G;  // relative to b0
      const int32_t p = xs[e], q = qv[e];
      const bool pd = p != b0 + own;
      const int32_t sbk = b0 + (e / G) * CH + (CSTEP ? 0 : ((G * t) & ~511));
      const bool fin = pd && (q == p || q < sbk);
      const bool go = pd && !fin;
      fr[e] = fin ? q : fr[e];
      xs[e] = go ? q : b0 + own;
      any = any || go;
      nxt[own] = (uint16_t)q;
    }
    pending = any;
  };
  // Software pipeline over batches: while batch k's ordered steps (b) run, batch k+1 takes its
  // first hop (its descriptors are intact until its own steps) and one jump round after each
  // step barrier (nxt holds batch k+1 only: batch k's sources are final in registers by then).
  int32_t frA[NE], xsA[NE];
  bool pendA = false;
  int32_t cms = -1;     // carry into the current batch
  uint32_t cdesc = 0;
  first_hop(0, cms, cdesc, frA, xsA, pendA);
  // the carries into every batch, while every descriptor is intact (off the batches' critical
  // path: round 2 had wave 0 compute each one in front of the batch barrier)
  if (t < (rsize + BATCH - 1) / BATCH) {
    int32_t ncms = -1;
    uint32_t ncdesc = 0;
    const int32_t x = (t + 1) * BATCH - 1;  // batch t's last byte
    if (x + 1 < rsize) {
      const uint64_t m = bm64[x >> 6];  // bit 63 of the last word: every bit is at or before x
      const int32_t ms = m ? (x | 63) - (int32_t)__clzll(m) : (int32_t)L.u.r.last_start[(x >> 6) - 1];
      if (ms != 0xffff) {
        const uint32_t desc = load_desc(L, sh + ms);
        if (ms + (int32_t)(desc >> 15) + 3 > x + 1) {
          ncms = ms;
          ncdesc = desc;
        }
      }
    }
    L.u.r.carry_ms[t] = ncms;
    L.u.r.carry_desc[t] = ncdesc;
  }
  __syncthreads();
  for (int hop = 0; pendA && hop < WG + 2; hop++) jump_round(0, frA, xsA, pendA);
  for (int32_t bs = 0; bs < rsize; bs += BATCH) {
    const uint64_t tb0 = TIMING ? __builtin_amdgcn_s_memtime() : 0;
    const int32_t nbs = bs + BATCH;
    const bool more = nbs < rsize;
    __syncthreads();  // every wave's jumps of batch k are done: nxt is free for batch k+1
    const int32_t ncms = more ? L.u.r.carry_ms[bs / BATCH] : -1;
    const uint32_t ncdesc = more ? L.u.r.carry_desc[bs / BATCH] : 0u;
    int32_t frB[NE], xsB[NE];
    bool pendB = false;
    if (more) first_hop(nbs, ncms, ncdesc, frB, xsB, pendB);
    const uint64_t tb1 = TIMING ? __builtin_amdgcn_s_memtime() : 0;
    // (b) batch k's 512-byte steps in order: one LDS read + write per copied byte, one barrier.
    //     A step's reads are issued before the next batch's jump round that follows the previous
    //     barrier, so their latency overlaps it.
#pragma unroll
    for (int k = 0; k < NB; k++) {
#pragma unroll
      for (int j = 0; j < (CSTEP ? 1 : G); j++) {
        const bool mine = CSTEP || ((G * t) >> 9) == j;
        const int32_t g0 = bs + k * CH + G * t;
        uint8_t v[G];
        if (mine)
#pragma unroll
          for (int i = 0; i < G; i++) {
            DQ_CHK(g0 + i >= rsize || (frA[k * G + i] >= 0 && frA[k * G + i] <= g0 + i), CHK_K2_SRC);
            v[i] = O[min(frA[k * G + i], 65535)];
          }
        if ((k > 0 || j > 0) && pendB) jump_round(nbs, frB, xsB, pendB);
        if (mine)
#pragma unroll
          for (int i = 0; i < G; i++)
            if (g0 + i < rsize) L.out[sh + g0 + i] = v[i];  // a literal rewrites its own value
        __syncthreads();
      }
    }
    if (pendB) jump_round(nbs, frB, xsB, pendB);
    const uint64_t tb2 = TIMING ? __builtin_amdgcn_s_memtime() : 0;
    // (c) store the 16-byte U lines this batch completed
    const int32_t c1 = min(rsize, nbs);
    const int32_t lines_to = c1 >= head ? (c1 - head) / 16 : 0;
    if (!(sflags & 1)) {
      for (int32_t k = lines_done + t; k < lines_to; k += WG) {
        const uint4 v = *reinterpret_cast<const uint4*>(O + head + 16 * k);
        uint4* d = reinterpret_cast<uint4*>(dstU + head + 16 * k);
        if (sflags & 2) st_nt(d, v);
        else *d = v;
      }
      lines_done = lines_to;
    }
    const uint64_t tb3 = TIMING ? __builtin_amdgcn_s_memtime() : 0;
    for (int hop = 0; pendB && hop < WG + 2; hop++) jump_round(nbs, frB, xsB, pendB);
#pragma unroll
    for (int e = 0; e < NE; e++) frA[e] = frB[e];
    cms = ncms;
    cdesc = ncdesc;
    if (TIMING && t == 0) {
      tacc[9] += tb1 - tb0;   // carry + barrier + first hop of the next batch
      tacc[12] += tb2 - tb1;  // (b) the ordered steps with the next batch's jump rounds
      tacc[13] += tb3 - tb2;  // (c) issuing the U stores
      tacc[14] += __builtin_amdgcn_s_memtime() - tb3;  // the rest of wave 0's jumps
      tacc[15] += 1;
    }
  }
  if (sflags & 1) {  // the whole block at the end
    const int32_t lines_to = rsize >= head ? (rsize - head) / 16 : 0;
    for (int32_t k = t; k < lines_to; k += WG) {
      const uint4 v = *reinterpret_cast<const uint4*>(O + head + 16 * k);
      uint4* d = reinterpret_cast<uint4*>(dstU + head + 16 * k);
      if (sflags & 2) st_nt(d, v);
      else *d = v;
    }
    lines_done = lines_to;
  }
  // the CRC's constants, loaded ahead of the U tail stores and the barrier below (their latency
  // overlaps them): this thread's two table words, its slice's shift, and for thread 0 the
  // initial-value term and the gzip trailer
  uint32_t ct0 = 0, ct1 = 0, cshift = 0, cinit = 0, cwant = 0;
  if (verify_crc) {
    ct0 = (&c_crc4[0][0])[t];
    ct1 = t + WG < 1024 ? (&c_crc4[0][0])[t + WG] : 0u;
    cshift = c_slice_shift[WG - 1 - t];
    if (t == 0) {
      cinit = crc_init[rsize];  // x^(8 rsize) * 0xffffffff mod P
      const uint8_t* tr = C + cpos + csize - 8;
      cwant = (uint32_t)tr[0] | ((uint32_t)tr[1] << 8) | ((uint32_t)tr[2] << 16) | ((uint32_t)tr[3] << 24);
    }
  }
  static_assert(2 * WG >= 1024, "at most two CRC table words per thread");
  for (int x = t; x < head; x += WG) dstU[x] = O[x];
  for (int x = head + 16 * lines_done + t; x < rsize; x += WG) dstU[x] = O[x];
  TST(6);
  // ---- 7. CRC32: thread t hashes the CRC_SL-byte slice ending (511 - t) * CRC_SL bytes before rsize
  if (verify_crc) {
    __syncthreads();  // the resolve scratch is dead: the CRC tables reuse it
    if (t < 1024) (&L.u.crc4[0][0])[t] = ct0;
    if (t + WG < 1024) (&L.u.crc4[0][0])[t + WG] = ct1;
    __syncthreads();
    const int32_t e = rsize - (WG - 1 - t) * CRC_SL;
    const int32_t s0 = max(0, e - CRC_SL);
    uint32_t cr = 0;
    if (e > 0) {
      int32_t x = s0;
      while (x < e && ((sh + x) & 3)) cr = L.u.crc4[0][(cr ^ O[x++]) & 0xff] ^ (cr >> 8);
      for (; x + 4 <= e; x += 4) {
        const uint32_t v = cr ^ *reinterpret_cast<const uint32_t*>(O + x);
        cr = L.u.crc4[3][v & 0xff] ^ L.u.crc4[2][(v >> 8) & 0xff] ^ L.u.crc4[1][(v >> 16) & 0xff] ^
             L.u.crc4[0][v >> 24];
      }
      while (x < e) cr = L.u.crc4[0][(cr ^ O[x++]) & 0xff] ^ (cr >> 8);
      cr = gf2_mulmod(cshift, cr);
    }
    cr = wave_incl_xor(cr);  // DPP: lane 63 holds the wave's xor
    if (lane == 63) L.wsum[wv] = (int32_t)cr;
    __syncthreads();
    if (t == 0) {
      uint32_t x = 0;
      for (int w = 0; w < WG / 64; w++) x ^= (uint32_t)L.wsum[w];
      if (deferred) {  // the prefix's CRC register; the tail kernel finishes the block's CRC
        tails[blockIdx.x].crc_raw = x;
      } else {
        const uint32_t crc = (x ^ cinit) ^ 0xffffffffu;
        if (crc != cwant) status[b] = ST_CRC;
      }
    }
  }
  TST(7);
  if (TIMING && t == 0)
    for (int i = 0; i < 24; i++) tim[(int64_t)blockIdx.x * TIM_W + i] = tacc[i];
  if (TIMING && t == 0)  // [24..30] the rounds' re-decodes: lanes, merges, checkpoint sum, non-merges
    for (int i = 0; i < 7; i++) tim[(int64_t)blockIdx.x * TIM_W + 24 + i] = (uint64_t)L.misc[21 + i];
}

// ================================================================ the tail kernel
// Per-wave LDS of inflate_tail_kernel (~13 KB: four tails per workgroup, three workgroups per CU).
struct alignas(16) LdsW {
  // root tables only: a tail's codes longer than the roots take the canonical path (E_SLOW), and
  // code-less root indices hold invalid-code entries (build_tables_wave), so the second-level
  // areas are never read (their offsets point into the litlen root only to stay in bounds)
  static constexpr int kLSUB = 0, kDROOT = 1 << LR, kDSUB = 0, kTEND = (1 << LR) + (1 << DR);
  // no literal-pair table: with it a tail takes 11.3 KB and four 4-wave workgroups do not fit a CU
  static constexpr bool kPair = false;
  union {
    struct {
      uint16_t T[kTEND];
      HuffCanon hl, hd;
      uint16_t lend[16], dend[16];
      uint16_t lent[288];
      uint16_t dent[32];
      union {
        struct {
          uint8_t lens[320];
          uint8_t clen[20];
          uint16_t clt[128];
          int32_t cnt[32];  // code-length counts: litlen [0, 16), distance [16, 32)
          int32_t run[32];  // ranks so far per length over the symbol chunks (same split)
        } h;
      } x;
    } d;
    uint32_t crc4[4][256];        // CRC: the slice-by-4 tables
  } u;
  alignas(16) uint8_t out[TOUT + 32]; // the tail's output image: tail byte k at out[sh + k]
  alignas(8) uint32_t bm[TOUT / 32];  // match-start bitmap of the tail (bit k: tail byte k)
  uint32_t ck[T_NCK * 64];            // checkpoints [j * 64 + lane]; emit's dummy words; the
                                      // resolve's next pointers (256 x 16 bits)
  int32_t misc[8];
  uint32_t scratch[16];               // run_seg's dummy words
};
static_assert(HB_WORDS * 4 <= LdsW::kTEND * 2, "header staging fits the decode table");
static_assert(4 * 4 * sizeof(LdsW) <= 160 * 1024, "four tails per workgroup, four workgroups per CU");
DQ_AI uint32_t* emit_dummy(LdsW& L) { return L.ck; }

// The code-length sequence of a dynamic header, decoded by one wave, 64 bits at a time: lane i
// decodes the code-length symbol at bit i of the window, the window's successor table is doubled
// by shuffles, lane k finds the k-th symbol of the path from the window's entry (carried from the
// previous window), repeat values are forward-filled by a max-scan and runs placed by a sum-scan.
// The header's words are staged in the decode table (not built yet).  Returns the bit position
// after the header, or sets M_ERR.
DQ_AI uint32_t read_lengths_wave(LdsW& L, uint32_t P, int nlen, int ndist, uint32_t endbits,
                                 uint32_t hbase) {
  const uint32_t* hb = reinterpret_cast<const uint32_t*>(L.u.d.T);
  auto& H = L.u.d.x.h;
  const int lane = tid_fresh() & 63;
  const int total = nlen + ndist;
  int have = 0, prev = -1, entry = 0;  // uniform
  for (uint32_t W0 = P;; W0 += 64) {
    if (W0 > endbits) {
      set_err(L, ST_OVERREAD);
      return W0;
    }
    const uint32_t p = W0 + (uint32_t)lane;
    const uint32_t wi = min((p >> 5) - hbase, (uint32_t)HB_WORDS - 2);
    const uint32_t v = (uint32_t)((((uint64_t)hb[wi + 1] << 32) | hb[wi]) >> (p & 31));
    const uint32_t ent = H.clt[v & 127];
    const uint32_t cl = ent & 7, sy = ent >> 3;
    const uint32_t ex = sy == 16 ? 2u : sy == 17 ? 3u : sy == 18 ? 7u : 0u;
    const int xv = (int)((v >> cl) & ((1u << ex) - 1));
    const int rep = sy < 16 ? 1 : sy == 16 ? 3 + xv : sy == 17 ? 3 + xv : 11 + xv;
    const int adv = cl ? (int)(cl + ex) : 0;  // 0: no code (a path reaching it stops)
    // successor^(2^b), 64 = past the window; an invalid code is a self-loop.  (Computing the next
    // window's table while this window's path is taken measured no faster, profiles/r6g_*: the
    // shuffles' results return in order, so the path waits for the prefetched ones too.)
    int J[6];
    J[0] = adv ? min(lane + adv, 64) : lane;
#pragma unroll
    for (int k = 1; k < 6; k++) {
      const int y = __shfl(J[k - 1], J[k - 1] & 63, 64);
      J[k] = J[k - 1] >= 64 ? 64 : y;
    }
    // lane k: offset of the k-th path symbol from `entry` (64: none)
    int pk = entry;
#pragma unroll
    for (int k = 0; k < 6; k++) {
      const int y = __shfl(J[k], pk & 63, 64);
      if ((lane >> k) & 1) pk = pk >= 64 ? 64 : y;
    }
    const bool onp = pk < 64;
    const int src = pk & 63;
    const int s_rep = __shfl(rep, src, 64), s_adv = __shfl(adv, src, 64);
    const int s_sy = __shfl((int)sy, src, 64);
    // a path stuck at an invalid code repeats one offset: only its first occurrence counts
    const int pprev = __shfl_up(pk, 1, 64);
    const bool real = onp && (lane == 0 || pprev != pk);
    const bool bad = real && s_adv == 0;
    const int r = real && !bad ? s_rep : 0;
    const int incl = wave_incl_scan(r, lane);
    // the value: a literal length, 0 for 17/18, else the last non-repeat value before it
    const int key = wave_incl_max(real && !bad && s_sy != 16 ? ((lane + 1) << 5) | (s_sy < 16 ? s_sy : 0) : 0);
    const int kprev = __shfl_up(key, 1, 64);
    const int before = lane == 0 ? 0 : kprev;
    const int val = s_sy < 16 ? s_sy : s_sy == 16 ? (before > 0 ? (before & 31) : prev) : 0;
    // symbols whose run starts before `total`; the one that reaches it ends the header
    const bool take = real && have + incl - r < total;
    if (__any((take && bad) || (take && s_sy == 16 && val < 0) || (take && have + incl > total))) {
      set_err(L, ST_BAD_TABLE);
      return W0;
    }
    if (take && val != 0)  // lens is zero-filled: zero runs need no stores
      for (int i = have + incl - r; i < have + incl; i++) H.lens[i < nlen ? i : 288 + i - nlen] = (uint8_t)val;
    const uint64_t tk = __ballot(take);
    const int lastk = tk ? 63 - (int)__clzll(tk) : -1;
    if (lastk >= 0 && __shfl(have + incl, lastk, 64) >= total) {  // the header ends in this window
      __builtin_amdgcn_wave_barrier();
      return W0 + (uint32_t)__shfl(pk + s_adv, lastk, 64);
    }
    // carry into the next window: the lengths written, the last value, the path's exit
    const uint64_t rm = __ballot(real);
    const int lastr = rm ? 63 - (int)__clzll(rm) : -1;
    if (lastr < 0 || __shfl((int)bad, lastr, 64)) {  // no path symbol / stuck at an invalid code
      set_err(L, ST_BAD_TABLE);
      return W0;
    }
    have = __shfl(have + incl, lastr, 64);
    const int kl = __shfl(key, 63, 64);
    prev = kl > 0 ? (kl & 31) : prev;
    entry = __shfl(pk + s_adv, lastr, 64) - 64;
  }
}

// The decode tables by one wave: root tables as the block kernel's (entries carry the decoded
// values), and the canonical slow path (E_SLOW) for every root prefix of a longer code -- a tail
// decodes ~700 symbols, so the second-level tables are not worth their build.  Sets M_SLOW.
DQ_AI void build_tables_wave(LdsW& L, int nlen, int ndist) {
  const int lane = tid_fresh() & 63;
  auto& H = L.u.d.x.h;
  if (lane < 32) {
    H.cnt[lane] = 0;
    H.run[lane] = 0;
  }
  __builtin_amdgcn_wave_barrier();
  // code-length counts of both alphabets (LDS atomics: one pass over the symbols)
  for (int k = lane; k < 320; k += 64) {
    const bool isl = k < 288;
    const int len = isl ? (k < nlen ? H.lens[k] : 0) : (k - 288 < ndist ? H.lens[k] : 0);
    if (len) atomicAdd(&H.cnt[(isl ? 0 : 16) + len], 1);
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  // canonical descriptions (lanes 1..15: litlen; 17..31: distance), as canon_from_counts
  int e = 0;
  {
    const int l = lane & 15;
    const bool in = lane < 32 && l >= 1;
    const int c = in ? H.cnt[lane] : 0;
    // segmented inclusive scans: the distance half (lanes 16..31) starts from zero
    int offi = wave_incl_scan(c, lane);
    const int tt = in ? c << (16 - l) : 0;
    int cs = wave_incl_scan(tt, lane);
    const int base_o = __shfl(offi, 15, 64), base_c = __shfl(cs, 15, 64);
    if (lane >= 16) {
      offi -= base_o;
      cs -= base_c;
    }
    const int code = in ? (int)((uint32_t)(cs - tt) >> (16 - l)) : 0;
    const int left = in ? (1 << l) - (code + c) : 0;
    const bool isd = lane >= 16;
    HuffCanon& h = isd ? L.u.d.hd : L.u.d.hl;
    uint16_t* end = isd ? L.u.d.dend : L.u.d.lend;
    const int R = isd ? DR : LR;
    if (lane < 32) {
      h.first[l] = (uint16_t)code;
      h.count[l] = (uint16_t)c;
      h.offs[l] = (uint16_t)(offi - c);
      if (in && l <= R) end[l] = (uint16_t)((code + c) << (R - l));
    }
    const uint64_t over = __ballot(in && left < 0);
    const uint64_t used = __ballot(c > 0);
    const int left15l = __shfl(left, 15, 64), left15d = __shfl(left, 31, 64);
    const uint64_t ul = used & 0xffffull, ud = (used >> 16) & 0xffffull;
    const int maxll = ul ? 63 - __clzll(ul) : 0, maxld = ud ? 63 - __clzll(ud) : 0;
    if (over) e = ST_BAD_TABLE;
    if (maxll > 0 && left15l > 0 && maxll != 1) e = ST_BAD_TABLE;  // zlib inflate_table rule
    if (maxld > 0 && left15d > 0 && maxld != 1) e = ST_BAD_TABLE;
    // codes no longer than the roots, all codes (the long ones take the canonical slow path)
    const int ql0 = __shfl(offi, LR, 64), qln = __shfl(offi, 15, 64);
    const int qd0 = __shfl(offi, 16 + DR, 64), qdn = __shfl(offi, 31, 64);
    if (lane == 0) L.misc[M_SLOW] = (qln > ql0 || qdn > qd0) ? 1 : 0;
  }
  if (e) {
    if (lane == 0) set_err(L, e);
    return;
  }
  __builtin_amdgcn_wave_barrier();
  // ranks among equal lengths, chunk by chunk: the lanes with the same key (alphabet, length) are
  // found by five ballots on the key's bits, a symbol's rank is the number of those peers below it
  // plus the key's running count over the earlier chunks, and the key's highest lane advances that
  // count (deterministic: round 5 took the rank from one LDS atomic add per symbol, which relied on
  // gfx950 returning the values of same-address lanes in lane order -- observed, not documented)
  const uint64_t below = lanes_below(lane);
  for (int k0 = 0; k0 < 320; k0 += 64) {
    const int k = k0 + lane;
    const bool isl = k < 288;
    const int sym = isl ? k : k - 288;
    const int len = k < 320 ? (isl ? (k < nlen ? H.lens[k] : 0) : (sym < ndist ? H.lens[k] : 0)) : 0;
    const int key = (isl ? 0 : 16) + len;  // 5 bits
    uint64_t peers = ~0ull;
#pragma unroll
    for (int bt = 0; bt < 5; bt++) {
      const uint64_t bl = __ballot((key >> bt) & 1);
      peers &= ((key >> bt) & 1) ? bl : ~bl;
    }
    const int run0 = H.run[key];
    const int rank = run0 + __popcll(peers & below);
    __builtin_amdgcn_wave_barrier();  // every lane has read its count before the updates
    if (len && (peers >> lane) == 1ull) H.run[key] = run0 + __popcll(peers);  // the key's last lane
    if (len) {
      const HuffCanon& hh = isl ? L.u.d.hl : L.u.d.hd;
      const int q = hh.offs[len] + rank;
      if (isl) L.u.d.lent[q] = ent_ll((uint32_t)sym, (uint32_t)len);
      else L.u.d.dent[q] = ent_d((uint32_t)sym, (uint32_t)len);
    }
    __builtin_amdgcn_wave_barrier();
  }
  __builtin_amdgcn_wave_barrier();
  // root tables: 16 litlen and 4 distance entries per lane; an index without a short code is the
  // prefix of long codes (a complete code), decoded canonically
  const bool lslow = L.u.d.hl.count[11] + L.u.d.hl.count[12] + L.u.d.hl.count[13] +
                         L.u.d.hl.count[14] + L.u.d.hl.count[15] > 0;
  const bool dslow = L.u.d.hd.count[9] + L.u.d.hd.count[10] + L.u.d.hd.count[11] + L.u.d.hd.count[12] +
                         L.u.d.hd.count[13] + L.u.d.hd.count[14] + L.u.d.hd.count[15] > 0;
  // (an index with no code in an incomplete code -- zlib allows one code of length 1 -- gets an
  // invalid-code entry of length 1: decoding it stops the run, as zlib's "invalid code")
#if DQ_ROOT_REG
  const RootEnds<LR> le = root_ends<LR>(L.u.d.lend);
  const RootEnds<DR> de = root_ends<DR>(L.u.d.dend);
#endif
  for (int i = lane; i < (1 << LR); i += 64) {
#if DQ_ROOT_REG
    const uint16_t v = root_entry_r<LR>(L.u.d.hl, le, L.u.d.lent, bitrev((uint32_t)i, LR));
#else
    const uint16_t v = root_entry<LR>(L, L.u.d.hl, L.u.d.lend, L.u.d.lent, bitrev((uint32_t)i, LR));
#endif
    L.u.d.T[i] = v ? v : lslow ? E_SLOW : (uint16_t)(LL_BAD | 1u);
  }
  for (int i = lane; i < (1 << DR); i += 64) {
#if DQ_ROOT_REG
    const uint16_t v = root_entry_r<DR>(L.u.d.hd, de, L.u.d.dent, bitrev((uint32_t)i, DR));
#else
    const uint16_t v = root_entry<DR>(L, L.u.d.hd, L.u.d.dend, L.u.d.dent, bitrev((uint32_t)i, DR));
#endif
    L.u.d.T[LdsW::kDROOT + i] = v ? v : dslow ? E_SLOW : (uint16_t)0x4001u;
  }
  __builtin_amdgcn_wave_barrier();
}

// x^(8 n) mod P (reflected), from x^(2^k)
DQ_AI uint32_t x8n_tail(uint32_t n) {
  uint32_t p = 1u << 31;  // x^0
  for (int k = 3; n; n >>= 1, k++)
    if (n & 1) p = gf2_mulmod(c_x2n[k & 31], p);
  return p;
}

// One wave per deferred tail: the deflate blocks of BGZF block b after the first `produced` bytes
// (TailDesc), decoded as the block kernel decodes its first one -- speculative segments (at most
// 64, one per lane), checkpoint merges, wave-local rounds instead of barrier-separated ones, the
// emit into the tail image -- then resolved row by row (64 bytes, one per lane): a source before
// the tail is read from U (written by the block kernel), one in an earlier row from the image, one
// in the same row waits for its lane.  Stores the tail's bytes and finishes the block's CRC32 from
// the prefix's CRC register.  No workgroup barrier: the waves of a workgroup are independent.
template <bool TIMING>
__global__ __launch_bounds__(64 * TW, 4) void inflate_tail_kernel(
    const uint8_t* __restrict__ C, const int64_t* __restrict__ blk_pos,
    const int32_t* __restrict__ blk_csize, const int32_t* __restrict__ blk_usize,
    const int64_t* __restrict__ uoff, int64_t ngrid, uint8_t* __restrict__ U,
    int32_t* __restrict__ status, int32_t verify_crc, const uint32_t* __restrict__ crc_init,
    uint32_t OV, uint32_t sflags, const int32_t* __restrict__ sel,
    const TailDesc* __restrict__ tails, uint64_t* __restrict__ tim) {
  constexpr uint32_t CKI = CKI_DEFAULT;
  __shared__ LdsW Ls[TW];
  // the wave's index is uniform: the tail's descriptor and block fields become scalar loads held in
  // SGPRs (as vector loads they held 10 VGPRs for the whole kernel and forced spills to scratch)
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), lane = (int)(threadIdx.x & 63);
  const int64_t gi = (int64_t)blockIdx.x * TW + wv;
  if (gi >= ngrid) return;
  const TailDesc td = tails[gi];
  if (td.flag != 1) return;
  LdsW& L = Ls[wv];
  const uint64_t t0 = TIMING ? __builtin_amdgcn_s_memtime() : 0;
  const int64_t b = sel ? (int64_t)sel[gi] : gi;
  const int64_t cpos = blk_pos[b];
  const int32_t csize = blk_csize[b];
  const int32_t isize = blk_usize[b];
  const int64_t ub = uoff[b];
  const int32_t p0 = td.produced;       // tail byte k is block byte p0 + k
  const int sh = (int)((ub + p0) & 15);  // image byte sh + k: U's 16-byte lines align with the image
  const uint8_t* dp = C + cpos + 18;
  const int mis = (int)(reinterpret_cast<uintptr_t>(dp) & 15);
  const uint32_t* W = reinterpret_cast<const uint32_t*>(__builtin_assume_aligned(dp - mis, 16));
  const int32_t dbytes = csize - 26;
  const uint32_t endbits = 8u * (uint32_t)mis + 8u * (uint32_t)max(dbytes, 0);
#ifdef DQ_CHECKED
  GSrc gsrc{W, (endbits >> 5) + 8, 4u << 12};
#else
  const GSrc gsrc{W};
#endif
  // warm the cache with the tail's compressed bytes (this kernel runs after the block kernel has
  // streamed the whole file: they are long out of L2): one 128-byte line per lane, up to 8 KB;
  // the value is consumed at the end, so no wait is added
  uint32_t warm = 0;
  {
    const uint32_t lo = (uint32_t)td.pos >> 3, nbytes = endbits / 8 - min(endbits / 8, lo);
    if ((uint32_t)lane * 128 < nbytes)
      warm = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(W) + ((lo + 128 * lane) & ~3u));
  }
  for (int i = lane; i < TOUT / 32; i += 64) L.bm[i] = 0;
  if (lane < 8) L.misc[lane] = 0;
  __builtin_amdgcn_wave_barrier();
  int32_t produced = p0;
  uint32_t pos = (uint32_t)td.pos;
  uint64_t tph[5] = {0, 0, 0, 0, 0};  // TIMING: header, tables + pair table, spec, rounds, emit
  uint64_t tl = TIMING ? __builtin_amdgcn_s_memtime() : 0;
  auto tick = [&](int k) {
    if (TIMING) {
      const uint64_t now = __builtin_amdgcn_s_memtime();
      tph[k] += now - tl;
      tl = now;
    }
  };
  while (L.misc[M_ERR] == 0 && produced < isize) {
    // ---- header (as the block kernel: every lane reads it, the branches are uniform)
    const uint32_t clpos = pos + 17;
    const uint32_t hbase = clpos >> 5;
#if DQ_TAIL_HDR1
    // every load of the header in one round trip: the block header, a dynamic header's staged
    // words and its code-length code lengths (HCLEN is not known yet: all 19 are loaded; a stored
    // or fixed block's over-read stays inside the 4096 zero bytes that follow C)
    constexpr int HWN = (HB_WORDS + 63) / 64;
    uint32_t hw[HWN];
#pragma unroll
    for (int j = 0; j < HWN; j++) hw[j] = lane + 64 * j < HB_WORDS ? W[hbase + lane + 64 * j] : 0u;
    const uint32_t clv = lane < 19 ? peek_bits(W, clpos + 3 * (uint32_t)lane, 3) : 0u;
#endif
    const uint32_t h = peek_bits(W, pos, 17);
    const int32_t bfinal = (int32_t)(h & 1), btype = (int32_t)((h >> 1) & 3);
    const int32_t herr = pos + 3 > endbits ? ST_OVERREAD : btype == 3 ? ST_BAD_BLOCKTYPE : 0;
    if (herr) {
      set_err(L, herr);
      break;
    }
    if (btype == 0) {  // stored block: copy
      const uint32_t q = (pos + 3 + 7) & ~7u;
      const uint8_t* bp = reinterpret_cast<const uint8_t*>(W) + q / 8;
      const uint32_t len = bp[0] | ((uint32_t)bp[1] << 8), nl = bp[2] | ((uint32_t)bp[3] << 8);
      const int32_t serr = (len ^ 0xffffu) != nl ? ST_BAD_STORED : q + 32 + 8 * len > endbits ? ST_OVERREAD : 0;
      if (serr) {
        set_err(L, serr);
        break;
      }
      const int32_t n = min((int32_t)len, isize - produced);
      if (produced + n - p0 > TOUT) {
        set_err(L, ST_SHORT);
        break;
      }
      for (int i = lane; i < n; i += 64) L.out[sh + produced - p0 + i] = bp[4 + i];
      produced += n;
      pos = q + 32 + 8 * len;
      __builtin_amdgcn_wave_barrier();
      if (bfinal) break;
      continue;
    }
    const int nlen = btype == 1 ? 288 : (int)((h >> 3) & 31) + 257;
    const int ndist = btype == 1 ? 32 : (int)((h >> 8) & 31) + 1;
    if (btype == 2 && (nlen > 286 || ndist > 30)) {
      set_err(L, ST_BAD_TABLE);
      break;
    }
    uint32_t a;
    if (btype == 1) {
      for (int i = lane; i < 320; i += 64) L.u.d.x.h.lens[i] = fixed_len(i);
      a = pos + 3;
    } else {
      const int ncode = (int)((h >> 13) & 15) + 4;
      for (int i = lane; i < 320; i += 64) L.u.d.x.h.lens[i] = 0;
#if DQ_TAIL_HDR1
#pragma unroll
      for (int j = 0; j < HWN; j++)
        if (lane + 64 * j < HB_WORDS) reinterpret_cast<uint32_t*>(L.u.d.T)[lane + 64 * j] = hw[j];
      if (lane < 19) L.u.d.x.h.clen[c_clorder3[lane]] = lane < ncode ? (uint8_t)clv : 0;
#else
      for (int i = lane; i < HB_WORDS; i += 64) reinterpret_cast<uint32_t*>(L.u.d.T)[i] = W[hbase + i];
      if (lane < 19)
        L.u.d.x.h.clen[c_clorder3[lane]] = lane < ncode ? (uint8_t)peek_bits(W, clpos + 3 * lane, 3) : 0;
#endif
      __builtin_amdgcn_wave_barrier();
      bool ok = true;
      L.u.d.x.h.clt[lane] = clt_entry(L.u.d.x.h.clen, lane, &ok);
      L.u.d.x.h.clt[lane + 64] = clt_entry(L.u.d.x.h.clen, lane + 64, &ok);
      if (__any(!ok)) {
        set_err(L, ST_BAD_TABLE);
        break;
      }
      __builtin_amdgcn_wave_barrier();
      a = read_lengths_wave(L, clpos + 3 * (uint32_t)ncode, nlen, ndist, endbits, hbase);
      __builtin_amdgcn_wave_barrier();
      if (L.misc[M_ERR]) break;
      if (L.u.d.x.h.lens[256] == 0) {  // an EOB code is required
        set_err(L, ST_BAD_TABLE);
        break;
      }
    }
    tick(0);
    // ---- tables
    build_tables_wave(L, nlen, ndist);
    if (L.misc[M_ERR]) break;
    __builtin_amdgcn_wave_barrier();
    const bool slow = L.misc[M_SLOW] != 0;
    if (a > endbits) {
      set_err(L, ST_OVERREAD);
      break;
    }
    tick(1);
    // ---- speculative segments, one per lane (registers hold the per-lane arrays)
    const uint32_t span = endbits - a;
    const int nl = (int)max(1u, min(64u, span / (uint32_t)TAIL_SEG_MIN));
    const uint32_t seg = (span + nl - 1) / nl;
    const bool act = lane < nl;
    const uint32_t sB = a + (uint32_t)lane * seg;
    const uint32_t sE = lane == nl - 1 ? 0xffffffffu : sB + seg;
    int32_t AB = -1, AE = 0, AC = 0, SE = 0, SC = 0;
    if (act) {
      const uint32_t start = lane == 0 ? a : (sB > a + OV ? sB - OV : a);
      for (int j = 0; j < T_NCK; j++) L.ck[j * 64 + lane] = 0xffffffffu;
      int32_t B = -1, E = 0, c = 0;
      const int f = slow ? run_seg<true>(gsrc, L, start, sB, sE, endbits, &B, &E, &c, L.ck + lane, 64, CKI, T_NCK)
                         : run_seg<false>(gsrc, L, start, sB, sE, endbits, &B, &E, &c, L.ck + lane, 64, CKI, T_NCK);
      AB = B;
      AE = (E << 3) | f;
      AC = c;
      SE = AE;
      SC = c;
    }
    tick(2);
    // ---- rounds, wave-local: a lane whose first boundary differs from its predecessor's exit
    //      re-decodes from that exit until it meets its speculative path at a checkpoint
#ifdef DQ_CHECKED
    gsrc.tag = 5u << 12;
#endif
    for (int round = 0; round <= nl; round++) {
      const int32_t pe = __shfl_up(AE, 1, 64);
      const bool need = act && lane > 0 && (pe & 7) == F_EXIT && AB != (pe >> 3);
      if (!__any(need)) break;
      bool changed = false;
      if (need) {
        const uint32_t s0 = (uint32_t)(pe >> 3);
        int32_t E = 0, c = 0;
        const int f = slow ? run_redo<true>(gsrc, L, s0, sB, sE, endbits, L.ck + lane, 64, SE, SC, &E, &c, CKI, T_NCK)
                           : run_redo<false>(gsrc, L, s0, sB, sE, endbits, L.ck + lane, 64, SE, SC, &E, &c, CKI, T_NCK);
        const int32_t ae = (E << 3) | f;
        changed = ae != AE;
        AB = (int32_t)s0;
        AE = ae;
        AC = c;
      }
      if (!__any(changed)) break;
    }
    // ---- counts -> offsets (the first non-exit lane ends the deflate block)
    const int myF = act ? (AE & 7) : F_DEAD;
    const uint64_t nonexit = __ballot(act && myF != F_EXIT);
    const int last = nonexit ? (int)__builtin_ctzll(nonexit) : nl - 1;
    const int32_t cv = lane <= last ? AC : 0;
    const int32_t incl = wave_incl_scan(cv, lane);
    const int32_t total = __shfl(incl, 63, 64);
    const int32_t myoff = produced + incl - cv;
    const bool full = produced + total >= isize;
    const int32_t fl = __shfl(myF, last, 64);
    const int32_t nextpos = __shfl(AE >> 3, last, 64);
    if (!full && fl != F_EOB) {
      set_err(L, fl == F_ERR ? ST_BAD_CODE : ST_SHORT);
      break;
    }
    if (min(isize, produced + total) - p0 > TOUT) {  // the block kernel checked the bound
      set_err(L, ST_SHORT);
      break;
    }
    tick(3);
    // ---- emit into the tail image
#ifdef DQ_CHECKED
    gsrc.tag = 6u << 12;
#endif
    if (lane <= last && myoff < isize) {
      if (slow) emit_seg<true>(gsrc, L, (uint32_t)AB, sE, endbits, myoff, isize, sh, p0);
      else emit_seg<false>(gsrc, L, (uint32_t)AB, sE, endbits, myoff, isize, sh, p0);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    produced = min(isize, produced + total);
    tick(4);
    if (full || bfinal) break;
    pos = (uint32_t)nextpos;
  }
  int32_t err = L.misc[M_ERR];
  if (!err && produced != isize) err = ST_SHORT;
  if (err) {
    if (lane == 0) status[b] = err;
    return;
  }
  const uint64_t t1 = TIMING ? __builtin_amdgcn_s_memtime() : 0;
  // ---- resolve the tail in rows of 256 image bytes, in order, lane l owning image bytes
  //      4 l .. 4 l + 3 (one dword: every write is one aligned ds_write_b32).  Per row: every
  //      byte's copy source from the bitmap (at most two owners per lane; the match carried into
  //      the row held in registers); the bytes whose source lies before the tail are loaded from
  //      U three rows ahead (software-pipelined: the HBM latency overlaps three rows' work) and written
  //      in place with the literals; the rest follow in-row pointers by lock-step pointer jumping
  //      (256 16-bit next pointers in the dead checkpoint area) to a byte in place or of an earlier
  //      row, then copy.  Round 4 resolved 64-byte rows by ballot rounds, a lane copying once its
  //      source lane had: in-row chains of short distances ran one lane per round.
  const int32_t n = isize - p0;
  const int nrows = (sh + n + 255) >> 8;
  uint8_t* const O = L.out + sh;  // tail byte k at O[k]
  const uint8_t* Ub = U + ub + p0;  // the tail's first byte in U: sources before it are final
  // the copy sources of row `row`: src[i] (tail coordinates, < 0 before the tail), copy bits, and
  // the carried match (cms, cdesc) advanced past the row (its descriptor read while intact)
  auto hops = [&](int row, int32_t& cms, uint32_t& cdesc, int32_t (&src)[4], uint32_t& cpy) {
    const int32_t x0 = 256 * row + 4 * lane - sh;  // tail byte of the lane's first byte
    const int32_t nval = min(max(n - x0, 0), 4);
    uint32_t b4 = 0;
    if (nval > 0) {
      if (x0 >= 0) {
        const int32_t wi = x0 >> 5;
        b4 = __builtin_amdgcn_alignbit(L.bm[min(wi + 1, TOUT / 32 - 1)], L.bm[wi], (uint32_t)x0 & 31u);
      } else if (x0 > -4) {
        b4 = L.bm[0] << (-x0);
      }
      b4 &= (1u << nval) - 1u;
    }
    const int32_t lst = b4 ? x0 + 31 - (int32_t)__clz(b4) : -1;
    const int32_t incl = wave_incl_max(lst);
    int32_t pre = __shfl_up(incl, 1, 64);
    pre = lane == 0 ? -1 : pre;
    const int32_t o0 = (b4 & 1u) ? x0 : max(pre, cms);
    const uint32_t r1 = b4 & ~1u;  // a second start in the lane (>= 3 bytes after the first)
    const int32_t p1 = r1 ? x0 + (int32_t)__builtin_ctz(r1) : -1;
    const uint32_t d0 = o0 < 0 ? 0u : (o0 == cms ? cdesc : load_desc(L, sh + o0));
    const uint32_t d1 = p1 < 0 ? 0u : load_desc(L, sh + p1);
    const int32_t last = max(__builtin_amdgcn_readlane(incl, 63), cms);  // uniform
    if (last != cms) {
      cdesc = load_desc(L, sh + last);
      cms = last;
    }
    cpy = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int32_t x = x0 + i;
      const bool at1 = p1 >= 0 && x >= p1;
      const int32_t ms = at1 ? p1 : o0;
      const uint32_t ds = at1 ? d1 : d0;
      const int32_t len = (int32_t)(ds >> 15) + 3, D = (int32_t)(ds & 0x7fff) + 1;
      const bool copy = ms >= 0 && i < nval && x >= 0 && x < ms + len;
      const int32_t jj = x - ms;
      int32_t rm = jj;  // (x - ms) mod D: only past the first period of an overlapping match
      if (__builtin_expect(__any(copy && jj >= D), 0)) {
        const int32_t q = (int32_t)((float)jj * __builtin_amdgcn_rcpf((float)D));
        rm = jj - q * D;
        rm = rm >= D ? rm - D : rm;
      }
      src[i] = ms - D + rm;
      DQ_CHK(!copy || (src[i] >= -p0 && src[i] < x), CHK_K2_SRC);
      cpy |= copy ? 1u << i : 0u;
    }
  };
  const int32_t Yend = sh + n;  // image bytes of the tail: [sh, Yend)
  uint64_t rst[4] = {0, 0, 0, 0};  // TIMING: rows, jump rounds, rows with pending bytes, round cycles
  const uint64_t t2 = TIMING ? __builtin_amdgcn_s_memtime() : 0;
  {  // the rows in order; a row's sources before the tail are loaded from U three rows ahead
    constexpr uint32_t TERM = 0x8000u;  // next pointer of a byte whose value is in place
    uint16_t* const nx = reinterpret_cast<uint16_t*>(L.ck);  // the row's 256 next pointers
    int32_t cms = -1;
    uint32_t cdesc = 0;
    // a row's sources and its loads from U: unconditional loads (a byte that needs none loads the
    // prefix's last byte, or the tail's first when the prefix is empty -- p0 = 0 after an empty
    // first deflate block: Ub[-1] would lie before the block, for block 0 before U) into fixed
    // registers per slot, so the compiler's wait for a slot's values counts only the loads issued
    // before them (no branch, no register shuffling)
    const int32_t dmy = p0 > 0 ? -1 : 0;  // uniform
    auto prefetch = [&](int row, int32_t (&s)[4], uint32_t& c, uint32_t (&g)[4]) {
      c = 0;
      hops(row, cms, cdesc, s, c);  // rows in order (the carry); past the last row: no copies
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int32_t gi = ((c >> i) & 1u) && s[i] < 0 ? s[i] : dmy;
        DQ_CHK(gi >= -p0 && gi < max(n, 1), CHK_K2_SRC);
        g[i] = Ub[gi];
      }
    };
    auto do_row = [&](int row, const int32_t (&src)[4], uint32_t cpy, const uint32_t (&g)[4]) {
      const int32_t Y = 256 * row + 4 * lane;  // the lane's image dword
      const int32_t x0 = Y - sh, xr = 256 * row - sh;
      const bool live = Y < Yend;
      // (a) bytes whose value is known now -- literals (in place) and sources before the tail
      //     (loaded) -- are written and marked terminal; the others' next pointers published
      uint32_t own = live ? *reinterpret_cast<const uint32_t*>(L.out + Y) : 0u;
      uint32_t pend = 0;
      int32_t p[4];
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const bool c = (cpy >> i) & 1u;
        const bool pre = c && src[i] < 0;
        own = pre ? (own & ~(0xffu << (8 * i))) | (g[i] << (8 * i)) : own;
        p[i] = !c || pre ? (int32_t)((uint32_t)(x0 + i) | TERM) : src[i];
        pend |= c && !pre && src[i] >= xr ? 1u << i : 0u;
      }
      if (live) *reinterpret_cast<uint32_t*>(L.out + Y) = own;
      auto publish = [&]() {
        uint2 w;
        w.x = ((uint32_t)p[0] & 0xffffu) | ((uint32_t)p[1] << 16);
        w.y = ((uint32_t)p[2] & 0xffffu) | ((uint32_t)p[3] << 16);
        *reinterpret_cast<uint2*>(nx + 4 * lane) = w;
        // the pointers are read back as 16-bit words: no reordering across the 8-byte store (a
        // different type, so the compiler could otherwise move the next reads above it)
        asm volatile("" ::: "memory");
      };
      publish();
      // (b) pointer jumping inside the row (lock-step: a round's reads precede its writes): a
      //     pending pointer into the row takes that byte's pointer; a terminal byte or a byte of
      //     an earlier row ends it
      const uint64_t tj0 = TIMING ? __builtin_amdgcn_s_memtime() : 0;
      if (TIMING) {
        rst[0] += 1;
        rst[2] += __any(pend != 0) ? 1 : 0;
      }
      for (int rnd = 0; __any(pend != 0) && rnd < 10; rnd++) {
        if (TIMING) rst[1] += 1;
        uint32_t q[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const bool pd = (pend >> i) & 1u;
          DQ_CHK(!pd || (p[i] - xr >= 0 && p[i] - xr < 256), CHK_K2_NXT);
          q[i] = zx16(nx[pd ? p[i] - xr : 4 * lane + i]);
        }
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const bool pd = (pend >> i) & 1u;
          // q: a terminal (the byte holding the value, flagged), a byte of an earlier row, or a
          // byte of this row further down the chain
          const bool fin = pd && ((q[i] & TERM) || (int32_t)q[i] < xr);
          p[i] = pd ? (int32_t)q[i] : p[i];
          pend &= fin ? ~(1u << i) : ~0u;
        }
        publish();
      }
      if (TIMING) rst[3] += __builtin_amdgcn_s_memtime() - tj0;
      // (c) the copies: every pointer is now a byte in place (terminal) or of an earlier row
      uint32_t v = own;
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const bool c = (cpy >> i) & 1u;
        const int32_t s = (int32_t)((uint32_t)p[i] & ~TERM);
        const bool done = !c || src[i] < 0;
        const uint32_t b = done ? 0u : (uint32_t)O[s];
        v = done ? v : (v & ~(0xffu << (8 * i))) | (b << (8 * i));
      }
      if (live) *reinterpret_cast<uint32_t*>(L.out + Y) = v;
    };
    int32_t sA[4], sB[4], sC[4];
    uint32_t cA = 0, cB = 0, cC = 0, gA[4], gB[4], gC[4];
    prefetch(0, sA, cA, gA);
    prefetch(1, sB, cB, gB);
    prefetch(2, sC, cC, gC);
    for (int row = 0; row < nrows; row += 3) {  // three rows per pass, a fixed slot each
      do_row(row, sA, cA, gA);
      prefetch(row + 3, sA, cA, gA);
      do_row(row + 1, sB, cB, gB);
      prefetch(row + 4, sB, cB, gB);
      do_row(row + 2, sC, cC, gC);
      prefetch(row + 5, sC, cC, gC);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  const uint64_t t3 = TIMING ? __builtin_amdgcn_s_memtime() : 0;
  // ---- store: bytes up to the first 16-byte line of U, the lines, the last bytes
  uint8_t* dst = U + ub + p0;
  const int head = min((16 - sh) & 15, n);
  const int32_t lines = (n - head) / 16;
  for (int x = lane; x < head; x += 64) dst[x] = O[x];
  for (int32_t k = lane; k < lines; k += 64) {
    const uint4 v = *reinterpret_cast<const uint4*>(O + head + 16 * k);
    uint4* d = reinterpret_cast<uint4*>(dst + head + 16 * k);
    if (sflags & 2) st_nt(d, v);
    else *d = v;
  }
  for (int x = head + 16 * lines + lane; x < n; x += 64) dst[x] = O[x];
  // ---- CRC32 of the block: the prefix's register shifted past the tail, xor the tail's
  if (verify_crc) {
    // slice-by-4 over a slice of ceil(n / 64) bytes per lane (dwords where the image allows),
    // moved to the tail's end by x^(8 k) from a table (round 4: byte steps, and the shift by a
    // loop of one 32-step multiply per bit of k)
    for (int i = lane; i < 1024; i += 64) (&L.u.crc4[0][0])[i] = (&c_crc4[0][0])[i];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const int32_t sl = (n + 63) >> 6;
    const int32_t s0 = min(n, lane * sl), s1 = min(n, s0 + sl);
    uint32_t cr = 0;
    int32_t x = s0;
    while (x < s1 && ((sh + x) & 3)) cr = L.u.crc4[0][(cr ^ O[x++]) & 0xff] ^ (cr >> 8);
    for (; x + 4 <= s1; x += 4) {
      const uint32_t v = cr ^ *reinterpret_cast<const uint32_t*>(O + x);
      cr = L.u.crc4[3][v & 0xff] ^ L.u.crc4[2][(v >> 8) & 0xff] ^ L.u.crc4[1][(v >> 16) & 0xff] ^
           L.u.crc4[0][v >> 24];
    }
    while (x < s1) cr = L.u.crc4[0][(cr ^ O[x++]) & 0xff] ^ (cr >> 8);
    cr = gf2_mulmod(c_x8n[n - s1], cr);
    cr = (uint32_t)__shfl((int)wave_incl_xor(cr), 63, 64);
    if (lane == 0) {
      const uint32_t raw = gf2_mulmod(c_x8n[n], td.crc_raw) ^ cr;
      const uint32_t crc = (raw ^ crc_init[isize]) ^ 0xffffffffu;
      const uint8_t* tr = C + cpos + csize - 8;
      const uint32_t want = (uint32_t)tr[0] | ((uint32_t)tr[1] << 8) | ((uint32_t)tr[2] << 16) | ((uint32_t)tr[3] << 24);
      if (crc != want) status[b] = ST_CRC;
    }
  }
  if (warm == 0x9e3779b9u && lane == 64) status[b] = 0;  // (keeps the warming load alive)
  if (TIMING && lane == 0) {
    tim[gi * 16] = t1 - t0;      // decode: headers, tables, spec, rounds, emit
    tim[gi * 16 + 1] = t3 - t2;  // resolve: the rows
    tim[gi * 16 + 2] = __builtin_amdgcn_s_memtime() - t3;  // store, CRC
    tim[gi * 16 + 3] = 1;
    for (int k = 0; k < 5; k++) tim[gi * 16 + 4 + k] = tph[k];
    for (int k = 0; k < 4; k++) tim[gi * 16 + 9 + k] = rst[k];
  }
}

uint32_t h_mul(uint32_t a, uint32_t b) {
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
}

// Host-side CRC tables, computed once per process.
struct HostTables {
  uint32_t crc4[4][256];
  uint32_t slice[WG];
  uint32_t x2n[32];  // x^(2^k) mod P
  uint32_t x8n[TOUT + 1];  // x^(8 n) mod P, n <= TOUT
  std::vector<uint32_t> init;  // CRC of n zero bytes with initial register ~0, n = 0..65536
  HostTables() : init(65537) {
    for (uint32_t i = 0; i < 256; i++) {
      uint32_t c = i;
      for (int k = 0; k < 8; k++) c = c & 1 ? (c >> 1) ^ 0xEDB88320u : c >> 1;
      crc4[0][i] = c;
    }
    for (int j = 1; j < 4; j++)
      for (uint32_t i = 0; i < 256; i++) crc4[j][i] = (crc4[j - 1][i] >> 8) ^ crc4[0][crc4[j - 1][i] & 0xff];
    uint32_t p = 1u << 30;  // x^1
    x2n[0] = p;
    for (int k = 1; k < 32; k++) x2n[k] = p = h_mul(p, p);
    // x^(8 * CRC_SL * k) mod P: x^(8 CRC_SL) from the x^(2^k) of its set bits; powers by
    // repeated multiplication
    uint32_t step = 1u << 31;  // x^0
    for (int k = 0; k < 31; k++)
      if (((uint32_t)(8 * CRC_SL) >> k) & 1u) step = h_mul(step, x2n[k]);
    slice[0] = 1u << 31;  // x^0
    for (int k = 1; k < WG; k++) slice[k] = h_mul(slice[k - 1], step);
    uint32_t x8 = 1u << 31;          // x^0
    const uint32_t x8step = x2n[3];  // x^8
    for (int n = 0; n <= 65536; n++) {
      if (n <= TOUT) x8n[n] = x8;
      init[(size_t)n] = h_mul(x8, 0xffffffffu);
      x8 = h_mul(x8, x8step);
    }
  }
};

// Per-device state: the __constant__ tables are per-device copies of the code object, and the
// init table is device memory, so every device is initialised on its own, once.
constexpr int kMaxDevices = 64;
struct DevTables {
  std::once_flag once;
  uint32_t* crc_init = nullptr;
  bool ok = false;
};
DevTables g_dev[kMaxDevices];

}  // namespace

DQ_CHK_UNIT(inflate)

const uint32_t* inflate3_tables(int device) {
  if (device < 0 || device >= kMaxDevices) return nullptr;
  DevTables& D = g_dev[device];
  std::call_once(D.once, [&] {
    static const HostTables H;
    int prev = -1;
    (void)hipGetDevice(&prev);
    bool ok = hipSetDevice(device) == hipSuccess;
    ok = ok && hipMemcpyToSymbol(HIP_SYMBOL(c_crc4), H.crc4, sizeof H.crc4) == hipSuccess;
    ok = ok && hipMemcpyToSymbol(HIP_SYMBOL(c_slice_shift), H.slice, sizeof H.slice) == hipSuccess;
    ok = ok && hipMemcpyToSymbol(HIP_SYMBOL(c_x2n), H.x2n, sizeof H.x2n) == hipSuccess;
    ok = ok && hipMemcpyToSymbol(HIP_SYMBOL(c_x8n), H.x8n, sizeof H.x8n) == hipSuccess;
    ok = ok && hipMalloc(&D.crc_init, sizeof(uint32_t) * H.init.size()) == hipSuccess;
    ok = ok && hipMemcpy(D.crc_init, H.init.data(), sizeof(uint32_t) * H.init.size(),
                         hipMemcpyHostToDevice) == hipSuccess;
    D.ok = ok;
    if (prev >= 0) (void)hipSetDevice(prev);
  });
  return D.ok ? D.crc_init : nullptr;
}

void launch_inflate3(const uint8_t* C, const int64_t* blk_pos, const int32_t* blk_csize,
                     const int32_t* blk_usize, const int64_t* uoff, int64_t nblk, uint8_t* U,
                     int32_t* status, int32_t verify_crc, const uint32_t* crc_init, uint64_t* tim,
                     hipStream_t s, const int32_t* sel, int64_t nsel, void* tails_buf) {
  if (nblk <= 0) return;
  const int64_t ngrid = sel ? nsel : nblk;
  if (ngrid <= 0) return;
#ifdef DQ_TUNING
  // Decode-shape knobs of the tuning builds only (tools/build_variant.sh NAME -DDQ_TUNING): the
  // product library has a single configuration, so an executor's inherited environment cannot
  // select an untested path.  DQ_OV warm-up bits, DQ_STORE U store mode (bit 0 whole block at the
  // end, bit 1 non-temporal), DQ_NDEC lane cap, DQ_SEGBITS minimum segment bits, DQ_WARM L2 warm-up,
  // DQ_LDSPAD extra dynamic LDS (80000 = one workgroup per CU), DQ_TAIL=0 no tail kernel.
  static const uint32_t ov = getenv("DQ_OV") ? (uint32_t)atoi(getenv("DQ_OV")) : OV_DEFAULT;
  static const uint32_t sflags =
      (getenv("DQ_STORE") ? (uint32_t)atoi(getenv("DQ_STORE")) & 3u : 2u) |
      (getenv("DQ_NDEC") ? (uint32_t)(atoi(getenv("DQ_NDEC")) & 1023) << 8 : 0u) |
      (getenv("DQ_SEGBITS") ? (uint32_t)(atoi(getenv("DQ_SEGBITS")) & 1023) << 20 : 0u) |
      (getenv("DQ_WARM") && atoi(getenv("DQ_WARM")) ? 16u : 0u);
  static const unsigned ldspad = getenv("DQ_LDSPAD") ? (unsigned)atoi(getenv("DQ_LDSPAD")) : 0u;
  static const bool tail_on = !getenv("DQ_TAIL") || atoi(getenv("DQ_TAIL")) != 0;
#else
  constexpr uint32_t ov = OV_DEFAULT;
  constexpr uint32_t sflags = 2u;  // U lines stored per batch, non-temporal
  constexpr unsigned ldspad = 0u;
  constexpr bool tail_on = true;
#endif
  TailDesc* td = tail_on ? static_cast<TailDesc*>(tails_buf) : nullptr;
  if (td) (void)hipMemsetAsync(td, 0, sizeof(TailDesc) * (size_t)ngrid, s);
#define DQ_LAUNCH(TM, NBT, GT)                                                                  \
  hipLaunchKernelGGL((inflate_block_kernel<TM, NBT, GT>), dim3((unsigned)ngrid), dim3(WG), ldspad, s, C, \
                     blk_pos, blk_csize, blk_usize, uoff, ngrid, U, status, verify_crc, crc_init, tim, ov, \
                     sflags, sel, td)
  // NB = 4 chunks of G = 1 byte per thread: (1, 4) measures the same, (2, 1) slower (round 5)
  if (tim)
    DQ_LAUNCH(true, DQ_RES_NB, DQ_RES_G);
  else
    DQ_LAUNCH(false, DQ_RES_NB, DQ_RES_G);
#undef DQ_LAUNCH
  // DQ_TIMING: the block kernel's phases in tim[0, TIM_W ngrid), the tail kernel's in the 16 ngrid
  // words after them (16 per tail; dq_api allocates TIM_W + 16 per block)
  if (td && tim)
    hipLaunchKernelGGL((inflate_tail_kernel<true>), dim3((unsigned)((ngrid + TW - 1) / TW)), dim3(64 * TW), 0, s,
                       C, blk_pos, blk_csize, blk_usize, uoff, ngrid, U, status, verify_crc, crc_init,
                       ov == OV_DEFAULT ? (uint32_t)DQ_TAIL_OV : ov, sflags, sel, td, tim + TIM_W * ngrid);  // 16 words per tail
  else if (td)
    hipLaunchKernelGGL((inflate_tail_kernel<false>), dim3((unsigned)((ngrid + TW - 1) / TW)), dim3(64 * TW), 0, s,
                       C, blk_pos, blk_csize, blk_usize, uoff, ngrid, U, status, verify_crc, crc_init,
                       ov == OV_DEFAULT ? (uint32_t)DQ_TAIL_OV : ov, sflags, sel, td, nullptr);
}

}  // namespace dq
