// dq_inflate_core.h -- DEFLATE (RFC 1951) decode primitives shared by the inflate kernel
// (dq_inflate.hip) and its host-side model (tests/native/inflate_model.cpp, used to validate the
// speculative-segment algorithm against zlib on the CPU before it runs on gfx950).
//
// Decode tables: a 9-bit (litlen) / 8-bit (distance) root table of packed 32-bit entries
//   bits 0..3   code length in bits (0 = longer than the root: canonical slow path)
//   bits 4..7   extra bits that follow the code (length / distance extra bits)
//   bits 8..9   kind: K_LIT literal, K_LEN length (or distance for the distance table), K_EOB, K_BAD
//   bits 16..31 value: literal byte, length base (3..258) or distance base (1..24577)
// Codes longer than the root bits are decoded canonically from per-length first-code / count /
// offset arrays and the symbols sorted in canonical order (HuffCanon).
#pragma once
#include <stdint.h>

#ifndef __HIPCC__
#ifndef __host__
#define __host__
#define __device__
#endif
#endif

#define DQI_INLINE __host__ __device__ inline __attribute__((always_inline))

namespace dqi {

constexpr int LB = 9;   // litlen root bits
constexpr int DB = 8;   // distance root bits
enum : uint32_t { K_LIT = 0, K_LEN = 1, K_EOB = 2, K_BAD = 3 };

struct HuffCanon {       // one alphabet's canonical description (for codes longer than the root)
  uint16_t first[16];    // first canonical code of length l
  uint16_t count[16];    // number of codes of length l
  uint16_t offs[16];     // index in the sorted symbol list of the first code of length l
};

DQI_INLINE uint32_t mk_entry(uint32_t nbits, uint32_t extra, uint32_t kind, uint32_t value) {
  return nbits | (extra << 4) | (kind << 8) | (value << 16);
}

// Length symbols 257..285 (RFC 1951 3.2.5): base and extra bits.
DQI_INLINE uint32_t len_base(uint32_t k) {  // k = sym - 257, 0..28
  if (k < 8) return 3 + k;
  if (k == 28) return 258;
  const uint32_t e = (k - 4) >> 2;          // extra bits 1..5
  return ((4u + (k & 3)) << e) + 3;
}
DQI_INLINE uint32_t len_extra(uint32_t k) { return (k < 8 || k == 28) ? 0u : ((k - 4) >> 2); }
// Distance symbols 0..29.
DQI_INLINE uint32_t dist_base(uint32_t d) {
  if (d < 4) return d + 1;
  const uint32_t e = (d - 2) >> 1;          // extra bits 1..13
  return ((2u + (d & 1)) << e) + 1;
}
DQI_INLINE uint32_t dist_extra(uint32_t d) { return d < 4 ? 0u : ((d - 2) >> 1); }

// Packed entry of litlen symbol `sym` with an `nbits`-bit code.
DQI_INLINE uint32_t ll_entry(uint32_t sym, uint32_t nbits) {
  if (sym < 256) return mk_entry(nbits, 0, K_LIT, sym);
  if (sym == 256) return mk_entry(nbits, 0, K_EOB, 0);
  if (sym <= 285) return mk_entry(nbits, len_extra(sym - 257), K_LEN, len_base(sym - 257));
  return mk_entry(nbits, 0, K_BAD, 0);     // 286, 287: valid codes, invalid symbols
}
DQI_INLINE uint32_t d_entry(uint32_t sym, uint32_t nbits) {
  if (sym < 30) return mk_entry(nbits, dist_extra(sym), K_LEN, dist_base(sym));
  return mk_entry(nbits, 0, K_BAD, 0);
}

DQI_INLINE uint32_t bitrev(uint32_t v, int n) {
#ifdef __HIPCC__
  return __builtin_bitreverse32(v) >> (32 - n);
#else
  uint32_t r = 0;
  for (int i = 0; i < n; i++) r |= ((v >> i) & 1u) << (n - 1 - i);
  return r;
#endif
}

// Canonical decode of the code at the low end of `bits` (LSB-first stream), lengths lo..15.
// Returns the symbol index in the sorted list and the length, or -1 when no code matches.
DQI_INLINE int canon_decode(uint32_t bits, const HuffCanon& h, int lo, int* len) {
  const uint32_t r = bitrev(bits & 0x7fffu, 15);
  for (int l = lo; l <= 15; l++) {
    const uint32_t c = r >> (15 - l);
    const uint32_t d = c - h.first[l];
    if (d < h.count[l]) {
      *len = l;
      return (int)(h.offs[l] + d);
    }
  }
  return -1;
}

// Build a canonical description from code lengths.  Over-subscribed codes and incomplete codes
// are rejected as zlib's inflate_table does; a distance alphabet with a single length-1 code is
// allowed (allow_single).  Returns 0 on success.  sym_out receives the symbols in canonical order.
template <typename SymT>
DQI_INLINE int canon_build(const uint8_t* lens, int n, HuffCanon& h, SymT* sym_out,
                           bool allow_single) {
  uint16_t cnt[16];
  for (int l = 0; l < 16; l++) cnt[l] = 0;
  for (int s = 0; s < n; s++) cnt[lens[s]]++;
  cnt[0] = 0;
  int left = 1, maxl = 0;
  for (int l = 1; l <= 15; l++) {
    left <<= 1;
    left -= cnt[l];
    if (left < 0) return -1;
    if (cnt[l]) maxl = l;
  }
  if (maxl > 0 && left > 0 && !(allow_single && maxl == 1)) return -1;
  uint32_t code = 0, off = 0;
  uint16_t nxt[16];
  for (int l = 0; l < 16; l++) {
    h.first[l] = (uint16_t)code;
    h.count[l] = l ? cnt[l] : 0;
    h.offs[l] = (uint16_t)off;
    nxt[l] = (uint16_t)off;
    if (l) {
      off += cnt[l];
      code = (code + cnt[l]) << 1;
    }
  }
  for (int s = 0; s < n; s++)
    if (lens[s]) sym_out[nxt[lens[s]]++] = (SymT)s;
  return 0;
}

// Root-table entry for window `e` (root bits, LSB-first): canonical decode restricted to
// lengths <= root; a longer code gives an entry with nbits 0 (slow path); no code gives K_BAD.
DQI_INLINE uint32_t root_entry_ll(uint32_t e, const HuffCanon& h, const uint16_t* lsym) {
  const uint32_t r = bitrev(e, LB);
  for (int l = 1; l <= LB; l++) {
    const uint32_t c = r >> (LB - l);
    const uint32_t d = c - h.first[l];
    if (d < h.count[l]) return ll_entry(lsym[h.offs[l] + d], (uint32_t)l);
  }
  return mk_entry(0, 0, K_LIT, 0);  // slow path (or invalid: decided there)
}
DQI_INLINE uint32_t root_entry_d(uint32_t e, const HuffCanon& h, const uint8_t* dsym) {
  const uint32_t r = bitrev(e, DB);
  for (int l = 1; l <= DB; l++) {
    const uint32_t c = r >> (DB - l);
    const uint32_t d = c - h.first[l];
    if (d < h.count[l]) return d_entry(dsym[h.offs[l] + d], (uint32_t)l);
  }
  return mk_entry(0, 0, K_LEN, 0);
}

// Slow path: full entry for a litlen / distance code longer than the root (nbits 10..15), or
// K_BAD with nbits 1 when the window matches no code.
DQI_INLINE uint32_t slow_entry_ll(uint32_t bits, const HuffCanon& h, const uint16_t* lsym) {
  int l = 0;
  const int k = canon_decode(bits, h, LB + 1, &l);
  if (k < 0) return mk_entry(1, 0, K_BAD, 0);
  return ll_entry(lsym[k], (uint32_t)l);
}
DQI_INLINE uint32_t slow_entry_d(uint32_t bits, const HuffCanon& h, const uint8_t* dsym) {
  int l = 0;
  const int k = canon_decode(bits, h, DB + 1, &l);
  if (k < 0) return mk_entry(1, 0, K_BAD, 0);
  return d_entry(dsym[k], (uint32_t)l);
}

// Fixed Huffman code lengths (RFC 1951 3.2.6): 288 litlen + 32 distance.
DQI_INLINE uint8_t fixed_len(int i) {
  if (i < 144) return 8;
  if (i < 256) return 9;
  if (i < 280) return 7;
  if (i < 288) return 8;
  return 5;
}

}  // namespace dqi
