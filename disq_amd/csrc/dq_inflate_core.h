// dq_inflate_core.h -- DEFLATE (RFC 1951) primitives of the inflate kernel (dq_inflate3.hip):
// bit reversal, the canonical description of a Huffman code (the slow path for codes longer than
// the decode tables' root) and the fixed code lengths.  The __HIPCC__ guards only let host code
// (unit checks) compile the same primitives.
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

struct HuffCanon {       // one alphabet's canonical description (for codes longer than the root)
  uint16_t first[16];    // first canonical code of length l
  uint16_t count[16];    // number of codes of length l
  uint16_t offs[16];     // index in the sorted symbol list of the first code of length l
};

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

// Fixed Huffman code lengths (RFC 1951 3.2.6): 288 litlen + 32 distance.
DQI_INLINE uint8_t fixed_len(int i) {
  if (i < 144) return 8;
  if (i < 256) return 9;
  if (i < 280) return 7;
  if (i < 288) return 8;
  return 5;
}

}  // namespace dqi
