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
// One 256-thread workgroup per block, the block's bytes in LDS.  Match candidates first: the
// positions are walked in stripes of 256 (one per thread); each position reads, from an LDS table
// keyed by a hash of its next 3 bytes, the last position of an earlier stripe with that hash (its
// hash-chain link, kept in global scratch), then the stripe's positions update the table.  Lane t
// then owns bytes [255 t, 255 t + 255) and parses them greedily on its own: at each position the
// longest match of >= 3 bytes among the previous SHORT bytes and the first CHAIN links of its hash
// chain, clamped to its segment's end, so lanes never wait for each other.  Symbols are coded
// with the fixed Huffman code (BTYPE 01): a lane's bit count is known as it goes, so each lane
// stages its bits in its own global-memory slot; an exclusive scan of the counts places every
// lane's bits, which are OR-ed into the LDS image of the block (the input is dead by then) and
// stored with 16-byte writes.  A block whose code would not fit BSIZE is stored (BTYPE 00).
// CRC32: per-lane table CRC over the segment, combined with x^(8 n) mod P multipliers.
#include "dq_internal.h"

#include <mutex>

namespace dq {
namespace {

constexpr int DWG = 256;                 // threads per block
constexpr int BLK_U = 65280;             // htsjdk DEFAULT_UNCOMPRESSED_BLOCK_SIZE
constexpr int SEG = BLK_U / DWG;         // 255 bytes per lane
constexpr int SHORT = 8;                 // distances 1..SHORT always tried
constexpr int CHAIN = 6;                 // hash-chain links tried
constexpr int HBITS = 11;                // LDS head table: 2048 entries
constexpr int MAXM = 258;
constexpr int SLOT_WORDS = 80;           // staged bits per lane: <= 255 * 9 + 10 bits
constexpr int MAX_DEFLATE = 65536 - 26;  // BSIZE limit: 18-byte header + payload + 8 trailer

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

struct BitOut {
  uint32_t* w;  // staging slot
  uint64_t acc;
  int n;        // bits in acc
  int words;
  __device__ void put(uint32_t v, int len) {
    acc |= (uint64_t)v << n;
    n += len;
    if (n >= 32) {
      w[words++] = (uint32_t)acc;
      acc >>= 32;
      n -= 32;
    }
  }
  __device__ int flush() {  // total bits
    const int bits = words * 32 + n;
    if (n > 0) w[words] = (uint32_t)acc;
    return bits;
  }
};

struct alignas(16) DLds {
  uint8_t in[65536 + 16];     // the block's bytes; later the deflate image (<= 65510 bytes)
  uint32_t crc_t[256];
  uint32_t lane_bits[DWG];
  uint32_t lane_crc[DWG];
  int32_t head[1 << HBITS];
  int32_t misc[8];
};

__device__ inline uint32_t hash3(const uint8_t* in, int p) {
  const uint32_t v = (uint32_t)in[p] | ((uint32_t)in[p + 1] << 8) | ((uint32_t)in[p + 2] << 16);
  return (v * 2654435761u) >> (32 - HBITS);
}

__global__ __launch_bounds__(DWG) void bgzf_deflate_kernel(const uint8_t* __restrict__ src,
                                                           int64_t n_in, int64_t blk0,
                                                           int64_t nblk, uint32_t* __restrict__ stage,
                                                           uint16_t* __restrict__ link,
                                                           uint8_t* __restrict__ out_slots,
                                                           int32_t* __restrict__ out_size) {
  __shared__ DLds L;
  const int64_t b = (int64_t)blockIdx.x;  // block within this launch
  if (b >= nblk) return;
  const int t = threadIdx.x;
  const int64_t base = (blk0 + b) * (int64_t)BLK_U;
  const int n = (int)min<int64_t>(BLK_U, n_in - base);
  // load (16-byte loads where aligned)
  for (int i = t; i < 256; i += DWG) L.crc_t[i] = c_dcrc[i];
  for (int i = t; i < (1 << HBITS); i += DWG) L.head[i] = -1;
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
  }
  __syncthreads();
  const int s0 = min(n, t * SEG), s1 = min(n, s0 + SEG);
  // ---- CRC32 of the segment (raw register, init 0)
  {
    uint32_t c = 0;
    for (int i = s0; i < s1; i++) c = L.crc_t[(c ^ L.in[i]) & 0xff] ^ (c >> 8);
    L.lane_crc[t] = gf2_mul(x8n((uint32_t)(n - s1)), c);
  }
  // ---- hash-chain links: stripe r = positions [256 r, 256 r + 256), one per thread
  uint16_t* lk = link + b * 65536;
  for (int r = 0; r * DWG < n; r++) {
    const int p = r * DWG + t;
    uint32_t h = 0;
    int q = -1;
    if (p + 3 <= n) {
      h = hash3(L.in, p);
      q = L.head[h];
    }
    if (p < n) lk[p] = q < 0 ? (uint16_t)0xffff : (uint16_t)q;
    __syncthreads();
    if (p + 3 <= n) atomicMax(&L.head[h], p);
    __syncthreads();
  }
  __threadfence_block();
  __syncthreads();
  // ---- greedy LZ77 over the segment, fixed Huffman into the lane's staging slot
  BitOut bo{stage + ((int64_t)b * DWG + t) * SLOT_WORDS, 0, 0, 0};
  if (t == 0) bo.put(3u, 3);  // BFINAL = 1, BTYPE = 01
  for (int p = s0; p < s1;) {
    int best = 0, bd = 0;
    if (p + 3 <= s1) {
      const uint8_t c0 = L.in[p], c1 = L.in[p + 1], c2 = L.in[p + 2];
      const int lim = min(MAXM, s1 - p);
      auto try_q = [&](int q) {
        if (L.in[q] != c0 || L.in[q + 1] != c1 || L.in[q + 2] != c2) return;
        int l = 3;
        while (l < lim && L.in[q + l] == L.in[p + l]) l++;
        if (l > best) {
          best = l;
          bd = p - q;
        }
      };
      for (int d = 1; d <= SHORT && d <= p && best < lim; d++) try_q(p - d);
      // links were stored by other threads of this workgroup: read past the L1 (glc)
      const volatile uint16_t* vlk = lk;
      int q = vlk[p];
      // links only go back: stop at DEFLATE's 32 KiB window
      for (int k = 0; k < CHAIN && q != 0xffff && p - q <= 32768 && best < lim; k++) {
        if (p - q > SHORT) try_q(q);
        q = vlk[q];
      }
    }
    if (best >= 3) {
      int sym, nx, xv;
      len_code(best, sym, nx, xv);
      uint32_t code;
      int cl;
      fixed_ll(sym, code, cl);
      bo.put(code, cl);
      if (nx) bo.put((uint32_t)xv, nx);
      int ds, dnx, dxv;
      dist_code(bd, ds, dnx, dxv);
      bo.put(rev((uint32_t)ds, 5), 5);
      if (dnx) bo.put((uint32_t)dxv, dnx);
      p += best;
    } else {
      uint32_t code;
      int cl;
      fixed_ll(L.in[p], code, cl);
      bo.put(code, cl);
      p++;
    }
  }
  // the lane holding the block's last byte ends the deflate block (lane 0 for an empty block)
  const int last_lane = n > 0 ? (n - 1) / SEG : 0;
  if (t == last_lane) bo.put(0u, 7);  // end of block (256: seven 0 bits)
  L.lane_bits[t] = (uint32_t)bo.flush();
  __syncthreads();
  // ---- exclusive scan of lane bit counts (one wave), CRC fold
  if (t < 64) {
    uint32_t v[4], s = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      v[k] = L.lane_bits[4 * t + k];
      s += v[k];
    }
    uint32_t inc = s;
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(inc, d, 64);
      if (t >= d) inc += y;
    }
    uint32_t off = inc - s;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      L.lane_bits[4 * t + k] = off;  // now: bit offset of lane 4t+k
      off += v[k];
    }
    if (t == 63) L.misc[0] = (int32_t)inc;  // total bits
    uint32_t c = L.lane_crc[4 * t] ^ L.lane_crc[4 * t + 1] ^ L.lane_crc[4 * t + 2] ^ L.lane_crc[4 * t + 3];
    for (int o = 32; o >= 1; o >>= 1) c ^= __shfl_xor(c, o, 64);
    if (t == 0) L.misc[1] = (int32_t)(c ^ gf2_mul(x8n((uint32_t)n), 0xffffffffu) ^ 0xffffffffu);
  }
  __syncthreads();
  const uint32_t total_bits = (uint32_t)L.misc[0];
  const int dbytes = (int)((total_bits + 7) / 8);
  uint8_t* o = out_slots + b * 65536;
  const uint32_t crc = (uint32_t)L.misc[1];
  // stored when the code is no shorter than the bytes themselves (and always when it would not fit)
  const bool stored = dbytes > min(MAX_DEFLATE, n + 5);
  int payload;
  if (!stored) {
    // ---- place every lane's bits into the LDS image (the input is dead now)
    uint32_t* img = reinterpret_cast<uint32_t*>(L.in);
    __syncthreads();
    for (int i = t; i < (int)(sizeof(L.in) / 4); i += DWG) img[i] = 0;
    __syncthreads();
    {
      const uint32_t off = L.lane_bits[t];
      const uint32_t nb = (t == DWG - 1 ? total_bits : L.lane_bits[t + 1]) - off;
      const uint32_t* sw = stage + ((int64_t)b * DWG + t) * SLOT_WORDS;
      const uint32_t nw = (nb + 31) / 32, sh = off & 31, w0 = off >> 5;
      for (uint32_t k = 0; k < nw; k++) {
        uint32_t v = sw[k];
        const uint32_t rem = nb - 32 * k;
        if (rem < 32) v &= (1u << rem) - 1u;
        atomicOr(&img[w0 + k], v << sh);
        if (sh) atomicOr(&img[w0 + k + 1], v >> (32 - sh));
      }
    }
    __syncthreads();
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
size_t bgzf_stage_bytes(int64_t nblk) { return (size_t)nblk * DWG * SLOT_WORDS * 4; }

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
                         hipStream_t s) {
  if (nblk <= 0) return;
  hipLaunchKernelGGL(bgzf_deflate_kernel, dim3((unsigned)nblk), dim3(DWG), 0, s, src, n_in, blk0, nblk,
                     stage, link, out_slots, out_size);
}

void launch_bgzf_pack(const uint8_t* slots, const int32_t* size, const int64_t* off, int64_t nblk,
                      uint8_t* out, hipStream_t s) {
  if (nblk <= 0) return;
  hipLaunchKernelGGL(bgzf_pack_kernel, dim3((unsigned)nblk), dim3(256), 0, s, slots, size, off, nblk,
                     out);
}

}  // namespace dq
