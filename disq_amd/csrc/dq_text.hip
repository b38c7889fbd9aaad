// dq_text.hip -- BGZF text (VCF) path: the lines Hadoop's TextInputFormat returns per split of a
// BGZF-compressed text file read through Disq's splittable codecs.
//
// Reference behaviour (restated literally in oracle/disq_oracle.c, dqo_text_split_lines):
//   BGZFCodec.createInputStream (D/impl/formats/bgzf/BGZFCodec.java:57-68): the split's stream
//     starts at adjustedStart = guessNextBGZFPos(start, end).pos (end when there is none);
//   BGZFSplitCompressionInputStream (BGZFSplitCompressionInputStream.java:14-106): reads never
//     cross a block; crossing one returns a single byte of the next block and only then advertises
//     getPos = (that block's address) + 1;
//   Hadoop 2.7 LineRecordReader over CompressedSplitLineReader, 4096-byte fills: the first line is
//     thrown away unless adjustedStart == 0, and another line is read while getPos <= end (or one
//     more when a CR ... LF pair straddled a fill).
// Characterisation used here, on the resident decompressed stream U (kernels 1-2 inflate it):
//   * terminators: LF, CR LF, or a lone CR (LineReader.readDefaultLine); line k starts after
//     terminator k - 1;
//   * before reading line k the reader has fetched up to the end of the fill holding the byte it
//     last examined -- the line's own terminator end, or for a lone CR the byte after it -- so
//     getPos <= end  <=>  that byte lies before block B1, the first block after B0 with
//     address >= end (getPos of block B0 itself is its address);
//   * the extra line: needAdditionalRecord is the value set by the last fill that started right
//     after a CR (fills: B0 at U0 + 4096 m; later blocks at U_b, then U_b + 1 + 4096 m).
#include "dq_internal.h"

#include <algorithm>

namespace dq {
namespace {

constexpr int TT = 256;           // threads per terminator-scan workgroup
constexpr int TBY = 32;           // bytes per thread
constexpr int TILE = TT * TBY;    // 8 KiB of U per workgroup
constexpr int FILL = 4096;        // io.file.buffer.size (core-default.xml), LineReader buffer

// Terminator-end mask of the 32 bytes at x0 (bit i: byte x0 + i ends a line).  U holds >= 256
// readable zero bytes past ulen.
__device__ inline uint32_t term_mask(const uint8_t* __restrict__ U, int64_t ulen, int64_t x0) {
  if (x0 >= ulen) return 0u;
  const uint4 a = *reinterpret_cast<const uint4*>(U + x0);
  const uint4 b = *reinterpret_cast<const uint4*>(U + x0 + 16);
  const uint8_t nxt = U[x0 + 32];
  const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  uint32_t lf = 0, cr = 0;
#pragma unroll
  for (int i = 0; i < 32; i++) {
    const uint8_t c = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
    lf |= (uint32_t)(c == '\n') << i;
    cr |= (uint32_t)(c == '\r') << i;
  }
  // a CR followed by LF is the first half of CR LF; the byte after the window is `nxt`
  const uint32_t lf_next = (lf >> 1) | ((uint32_t)(nxt == '\n') << 31);
  uint32_t m = lf | (cr & ~lf_next);
  const int64_t valid = ulen - x0;
  if (valid < 32) {
    m &= (1u << valid) - 1u;
    // a CR as the stream's last byte ends a line (the zero pad is not an LF)
  }
  return m;
}

template <bool EMIT>
__global__ __launch_bounds__(TT) void text_terms_kernel(const uint8_t* __restrict__ U, int64_t ulen,
                                                        int32_t* __restrict__ tile_count,
                                                        const int64_t* __restrict__ tile_off,
                                                        int64_t* __restrict__ term_pos) {
  __shared__ int32_t wsum[TT / 64];
  const int64_t x0 = (int64_t)blockIdx.x * TILE + (int64_t)threadIdx.x * TBY;
  const uint32_t m = term_mask(U, ulen, x0);
  const int c = __popc(m);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // wave inclusive scan
  int inc = c;
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(inc, d, 64);
    if (lane >= d) inc += y;
  }
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();
  if (!EMIT) {
    if (threadIdx.x == 0) {
      int t = 0;
      for (int w = 0; w < TT / 64; w++) t += wsum[w];
      tile_count[blockIdx.x] = t;
    }
    return;
  }
  int base = 0;
  for (int w = 0; w < wv; w++) base += wsum[w];
  int64_t o = tile_off[blockIdx.x] + base + inc - c;
  uint32_t mm = m;
  while (mm) {
    const int i = __ffs(mm) - 1;
    mm &= mm - 1;
    term_pos[o++] = x0 + i;
  }
}

__device__ inline int64_t lb_i64(const int64_t* a, int64_t n, int64_t v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

struct Lines {
  const uint8_t* U;
  int64_t ulen;
  const int64_t* term;  // terminator end positions, ascending
  int64_t nterm;
  int64_t nl;           // lines
  __device__ int64_t start(int64_t k) const { return k == 0 ? 0 : term[k - 1] + 1; }
  // the byte the reader last examined before reading line k >= 1
  __device__ int64_t examined(int64_t k) const {
    const int64_t u = term[k - 1] + 1;
    return U[u - 1] == '\r' ? u : u - 1;
  }
};

// Per block: the last fill start f (grid of a block read after the split's first block:
// U_b, U_b + 1 + 4096 m) with U[f - 1] == CR, or -1.
__global__ void text_cr_fills_kernel(const uint8_t* __restrict__ U, const int64_t* __restrict__ uoff,
                                     const int32_t* __restrict__ blk_us, int64_t nblk,
                                     int64_t* __restrict__ last_cr_fill) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblk) return;
  const int64_t ub = uoff[b], n = blk_us[b];
  int64_t r = -1;
  if (n > 0) {
    if (ub > 0 && U[ub - 1] == '\r') r = ub;
    for (int64_t f = ub + 1; f < ub + n; f += FILL)
      if (U[f - 1] == '\r') r = f;
  }
  last_cr_fill[b] = r;
}

// One thread per split: the line index range [k0, k1) it reads.
__global__ void text_plan_kernel(const Cand* __restrict__ cand, const int64_t* __restrict__ ncand,
                                 const int64_t* __restrict__ blk_pos,
                                 const int32_t* __restrict__ blk_us,
                                 const int64_t* __restrict__ uoff, int64_t nblk, int64_t flen,
                                 const uint8_t* __restrict__ U, int64_t ulen,
                                 const int64_t* __restrict__ term, int64_t nterm,
                                 const int64_t* __restrict__ last_cr_fill,
                                 TextPlan* __restrict__ plans, int64_t nsplit) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nsplit) return;
  TextPlan& P = plans[i];
  P.k0 = P.k1 = 0;
  P.b0 = -1;
  P.status = 0;
  P.bom = 0;
  const int64_t s = P.split_start, e = P.split_end, nc = *ncand;
  Lines L{U, ulen, term, nterm, 0};
  L.nl = nterm + ((nterm == 0 ? ulen > 0 : term[nterm - 1] + 1 < ulen) ? 1 : 0);
  // ---- BGZFCodec.createInputStream: guessNextBGZFPos(start, end) (BgzfBlockGuesser.java:76-149)
  int64_t A = -1;
  {
    int64_t p = s;
    for (;;) {
      int64_t lo = 0, hi = nc;
      while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (cand[mid].pos < p) lo = mid + 1;
        else hi = mid;
      }
      if (lo >= nc) break;
      const Cand c = cand[lo];
      if (c.pos != p && c.pos >= e) break;
      if (c.valid == 1) {
        A = c.pos;
        break;
      }
      if (c.valid == 2) break;
      p = c.pos + 4;
    }
  }
  const bool guessed = A >= 0;
  if (!guessed) A = e;  // adjustedStart = end
  const int64_t j = lb_i64(blk_pos, nblk, A);
  if (j >= nblk || blk_pos[j] != A) {
    // the stream would start inside a block: the reference fails reading it, except at the end
    // of the file (an empty stream)
    if (!guessed && A >= flen) return;
    P.status = guessed ? ST_BAD_HEADER : ST_TEXT_START;
    return;
  }
  P.b0 = j;
  if (blk_us[j] == 0) return;  // an empty block: available() == 0, end of stream
  const int64_t U0 = uoff[j];
  // ---- LineRecordReader.initialize: unless the stream starts at 0, drop the first line
  int64_t k0;
  if (A == 0) {
    k0 = 0;
  } else {
    const int64_t t = lb_i64(term, nterm, U0);
    if (t >= nterm) return;  // the dropped line runs to the end
    k0 = t + 1;
    if (k0 >= L.nl) return;
    if (A > e) return;       // readLine saw getPos > end: finished before the first record
  }
  // ---- the lines read while getPos <= end: examined byte before block B1
  int64_t b1 = lb_i64(blk_pos, nblk, e);
  if (b1 <= j) b1 = j + 1;
  const int64_t lim = b1 < nblk ? uoff[b1] : INT64_MAX;
  int64_t lo = k0 == 0 ? 1 : k0, hi = L.nl;  // line 0 (stream start) is read unconditionally
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (L.examined(mid) < lim) lo = mid + 1;
    else hi = mid;
  }
  int64_t k1 = lo;
  // ---- one more line if the last fill after a CR did not start with LF
  if (k1 < L.nl) {
    const int64_t X = L.examined(k1);
    // block holding X
    int64_t bx = lb_i64(uoff, nblk, X + 1) - 1;
    int64_t f = -1;
    if (bx == j) {
      for (int64_t g = U0 + FILL; g <= X; g += FILL)
        if (U[g - 1] == '\r') f = g;
    } else {
      const int64_t ub = uoff[bx];
      if (U[ub - 1] == '\r') f = ub;
      for (int64_t g = ub + 1; g <= X; g += FILL)
        if (U[g - 1] == '\r') f = g;
      for (int64_t b = bx - 1; f < 0 && b > j; b--) f = last_cr_fill[b];
      if (f < 0)
        for (int64_t g = U0 + FILL; g < U0 + blk_us[j]; g += FILL)
          if (U[g - 1] == '\r') f = g;
    }
    if (f >= 0 && U[f] != '\n') k1++;
  }
  // ---- skipUtfByteOrderMark (line 0 only): a value starting EF BB BF loses those bytes, and a
  //      line of only them with no terminator is no record (newSize 0)
  if (k0 == 0 && k1 > 0) {
    int64_t z = ulen, consumed = ulen;
    if (nterm > 0) {
      const int64_t te = term[0];
      z = (U[te] == '\n' && te > 0 && U[te - 1] == '\r') ? te - 1 : te;
      consumed = te + 1;
    }
    if (z >= 3 && U[0] == 0xEF && U[1] == 0xBB && U[2] == 0xBF) {
      P.bom = 1;
      if (consumed == 3) k1 = 0;
    }
  }
  P.k0 = k0;
  P.k1 = k1 < k0 ? k0 : k1;
}

// Values of the listed lines: offset, length (terminator excluded, BOM stripped from line 0 when
// flagged), hash of the value bytes, keep flag (drop '#' lines when asked).  The hash is the
// record hash of DESIGN.md section 4 (8-byte little-endian words, zero padded, keyed by index):
// a line of up to TV_LONG bytes is hashed by its thread from aligned dword loads (one byte-align
// per half word); a longer line is left to text_long_hash_kernel, a wave per line.
constexpr int64_t TV_LONG = 2048;
__device__ inline uint32_t tv_funnel(uint32_t lo, uint32_t hi, uint32_t sh) {  // (hi:lo) >> 8 sh
  return __builtin_amdgcn_alignbyte(hi, lo, sh);
}
// word k of the value at byte a (len bytes), zero padded past len
__device__ inline uint64_t tv_word(const uint32_t* __restrict__ U32, int64_t a, int64_t len, int64_t k) {
  const int64_t wi = (a >> 2) + 2 * k;
  const uint32_t sh = (uint32_t)(a & 3);
  const uint32_t w0 = U32[wi], w1 = U32[wi + 1], w2 = U32[wi + 2];
  uint64_t w = ((uint64_t)tv_funnel(w1, w2, sh) << 32) | tv_funnel(w0, w1, sh);
  const int64_t rem = len - 8 * k;
  if (rem < 8) w &= (1ull << (8 * rem)) - 1;
  return w;
}
__global__ void text_values_kernel(const uint8_t* __restrict__ U, int64_t ulen,
                                   const int64_t* __restrict__ term, int64_t nterm,
                                   const int64_t* __restrict__ idx, int64_t n, int32_t bom,
                                   int32_t drop_hash, int64_t* __restrict__ vstart,
                                   int32_t* __restrict__ vlen, uint64_t* __restrict__ hash,
                                   uint8_t* __restrict__ keep) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const int64_t k = idx[t];
  int64_t a = k == 0 ? 0 : term[k - 1] + 1;
  int64_t z;
  if (k < nterm) {
    const int64_t te = term[k];
    z = te;  // exclusive end of the value
    if (U[te] == '\n' && te > a && U[te - 1] == '\r') z = te - 1;
  } else {
    z = ulen;
  }
  if (k == 0 && bom) a += 3;
  const int64_t len = z - a;
  vstart[t] = a;
  vlen[t] = (int32_t)len;
  keep[t] = (uint8_t)!(drop_hash && len > 0 && U[a] == '#');
  if (len > TV_LONG) return;  // text_long_hash_kernel
  const uint32_t* U32 = reinterpret_cast<const uint32_t*>(U);  // U: 256 bytes of slack past ulen
  uint64_t h = (uint64_t)len * DQ_K_LEN;
  const int64_t nw = (len + 7) / 8;
  for (int64_t w = 0; w < nw; w++) h += dq_mix64(tv_word(U32, a, len, w) ^ ((uint64_t)(w + 1) * DQ_K_WORD));
  hash[t] = dq_mix64(h);
}

// Lines longer than TV_LONG: one wave per line (a grid-stride over the lines' lengths), lane l
// hashing words l, l + 64, ... (the word sum is order-free), summed across the wave.
__global__ __launch_bounds__(256) void text_long_hash_kernel(const uint8_t* __restrict__ U,
                                                             const int64_t* __restrict__ vstart,
                                                             const int32_t* __restrict__ vlen,
                                                             int64_t n, uint64_t* __restrict__ hash) {
  const uint32_t* U32 = reinterpret_cast<const uint32_t*>(U);
  const int lane = threadIdx.x & 63;
  const int64_t nwave = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t t = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); t < n; t += nwave) {
    const int64_t len = vlen[t];
    if (len <= TV_LONG) continue;  // wave-uniform
    const int64_t a = vstart[t];
    uint64_t part = 0;
    const int64_t nw = (len + 7) / 8;
    for (int64_t w = lane; w < nw; w += 64) part += dq_mix64(tv_word(U32, a, len, w) ^ ((uint64_t)(w + 1) * DQ_K_WORD));
    for (int o = 32; o >= 1; o >>= 1) {
      const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)part, o, 64);
      const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(part >> 32), o, 64);
      part += ((uint64_t)hi << 32) | lo;
    }
    if (lane == 0) hash[t] = dq_mix64((uint64_t)len * DQ_K_LEN + part);
  }
}

// Line values gathered into a compact byte buffer: one wave per line.
__global__ __launch_bounds__(256) void text_gather_kernel(const uint8_t* __restrict__ U,
                                                          const int64_t* __restrict__ vstart,
                                                          const int32_t* __restrict__ vlen,
                                                          const int64_t* __restrict__ kept,
                                                          const int64_t* __restrict__ out_off,
                                                          int64_t n, uint8_t* __restrict__ out) {
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= n) return;
  const int64_t t = kept[w];
  const int64_t a = vstart[t], o = out_off[w];
  const int32_t len = vlen[t];
  for (int32_t x = threadIdx.x & 63; x < len; x += 64) out[o + x] = U[a + x];
}

// Partition p's kept lines: positions [koff[out_off[p]], koff[out_off[p + 1]]) of the kept list.
__global__ void text_parts_kernel(const int64_t* __restrict__ out_off, const int64_t* __restrict__ koff,
                                  int64_t nsplit, PartRange* __restrict__ parts) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= nsplit) return;
  parts[p].begin = koff[out_off[p]];
  parts[p].end = koff[out_off[p + 1]];
  parts[p].digest = 0;
}

// Kept lines' offset, length and hash in kept order (what crosses PCIe on export).
__global__ void text_export_kernel(const int64_t* __restrict__ kept, int64_t n,
                                   const int64_t* __restrict__ vstart, const int32_t* __restrict__ vlen,
                                   const uint64_t* __restrict__ hash, int64_t* __restrict__ o_start,
                                   int32_t* __restrict__ o_len, uint64_t* __restrict__ o_hash) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t t = kept[i];
  o_start[i] = vstart[t];
  o_len[i] = vlen[t];
  o_hash[i] = hash[t];
}

// VcfSource's OverlapDetector filter (D/impl/formats/vcf/VcfSource.java:108-111) on the raw line:
// VariantContext contig = CHROM, start = POS, end = POS + len(REF) - 1, or the INFO END value when
// present (htsjdk AbstractVCFCodec); kept when some interval of that contig overlaps
// [start, end] (1-based, closed).  Intervals per contig are sorted by start with a running
// maximum of their ends, so one binary search answers overlapsAny.
__device__ inline int64_t vcf_field_end(const uint8_t* U, int64_t x, int64_t z) {
  while (x < z && U[x] != '\t') x++;
  return x;
}
__device__ inline int64_t vcf_int(const uint8_t* U, int64_t x, int64_t z, bool* ok) {
  int64_t v = 0;
  bool any = false, neg = false;
  if (x < z && (U[x] == '-' || U[x] == '+')) neg = U[x++] == '-';
  while (x < z && U[x] >= '0' && U[x] <= '9') {
    v = v * 10 + (U[x++] - '0');
    any = true;
  }
  *ok = any;
  return neg ? -v : v;
}

__global__ void vcf_overlap_kernel(const uint8_t* __restrict__ U, const int64_t* __restrict__ vstart,
                                   const int32_t* __restrict__ vlen, int64_t n,
                                   const uint8_t* __restrict__ names, const int32_t* __restrict__ noff,
                                   int32_t nnames, const int32_t* __restrict__ ivbeg,
                                   const int32_t* __restrict__ ivstart,
                                   const int32_t* __restrict__ ivmaxend, uint8_t* __restrict__ keep) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n || !keep[t]) return;
  const int64_t a = vstart[t], z = a + vlen[t];
  const int64_t c1 = vcf_field_end(U, a, z);
  const int64_t clen = c1 - a;
  int cid = -1;
  for (int i = 0; i < nnames && cid < 0; i++) {
    if (noff[i + 1] - noff[i] != clen) continue;
    bool eq = true;
    for (int64_t k = 0; k < clen && eq; k++) eq = U[a + k] == names[noff[i] + k];
    if (eq) cid = i;
  }
  uint8_t k = 0;
  if (cid >= 0 && c1 < z) {
    bool ok = false;
    const int64_t pos = vcf_int(U, c1 + 1, z, &ok);
    const int64_t f2 = vcf_field_end(U, c1 + 1, z);           // end of POS
    const int64_t f3 = vcf_field_end(U, f2 + 1, z);           // end of ID
    const int64_t f4 = vcf_field_end(U, f3 + 1, z);           // end of REF
    int64_t end = pos + (f4 - (f3 + 1)) - 1;
    const int64_t f5 = vcf_field_end(U, f4 + 1, z);           // ALT
    const int64_t f6 = vcf_field_end(U, f5 + 1, z);           // QUAL
    const int64_t f7 = vcf_field_end(U, f6 + 1, z);           // FILTER
    const int64_t f8 = vcf_field_end(U, f7 + 1, z);           // INFO
    for (int64_t x = f7 + 1; x + 4 <= f8; x++) {              // END= at the start of a key
      if ((x == f7 + 1 || U[x - 1] == ';') && U[x] == 'E' && U[x + 1] == 'N' && U[x + 2] == 'D' &&
          U[x + 3] == '=') {
        bool ok2 = false;
        const int64_t e = vcf_int(U, x + 4, f8, &ok2);
        if (ok2) end = e;
        break;
      }
    }
    if (ok) {
      int lo = ivbeg[cid], hi = ivbeg[cid + 1];  // last interval with start <= end
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if ((int64_t)ivstart[mid] <= end) lo = mid + 1;
        else hi = mid;
      }
      if (lo > ivbeg[cid] && (int64_t)ivmaxend[lo - 1] >= pos) k = 1;
    }
  }
  keep[t] = k;
}

}  // namespace

void launch_vcf_overlap(const uint8_t* U, const int64_t* vstart, const int32_t* vlen, int64_t n,
                        const uint8_t* names, const int32_t* noff, int32_t nnames,
                        const int32_t* ivbeg, const int32_t* ivstart, const int32_t* ivmaxend,
                        uint8_t* keep, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(vcf_overlap_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, U,
                     vstart, vlen, n, names, noff, nnames, ivbeg, ivstart, ivmaxend, keep);
}

void launch_text_parts(const int64_t* out_off, const int64_t* koff, int64_t nsplit, PartRange* parts,
                       hipStream_t s) {
  if (nsplit <= 0) return;
  hipLaunchKernelGGL(text_parts_kernel, dim3((unsigned)((nsplit + 255) / 256)), dim3(256), 0, s,
                     out_off, koff, nsplit, parts);
}

void launch_text_export(const int64_t* kept, int64_t n, const int64_t* vstart, const int32_t* vlen,
                        const uint64_t* hash, int64_t* o_start, int32_t* o_len, uint64_t* o_hash,
                        hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(text_export_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, kept, n,
                     vstart, vlen, hash, o_start, o_len, o_hash);
}

void launch_text_terms(const uint8_t* U, int64_t ulen, int32_t* tile_count, const int64_t* tile_off,
                       int64_t* term_pos, bool emit, hipStream_t s) {
  const int64_t nt = (ulen + TILE - 1) / TILE;
  if (nt <= 0) return;
  if (emit)
    hipLaunchKernelGGL(text_terms_kernel<true>, dim3((unsigned)nt), dim3(TT), 0, s, U, ulen,
                       tile_count, tile_off, term_pos);
  else
    hipLaunchKernelGGL(text_terms_kernel<false>, dim3((unsigned)nt), dim3(TT), 0, s, U, ulen,
                       tile_count, tile_off, term_pos);
}
int64_t text_tiles(int64_t ulen) { return (ulen + TILE - 1) / TILE; }

void launch_text_cr_fills(const uint8_t* U, const int64_t* uoff, const int32_t* blk_us, int64_t nblk,
                          int64_t* last_cr_fill, hipStream_t s) {
  if (nblk <= 0) return;
  hipLaunchKernelGGL(text_cr_fills_kernel, dim3((unsigned)((nblk + 255) / 256)), dim3(256), 0, s, U,
                     uoff, blk_us, nblk, last_cr_fill);
}

void launch_text_plan(const Cand* cand, const int64_t* ncand, const int64_t* blk_pos,
                      const int32_t* blk_us, const int64_t* uoff, int64_t nblk, int64_t flen,
                      const uint8_t* U, int64_t ulen, const int64_t* term, int64_t nterm,
                      const int64_t* last_cr_fill, TextPlan* plans, int64_t nsplit, hipStream_t s) {
  if (nsplit <= 0) return;
  hipLaunchKernelGGL(text_plan_kernel, dim3((unsigned)((nsplit + 63) / 64)), dim3(64), 0, s, cand,
                     ncand, blk_pos, blk_us, uoff, nblk, flen, U, ulen, term, nterm, last_cr_fill,
                     plans, nsplit);
}

void launch_text_values(const uint8_t* U, int64_t ulen, const int64_t* term, int64_t nterm,
                        const int64_t* idx, int64_t n, int32_t bom, int32_t drop_hash,
                        int64_t* vstart, int32_t* vlen, uint64_t* hash, uint8_t* keep,
                        hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(text_values_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, U, ulen,
                     term, nterm, idx, n, bom, drop_hash, vstart, vlen, hash, keep);
  const int64_t nwg = std::min<int64_t>((n + 3) / 4, 4096);  // 4 waves per workgroup
  hipLaunchKernelGGL(text_long_hash_kernel, dim3((unsigned)nwg), dim3(256), 0, s, U, vstart, vlen, n,
                     hash);
}

void launch_text_gather(const uint8_t* U, const int64_t* vstart, const int32_t* vlen,
                        const int64_t* kept, const int64_t* out_off, int64_t n, uint8_t* out,
                        hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(text_gather_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, U, vstart,
                     vlen, kept, out_off, n, out);
}

DQ_CHK_UNIT(text)

}  // namespace dq
