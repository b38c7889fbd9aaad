// dq_kernels.hip -- Kernels 1, 3, 4 and the planning kernels of the BAM read path on gfx950.
//
// Kernel 1  bgzf_scan / chain      replaces BgzfBlockGuesser + BgzfBlockSource
//           (D/impl/formats/bgzf/BgzfBlockGuesser.java:76-149, BgzfBlockSource.java:63-84)
// planning  plan_blocks / first_record   replaces BamSource.getFirstReadInPartition +
//           BamRecordGuesser (D/impl/formats/bam/BamSource.java:110-153,
//           BamRecordGuesser.java:34-194)
// Kernel 3  seg_* / decode_records replaces htsjdk BAMFileIndexIterator + BAMRecordCodec.decode
//           (H/BAMFileReader2.java:1063-1096) and adds the per-record raw-byte hash
// Kernel 4  interval_filter        replaces BAMQueryMultipleIntervalsIteratorFilter
//           (AbstractBinarySamSource.java:86-134 via BamSource.java:177-182)
//
// All of it is integer/byte work bounded by HBM or latency: no MFMA.
#include "dq_internal.h"

namespace dq {
namespace {

__device__ inline uint32_t ld8(const uint8_t* p, int64_t i) { return p[i]; }
__device__ inline uint32_t ld16(const uint8_t* p, int64_t i) { return p[i] | (p[i + 1] << 8); }
__device__ inline int32_t ld32(const uint8_t* p, int64_t i) {
  return (int32_t)(p[i] | (p[i + 1] << 8) | (p[i + 2] << 16) | ((uint32_t)p[i + 3] << 24));
}

#ifdef DQ_REC_TIMING  // dev builds: s_memtime cycles per phase summed over waves (tools/records_timing.py)
__device__ unsigned long long g_rec_tim[8];
#define REC_T(k)                                             \
  do {                                                       \
    const uint64_t now_ = __builtin_amdgcn_s_memtime();      \
    rt_[k] += now_ - rt_last_;                               \
    rt_last_ = now_;                                         \
  } while (0)
#define REC_T_DECL uint64_t rt_[8] = {0, 0, 0, 0, 0, 0, 0, 0}, rt_last_ = __builtin_amdgcn_s_memtime()
#define REC_T_FLUSH                                                                  \
  do {                                                                               \
    if (threadIdx.x == 0)                                                            \
      for (int k_ = 0; k_ < 8; k_++) atomicAdd(&g_rec_tim[k_], (unsigned long long)rt_[k_]); \
  } while (0)
#define REC_T_PARAM , uint64_t (&rt_)[8], uint64_t &rt_last_
#define REC_T_ARG , rt_, rt_last_
#else
#define REC_T_PARAM
#define REC_T_ARG
#define REC_T(k) do {} while (0)
#define REC_T_DECL do {} while (0)
#define REC_T_FLUSH do {} while (0)
#endif

// ------------------------------------------------------------------ Kernel 1: BGZF scan
constexpr uint32_t BGZF_MAGIC = 0x04088b1fu;

// The part of BgzfBlockGuesser.guessNextBGZFPos after a magic match at q
// (BgzfBlockGuesser.java:93-144).  Returns 1 (block), 0 (cancelled: scan resumes at q+4) or
// 2 (an IOException: guessNextBGZFPos returns null).  L = readable bytes.
__device__ int guesser_at(const uint8_t* C, int64_t q, int64_t L, int32_t* cs, int32_t* us) {
  if (q + 12 > L) return 2;
  int64_t xlen = ld16(C, q + 10);
  int64_t p = q + 12;
  const int64_t sub_end = p + xlen;
  while (p < sub_end) {
    if (p + 4 > L) return 2;
    uint32_t id = (uint32_t)ld32(C, p);
    if (id != 0x00024342u) {
      p += 4 + ld16(C, p + 2);
      continue;
    }
    if (p + 6 > L) return 2;
    int64_t bsize = ld16(C, p + 4);
    p += 6;
    while (p < sub_end) {
      if (p + 4 > L) return 2;
      p += 4 + ld16(C, p + 2);
    }
    if (p != sub_end) return 0;
    p += bsize - xlen - 19 + 4;
    if (p < 0 || p + 4 > L) return 2;
    *cs = (int32_t)(p + 4 - q);
    *us = ld32(C, p);
    return 1;
  }
  return 0;
}

// One workgroup of 256 lanes per 16 KiB chunk; each lane tests 16 positions per step with one
// 16-byte coalesced load (+4 look-ahead bytes).  Hits are rare and collected in LDS, then
// written sorted into the chunk's fixed slot range of CAP entries.  Pass 1 (LISTED = false)
// covers every chunk with CAP = SCAN_CAP and lists the chunks with more hits (highly
// compressible data: BGZF blocks of ~100 bytes); pass 2 (LISTED = true) re-scans only those,
// with CAP = SCAN_CAP_BIG slots each (over_map[chunk] = their index).
template <int CAP, bool LISTED>
__global__ __launch_bounds__(256) void bgzf_scan_kernel(const uint8_t* __restrict__ C, int64_t n,
                                                        int64_t L, Cand* __restrict__ slots,
                                                        int32_t* __restrict__ counts,
                                                        int32_t* __restrict__ over_list,
                                                        int32_t* __restrict__ over_map) {
  __shared__ Cand hits[CAP];
  __shared__ int32_t nh;
  const int64_t chunk = LISTED ? (int64_t)over_list[1 + blockIdx.x] : (int64_t)blockIdx.x;
  const int64_t base = chunk * SCAN_CHUNK;
  if (threadIdx.x == 0) nh = 0;
  __syncthreads();
  for (int it = 0; it < SCAN_CHUNK / 4096; it++) {
    int64_t off = base + (int64_t)it * 4096 + threadIdx.x * 16;
    if (off >= n) break;
    // bytes off .. off+19 (C is padded by >= 64 bytes)
    const uint4 v = *reinterpret_cast<const uint4*>(C + off);
    const uint32_t nx = *reinterpret_cast<const uint32_t*>(C + off + 16);
    uint32_t w[5] = {v.x, v.y, v.z, v.w, nx};
#pragma unroll
    for (int k = 0; k < 16; k++) {
      int wi = k >> 2, sb = (k & 3) * 8;
      uint32_t win = sb ? (uint32_t)((((uint64_t)w[wi + 1] << 32) | w[wi]) >> sb) : w[wi];
      if (win == BGZF_MAGIC) {
        int64_t q = off + k;
        if (q + 4 <= L && q < n) {
          int32_t cs = 0, us = 0;
          int r = guesser_at(C, q, L, &cs, &us);
          int slot = atomicAdd(&nh, 1);
          if (slot < CAP) {
            Cand c;
            c.pos = q;
            c.csize = cs;
            c.usize = us;
            c.valid = r == 1 ? 1 : (r == 2 ? 2 : 0);
            c.pad = 0;
            hits[slot] = c;
          }
        }
      }
    }
  }
  __syncthreads();
  int32_t m = nh;
  if (m > CAP) {
    if (threadIdx.x == 0) {
      counts[chunk] = 0;
      if (LISTED) {
        over_list[0] = -1;  // more than SCAN_CAP_BIG magic positions in 16 KiB: unsupported
      } else {
        const int32_t k = atomicAdd(&over_list[0], 1);
        if (k < SCAN_OVER_MAX) over_list[1 + k] = (int32_t)chunk;
      }
    }
    return;
  }
  // rank sort by position
  const int64_t slot0 = LISTED ? (int64_t)blockIdx.x * CAP : chunk * CAP;
  for (int i = threadIdx.x; i < m; i += 256) {
    Cand c = hits[i];
    int rank = 0;
    for (int j = 0; j < m; j++) rank += hits[j].pos < c.pos;
    DQ_CHK(rank < CAP, CHK_K1_SLOT);
    slots[slot0 + rank] = c;
  }
  if (threadIdx.x == 0) {
    counts[chunk] = m;
    if (LISTED) over_map[chunk] = (int32_t)blockIdx.x;
  }
}

__global__ void gather_slots_kernel(const Cand* __restrict__ slots, const int32_t* __restrict__ counts,
                                    const int64_t* __restrict__ offs, int64_t nchunks,
                                    Cand* __restrict__ out, int64_t cap,
                                    const int32_t* __restrict__ over_map, const Cand* __restrict__ big) {
  int64_t ch = blockIdx.x;
  if (ch >= nchunks) return;
  int32_t m = counts[ch];
  int64_t o = offs[ch];
  const int32_t ov = over_map ? over_map[ch] : -1;
  const Cand* src = ov >= 0 ? big + (int64_t)ov * SCAN_CAP_BIG : slots + ch * SCAN_CAP;
  for (int i = threadIdx.x; i < m; i += blockDim.x)
    if (o + i < cap) out[o + i] = src[i];
}

// ------------------------------------------------------------------ scans
// Block-level exclusive scan of 1024 elements per block, then a recursive pass on block sums.
template <typename T>
__global__ __launch_bounds__(1024) void scan_block_kernel(const T* __restrict__ in, int64_t* out,
                                                          int64_t n, int64_t* __restrict__ sums) {
  __shared__ int64_t s[1024];
  int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x;
  int64_t v = i < n ? (int64_t)in[i] : 0;
  s[threadIdx.x] = v;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    int64_t t = threadIdx.x >= o ? s[threadIdx.x - o] : 0;
    __syncthreads();
    s[threadIdx.x] += t;
    __syncthreads();
  }
  if (i < n) out[i] = s[threadIdx.x] - v;
  if (threadIdx.x == 1023) sums[blockIdx.x] = s[1023];
}

__global__ void scan_add_kernel(int64_t* out, int64_t n, const int64_t* __restrict__ sums_scanned) {
  int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x;
  if (i < n) out[i] += sums_scanned[blockIdx.x];
}

template <typename T>
void exclusive_scan(const T* in, int64_t* out, int64_t n, int64_t* tmp, hipStream_t s) {
  // out has n + 1 entries; out[n] = total.  tmp needs >= 2 * ceil(n/1024) + 64 entries.
  if (n <= 0) {
    (void)hipMemsetAsync(out, 0, sizeof(int64_t), s);
    return;
  }
  int64_t nb = (n + 1023) / 1024;
  int64_t* sums = tmp;
  int64_t* sums_sc = tmp + nb + 1;
  hipLaunchKernelGGL(scan_block_kernel<T>, dim3((unsigned)nb), dim3(1024), 0, s, in, out, n, sums);
  if (nb > 1) {
    exclusive_scan<int64_t>(sums, sums_sc, nb, tmp + 2 * nb + 2, s);
    hipLaunchKernelGGL(scan_add_kernel, dim3((unsigned)nb), dim3(1024), 0, s, out, n, sums_sc);
    // total = sums_sc[nb]
    (void)hipMemcpyAsync(out + n, sums_sc + nb, sizeof(int64_t), hipMemcpyDeviceToDevice, s);
  } else {
    (void)hipMemcpyAsync(out + n, sums, sizeof(int64_t), hipMemcpyDeviceToDevice, s);
  }
}

// ------------------------------------------------------------------ chain
// htsjdk reads blocks one after another by BSIZE at header offset 16 and requires XLEN == 6
// (BlockGunzipper.unzipBlock).  Valid guesser candidates must form exactly that chain.
__device__ inline int htsjdk_block(const uint8_t* C, int64_t p, int64_t L, int32_t* cs) {
  if (p + 18 > L) return 0;
  if ((uint32_t)ld32(C, p) != BGZF_MAGIC || ld16(C, p + 10) != 6) return 0;
  int32_t c = (int32_t)ld16(C, p + 16) + 1;
  if (c < 26 || p + c > L) return 0;
  *cs = c;
  return 1;
}

__global__ void valid_flags_kernel(const Cand* __restrict__ cand, const int64_t* __restrict__ ncand,
                                   int32_t* __restrict__ flags) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < *ncand) flags[i] = cand[i].valid == 1;
}

__global__ void chain_kernel(const uint8_t* __restrict__ C, int64_t L, const Cand* __restrict__ cand,
                             const int64_t* __restrict__ ncand, const int64_t* __restrict__ voff,
                             int64_t* __restrict__ blk_pos, int32_t* __restrict__ blk_csize,
                             int32_t* __restrict__ blk_usize, int64_t cap, int64_t* d_nblk,
                             int32_t* d_broken, int32_t eof_in_buf) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t nc = *ncand;
  int64_t nv = voff[nc];
  if (i == 0) *d_nblk = nv;
  if (i >= nc || cand[i].valid != 1) return;
  int64_t k = voff[i];
  if (k >= cap) {
    *d_broken = 1;
    return;
  }
  const Cand c = cand[i];
  int32_t cs;
  if (!htsjdk_block(C, c.pos, L, &cs) || cs != c.csize) {
    *d_broken = 1;
    return;
  }
  blk_pos[k] = c.pos;
  blk_csize[k] = cs;
  blk_usize[k] = c.usize;
  // link to the next valid candidate
  int64_t nextpos = -1;
  for (int64_t j = i + 1; j < nc; j++)
    if (cand[j].valid == 1) {
      nextpos = cand[j].pos;
      break;
    }
  if (nextpos >= 0) {
    if (c.pos + cs != nextpos) *d_broken = 1;
  } else if (eof_in_buf && c.pos + cs != L) {
    *d_broken = 1;
  }
}

__global__ void chain_serial_kernel(const uint8_t* __restrict__ C, int64_t L, int64_t start,
                                    int64_t* __restrict__ blk_pos, int32_t* __restrict__ blk_csize,
                                    int32_t* __restrict__ blk_usize, int64_t cap, int64_t* d_nblk,
                                    int32_t* d_status) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int64_t p = start, n = 0;
  while (p < L) {
    int32_t cs;
    if (!htsjdk_block(C, p, L, &cs)) break;
    if (n >= cap) {
      *d_status = ST_BAD_HEADER;
      break;
    }
    blk_pos[n] = p;
    blk_csize[n] = cs;
    blk_usize[n] = ld32(C, p + cs - 4);
    n++;
    p += cs;
  }
  *d_nblk = n;
}

// ------------------------------------------------------------------ record guesser
// BamRecordGuesser.checkRecordStartInternal (BamRecordGuesser.java:79-194) on the linear stream.
// Returns 1 (start; *next set), 0 (no start), 3 (EOF), 4 (need data beyond the buffer).
__device__ inline int rd_ok(int64_t p, int64_t n, int64_t ulen, int u_is_eof) {
  if (p + n <= ulen) return 0;
  return u_is_eof ? 3 : 4;
}

__device__ int check_internal(const uint8_t* U, int64_t ulen, int u_is_eof, const int32_t* ref_len,
                              int32_t n_ref, int64_t v, int64_t* next) {
  int e;
  if ((e = rd_ok(v, 36, ulen, u_is_eof))) return e;
  int32_t remaining = ld32(U, v);
  int32_t id = ld32(U, v + 4), pos = ld32(U, v + 8);
  if (id < -1 || id >= n_ref || pos < -1) return 0;
  if (id >= 0 && pos > ref_len[id]) return 0;
  int32_t nid = ld32(U, v + 24), npos = ld32(U, v + 28);
  if (nid < -1 || nid >= n_ref || npos < -1) return 0;
  if (nid >= 0 && npos > ref_len[nid]) return 0;
  int32_t name_len = ld32(U, v + 12) & 0xff;
  if (name_len < 2) return 0;
  uint32_t flag_nc = (uint32_t)ld32(U, v + 16);
  int32_t flags = (int32_t)(flag_nc >> 16);
  int32_t n_cig = (int32_t)(flag_nc & 0xffff);
  int32_t cig_len = (int32_t)((uint32_t)n_cig * 4u);
  int32_t l_seq = ld32(U, v + 20);
  int32_t seq_len = (int32_t)((uint32_t)l_seq + (uint32_t)((int32_t)((uint32_t)l_seq + 1u) / 2));
  if ((flags & 4) == 0 && (seq_len == 0 || n_cig == 0)) return 0;
  if ((e = rd_ok(v + 36, name_len, ulen, u_is_eof))) return e;
  if (U[v + 36 + name_len - 1] != 0) return 0;
  for (int i = 0; i < name_len - 1; i += 16) {  // 16 name bytes per round of loads
    uint8_t b16[16];
#pragma unroll
    for (int k = 0; k < 16; k++) b16[k] = i + k < name_len - 1 ? U[v + 36 + i + k] : (uint8_t)'A';
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const int8_t b = (int8_t)b16[k];
      if (!((b >= '!' && b <= '?') || (b >= 'A' && b <= '~'))) return 0;
    }
  }
  int64_t cp = v + 36 + name_len;
  int i = 0;
  // the ops 8 at a time from nine aligned dwords, all loads in flight (a long read's CIGAR has
  // thousands of ops: one dependent byte-load round trip per op made the guesser the planning's
  // critical path); the checks keep the op order
  const uint32_t* U32 = reinterpret_cast<const uint32_t*>(U);
  for (; i + 8 <= n_cig && cp + 32 <= ulen; i += 8, cp += 32) {
    const uint32_t sh = (uint32_t)(cp & 3);
    uint32_t d[9];
#pragma unroll
    for (int k = 0; k < 9; k++) d[k] = U32[(cp >> 2) + k];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const int32_t op = (int32_t)__builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
      if (op == -1) return 3;
      if ((op & 0xf) > 8) return 0;
    }
  }
  for (; i < n_cig; i++) {
    if ((e = rd_ok(cp, 4, ulen, u_is_eof))) return e;
    int32_t op = ld32(U, cp);
    if (op == -1) return 3;
    if ((op & 0xf) > 8) return 0;
    cp += 4;
  }
  int32_t zero_min =
      (int32_t)((uint32_t)32 + (uint32_t)name_len + (uint32_t)cig_len + (uint32_t)seq_len);
  if (remaining >= zero_min) {
    int32_t skip = (int32_t)(4u + (uint32_t)remaining);
    int64_t nv = v;
    if (skip > 0) {
      if (v + skip > ulen) return u_is_eof ? 3 : 4;
      nv = v + skip;
    }
    *next = nv;
    return 1;
  }
  return 0;
}

// checkRecordStart (BamRecordGuesser.java:34-52): 1 true, 0 false, 4 need more data.  NCHK
// chained records (READS_TO_CHECK = 10, :16); the record-chain speculation (seg_spec) uses 3: its
// guesses are verified link by link and a wrong one is repaired, so it needs a likely start, not
// Disq's planning decision.
template <int NCHK = 10>
__device__ int check_record_start(const uint8_t* U, int64_t ulen, int u_is_eof,
                                  const int32_t* ref_len, int32_t n_ref, int64_t v) {
  for (int k = 0; k < NCHK; k++) {
    int64_t nv = 0;
    int r = check_internal(U, ulen, u_is_eof, ref_len, n_ref, v, &nv);
    if (r == 1) {
      v = nv;
      continue;
    }
    if (r == 0) return 0;
    if (r == 3) return k > 0 ? 1 : 0;
    return 4;
  }
  return 1;
}

// ------------------------------------------------------------------ planning
__device__ inline int64_t lower_bound_cand(const Cand* c, int64_t n, int64_t p) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (c[mid].pos < p) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
__device__ inline int64_t lower_bound_i64(const int64_t* a, int64_t n, int64_t v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
__device__ inline int64_t lower_bound_u64(const uint64_t* a, int64_t n, uint64_t v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
// block containing linear offset x: largest j with uoff[j] <= x among blocks with data.
__device__ inline int64_t block_of(const int64_t* uoff, int64_t nblk, int64_t x) {
  int64_t lo = 0, hi = nblk - 1;
  while (lo < hi) {
    int64_t mid = (lo + hi + 1) >> 1;
    if (uoff[mid] <= x) lo = mid;
    else hi = mid - 1;
  }
  // skip back over trailing empty blocks sharing the offset: take the last block whose range
  // contains x (uoff[j] <= x < uoff[j+1]).
  while (lo > 0 && uoff[lo] > x) lo--;
  return lo;
}

// guessNextBGZFPos(p, end) over the candidate list (magic positions, in order), then the
// BgzfBlockSource chain of the split: blocks [first, last] with pos <= split end.
__global__ void plan_blocks_kernel(const Cand* __restrict__ cand, const int64_t* __restrict__ ncand,
                                   const int64_t* __restrict__ blk_pos,
                                   const int32_t* __restrict__ blk_usize,
                                   const int64_t* __restrict__ uoff, const int64_t* __restrict__ d_nblk,
                                   SplitPlan* __restrict__ plans, int64_t nsplit) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nsplit) return;
  SplitPlan& P = plans[i];
  const int64_t nc = *ncand, nb = *d_nblk;
  P.first_blk = -1;
  P.rec_lin = -1;
  P.status = 0;
  const int64_t s = P.split_start, e = P.split_end;
  int64_t p = s;
  int64_t found = -1, j = -1;
  // BgzfBlockSource's lazy iterator (BgzfBlockSource.java:63-84): guess from `start`, then from
  // the guessed block's end, while start <= split end.  A guess off the BGZF chain is a member
  // header inside payload (stored blocks keep payload bytes verbatim): an empty one (uSize 0)
  // gives getFirstReadInPartition no positions to test, so the iterator just moves on past it;
  // one with data would be inflated by the reference (which then fails on the bytes after it,
  // or reads garbage) -- not reproduced: reported as ST_BAD_HEADER.
  // No hop cap (the reference has none, BgzfBlockGuesser.java:78-145): every hop moves p forward
  // (past a magic or past an empty member), and empty members inside payload all lie inside one
  // real block (<= 65536 bytes, so <= 2341 of 28 bytes) before the chain reaches that block's
  // successor, a real block.
  while (found < 0) {
    if (p > e) return;
    int64_t g = -1;
    for (;;) {
      int64_t k = lower_bound_cand(cand, nc, p);
      if (k >= nc) break;             // scan runs off the data -> null
      const Cand c = cand[k];
      if (c.pos != p && c.pos >= e) break;  // :91 end check (skipped for the first position)
      if (c.valid == 1) {
        g = k;
        break;
      }
      if (c.valid == 2) break;        // IOException -> null
      p = c.pos + 4;                  // :144, tested without an end check
    }
    if (g < 0) return;
    const Cand c = cand[g];
    j = lower_bound_i64(blk_pos, nb, c.pos);
    if (j < nb && blk_pos[j] == c.pos) {
      found = c.pos;
    } else if (c.usize == 0 && c.csize > 0) {
      p = c.pos + c.csize;            // an empty member inside payload: skipped
    } else {
      P.status = ST_BAD_HEADER;       // a member with data inside payload
      return;
    }
  }
  // BgzfBlockSource: blocks while start <= split end
  int64_t jl = j;
  while (jl + 1 < nb && blk_pos[jl + 1] <= e) jl++;
  P.first_blk = j;
  P.u_lo = uoff[j];
  P.u_hi = uoff[jl] + blk_usize[jl];
}

// BamSource.getFirstReadInPartition: first position (<= 10,000,000 scanned) where the guesser
// fires.  FR_K workgroups per split scan interleaved 256-position steps (a split that starts
// inside a 2 Mb read has ~1.5 MB of positions before its first record: one workgroup stepping
// through them was the planning's critical path); hits go to the split's minimum by a 64-bit
// atomic, and a workgroup stops once its next step starts past the current minimum -- every
// position below the final minimum was checked by the workgroup that owns its step.
// first_record_final_kernel then fills the plan (one thread per split).
constexpr int FR_K = 16;
__global__ __launch_bounds__(256) void first_record_kernel(
    const uint8_t* __restrict__ U, int64_t ulen, int32_t u_is_eof, const int32_t* __restrict__ ref_len,
    int32_t n_ref, const SplitPlan* __restrict__ plans, int64_t nsplit,
    unsigned long long* __restrict__ best_all) {
  __shared__ unsigned long long cur;
  const int64_t i = blockIdx.x / FR_K, k = blockIdx.x % FR_K;
  if (i >= nsplit) return;
  const SplitPlan& P = plans[i];
  if (P.first_blk < 0 || P.status != 0) return;
  unsigned long long* best = best_all + i;  // the minimum hit; best[nsplit]: a "need more data" seen
  const int64_t lo = P.u_lo;
  const int64_t hi = min(P.u_hi, lo + (int64_t)10000000);
  for (int64_t b = lo + 256 * k; b < hi; b += 256 * FR_K) {
    if (threadIdx.x == 0) cur = __hip_atomic_load(best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const bool stop = (unsigned long long)b > cur;
    __syncthreads();
    if (stop) break;
    const int64_t v = b + threadIdx.x;
    if (v < hi) {
      const int r = check_record_start(U, ulen, u_is_eof, ref_len, n_ref, v);
      if (r == 1 || r == 4) atomicMin(best, (unsigned long long)v);
      if (r == 4) atomicOr(best + nsplit, 1ull);
    }
  }
}

__global__ void first_record_final_kernel(const uint8_t* __restrict__ U, int64_t ulen, int32_t u_is_eof,
                                          const int32_t* __restrict__ ref_len, int32_t n_ref,
                                          const int64_t* __restrict__ blk_pos,
                                          const int64_t* __restrict__ uoff,
                                          const int64_t* __restrict__ d_nblk,
                                          SplitPlan* __restrict__ plans, int64_t nsplit,
                                          const unsigned long long* __restrict__ best_all) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nsplit) return;
  SplitPlan& P = plans[i];
  if (P.first_blk < 0 || P.status != 0) return;
  const unsigned long long best = best_all[i];
  if (best != ~0ull) {
    // a "need more data" at the minimum position means the answer is unknown here
    const int64_t v = (int64_t)best;
    if (best_all[nsplit + i] && check_record_start(U, ulen, u_is_eof, ref_len, n_ref, v) == 4) {
      P.status = 100;  // caller must extend the buffer
      return;
    }
    const int64_t nb = *d_nblk;
    const int64_t j = block_of(uoff, nb, v);
    P.rec_lin = v;
    P.vstart = ((uint64_t)blk_pos[j] << 16) | (uint64_t)(v - uoff[j]);
    // bytes of the (up to) 10 records the guesser chained from v: the host sizes the record
    // chain's segments by the typical record length
    int64_t q = v;
    for (int k = 0; k < 10 && q + 4 <= ulen; k++) q += 4 + (int64_t)(uint32_t)ld32(U, q);
    P.rec_span = (int32_t)min(q - v, (int64_t)INT32_MAX);
  }
  P.vend = ((uint64_t)P.split_end << 16) | 0xffff;
}

// ------------------------------------------------------------------ Kernel 3: record chain
// Records are walked with next = p + 4 + block_size (htsjdk BAMRecordCodec.decode reads
// block_size, then block_size bytes).  Segment speculation uses the guesser; a segment whose
// speculated start differs from its predecessor's exit is re-walked from that exit, so the
// result is the exact sequential chain regardless of speculation quality.
constexpr int64_t END_CHAIN = INT64_MAX;

// Walk from `start` while p < seg_end.  Returns exit position (>= seg_end, or END_CHAIN), count.
__device__ int walk(const uint8_t* U, int64_t ulen, int u_is_eof, int64_t start, int64_t seg_end,
                    int64_t* exit, int64_t* count) {
  int64_t p = start, n = 0;
  while (p < seg_end) {
    if (p + 4 > ulen) {
      if (u_is_eof) {
        *exit = END_CHAIN;
        *count = n;
        return 0;
      }
      return 4;
    }
    int32_t bs = ld32(U, p);
    if (bs < 32) return ST_BAD_CODE;  // "Invalid record length" (SAMFormatException)
    n++;
    p += 4 + (int64_t)bs;
  }
  *exit = p;
  *count = n;
  return 0;
}

// walk() for a window of a sparse run: a record must also END inside the inflated bytes (the
// bytes after a window are not inflated); 4 = the window needs more blocks.
__device__ int walk_win(const uint8_t* U, int64_t ulen, int u_is_eof, int64_t start,
                        int64_t seg_end, int64_t* exit, int64_t* count) {
  int64_t p = start, n = 0;
  while (p < seg_end) {
    if (p + 4 > ulen) {
      if (u_is_eof) {
        *exit = END_CHAIN;
        *count = n;
        return 0;
      }
      return 4;
    }
    const int32_t bs = ld32(U, p);
    if (bs < 32) return ST_BAD_CODE;
    if (p + 4 + (int64_t)bs > ulen) return u_is_eof ? ST_SHORT : 4;
    n++;
    p += 4 + (int64_t)bs;
  }
  *exit = p;
  *count = n;
  return 0;
}

// One workgroup of NT threads per segment (grid-stride: a few thousand resident workgroups instead
// of one dispatch per segment): the first guesser hit at or after the segment start, NT positions
// per step.  Short reads: one wave (the first record is a few hundred bytes in); long reads: a
// 256-thread workgroup, since the first record start after a segment start lies a size-biased
// half record (~160 KB on the long-read file) in.
template <int NT>
__global__ __launch_bounds__(NT) void seg_spec_kernel(const uint8_t* __restrict__ U, int64_t ulen,
                                                      int32_t u_is_eof,
                                                      const int32_t* __restrict__ ref_len,
                                                      int32_t n_ref, Seg* __restrict__ segs,
                                                      int64_t nseg, int64_t seg_bytes,
                                                      int64_t start_lin, int64_t chain_end) {
  __shared__ unsigned long long hit_min;
  for (int64_t s = blockIdx.x; s < nseg; s += gridDim.x) {
    const int64_t sb = start_lin + s * seg_bytes;
    const int64_t se = min(chain_end, sb + seg_bytes);
    int64_t best = INT64_MAX;
    if (s == 0) {
      best = start_lin;
    } else if (NT == 64) {
      for (int64_t b = sb; b < se; b += 64) {
        const int64_t v = b + threadIdx.x;
        const bool hit = v < se && check_record_start<3>(U, ulen, u_is_eof, ref_len, n_ref, v) == 1;
        const uint64_t m = __ballot(hit);
        if (m) {
          best = b + __builtin_ctzll(m);
          break;
        }
      }
    } else {
      if (threadIdx.x == 0) hit_min = ~0ull;
      __syncthreads();
      for (int64_t b = sb; b < se; b += NT) {
        const int64_t v = b + threadIdx.x;
        if (v < se && check_record_start<3>(U, ulen, u_is_eof, ref_len, n_ref, v) == 1)
          atomicMin(&hit_min, (unsigned long long)v);
        __syncthreads();
        const bool done = hit_min != ~0ull;
        __syncthreads();  // every thread has read hit_min before the next step's atomics
        if (done) break;
      }
      if (hit_min != ~0ull) best = (int64_t)hit_min;
      __syncthreads();  // hit_min is read by every thread before the next segment resets it
    }
    if (threadIdx.x == 0) {
      Seg g;
      g.exact = s == 0;
      g.status = 0;
      g.start = best == INT64_MAX ? -1 : best;  // -1: no start speculated in this segment
      g.exit = -1;
      g.count = 0;
      segs[s] = g;
    }
  }
}

// seg_spec for short records with an LDS pre-filter: the wave stages 1 KiB windows of the segment
// (coalesced 16-byte LDS-DMA pieces) and tests each candidate's fixed header against the
// conditions checkInternal applies before it reads past the header (BamRecordGuesser.java:79-194:
// ref ids and positions, name length, CIGAR/sequence presence, the name's NUL, block_size >= the
// fixed parts).  Only candidates passing all of them run check_record_start<3> on U, so the
// speculated start is the one seg_spec_kernel<64> finds (the pre-filter rejects only positions
// whose first checkInternal returns 0, 3 or 4); seg_spec_kernel<64> ran the whole divergent check
// for 64 candidates per step (round 6: 47 k cycles per segment, 57 % waiting,
// profiles/r6h_records_pmc.txt).
#ifndef DQ_SPEC_LDS  // 0: seg_spec_kernel<64>, 1: seg_spec_lds_kernel, 2: seg_spec_split_kernel<DQ_SPEC_SL>
#define DQ_SPEC_LDS 2
#endif
#ifndef DQ_SPEC_SL
#define DQ_SPEC_SL 16
#endif
constexpr int SPEC_WIN = 1024;                   // candidates per staged window
constexpr int SPEC_PIECES = (SPEC_WIN + 64) / 16;  // + one header's bytes past the last candidate
__device__ __forceinline__ bool spec_prefilter(const __attribute__((address_space(3))) uint32_t* W,
                                               int o, int avail, int64_t v, int64_t ulen,
                                               const int32_t* __restrict__ ref_len, int32_t n_ref) {
  if (o + 36 > avail) return true;  // not staged: the full check decides
  if (v + 36 > ulen) return false;  // rd_ok(v, 36) fails: 3 or 4
  const uint32_t sh = (uint32_t)(o & 3);
  const int wi = o >> 2;
  uint32_t w[9], f[8];
#pragma unroll
  for (int k = 0; k < 9; k++) w[k] = W[wi + k];
#pragma unroll
  for (int k = 0; k < 8; k++) f[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
  const int32_t remaining = (int32_t)f[0], id = (int32_t)f[1], pos = (int32_t)f[2];
  if (id < -1 || id >= n_ref || pos < -1) return false;
  if (id >= 0 && pos > ref_len[id]) return false;
  const int32_t nid = (int32_t)f[6], npos = (int32_t)f[7];
  if (nid < -1 || nid >= n_ref || npos < -1) return false;
  if (nid >= 0 && npos > ref_len[nid]) return false;
  const int32_t name_len = (int32_t)(f[3] & 0xff);
  if (name_len < 2) return false;
  const int32_t flags = (int32_t)(f[4] >> 16), n_cig = (int32_t)(f[4] & 0xffff);
  const int32_t cig_len = (int32_t)((uint32_t)n_cig * 4u);
  const int32_t l_seq = (int32_t)f[5];
  const int32_t seq_len = (int32_t)((uint32_t)l_seq + (uint32_t)((int32_t)((uint32_t)l_seq + 1u) / 2));
  if ((flags & 4) == 0 && (seq_len == 0 || n_cig == 0)) return false;
  if (v + 36 + name_len > ulen) return false;  // rd_ok(v + 36, name_len) fails: 3 or 4
  const int t = o + 36 + name_len - 1;         // the name's NUL
  if (t < avail) {
    const uint32_t b = (W[t >> 2] >> (8 * (t & 3))) & 0xff;
    if (b != 0) return false;
  }
  const int32_t zero_min =
      (int32_t)((uint32_t)32 + (uint32_t)name_len + (uint32_t)cig_len + (uint32_t)seq_len);
  return remaining >= zero_min;  // checked last by checkInternal; a start must pass it
}

__global__ __launch_bounds__(64) void seg_spec_lds_kernel(const uint8_t* __restrict__ U, int64_t ulen,
                                                          int32_t u_is_eof,
                                                          const int32_t* __restrict__ ref_len,
                                                          int32_t n_ref, Seg* __restrict__ segs,
                                                          int64_t nseg, int64_t seg_bytes,
                                                          int64_t start_lin, int64_t chain_end) {
  __shared__ uint4 win[SPEC_PIECES + 1];
  const auto W = (const __attribute__((address_space(3))) uint32_t*)win;
  const int lane = threadIdx.x;
  for (int64_t s = blockIdx.x; s < nseg; s += gridDim.x) {
    const int64_t sb = start_lin + s * seg_bytes;
    const int64_t se = min(chain_end, sb + seg_bytes);
    int64_t best = INT64_MAX;
    if (s == 0) best = start_lin;
    for (int64_t v0 = sb; s != 0 && v0 < se && best == INT64_MAX;) {
      const int64_t wb = v0 & ~(int64_t)15;
      const int64_t vend = min(se, wb + SPEC_WIN);
      // pieces wholly inside [0, ulen) (U's padding is not assumed here)
      const int np = (int)max((int64_t)0, min((int64_t)SPEC_PIECES, (ulen - wb) / 16));
      const uint4* src = reinterpret_cast<const uint4*>(U + wb);
      for (int c0 = 0; c0 < np; c0 += 64)
        if (c0 + lane < np)
          __builtin_amdgcn_global_load_lds(static_cast<const void*>(src + c0 + lane),
                                           (__attribute__((address_space(3))) void*)(win + c0), 16, 0, 0);
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      for (int64_t b = v0; b < vend; b += 64) {
        const int64_t v = b + lane;
        bool hit = v < vend && spec_prefilter(W, (int)(v - wb), 16 * np, v, ulen, ref_len, n_ref);
        if (hit) hit = check_record_start<3>(U, ulen, u_is_eof, ref_len, n_ref, v) == 1;
        const uint64_t m = __ballot(hit);
        if (m) {
          best = b + __builtin_ctzll(m);
          break;
        }
      }
      v0 = vend;
      __syncthreads();  // every lane is done with the window before it is restaged
    }
    if (lane == 0) {
      Seg g;
      g.exact = s == 0;
      g.status = 0;
      g.start = best == INT64_MAX ? -1 : best;
      g.exit = -1;
      g.count = 0;
      segs[s] = g;
    }
  }
}

// The same search with SL lanes per segment, 64 / SL segments per wave at once: a segment's cost is
// the full check of its true start (three chained records, a dozen dependent round trips), so
// several segments' checks in one wave overlap those latencies; the windows are 512 bytes.  Piece
// k of sub-window u lands at LDS byte 1024 (k / SL) + 16 SL u + 16 (k % SL) (an LDS-DMA
// instruction writes 16 bytes per lane at consecutive lane slots).
template <int SL>
__global__ __launch_bounds__(64) void seg_spec_split_kernel(const uint8_t* __restrict__ U, int64_t ulen,
                                                            int32_t u_is_eof,
                                                            const int32_t* __restrict__ ref_len,
                                                            int32_t n_ref, Seg* __restrict__ segs,
                                                            int64_t nseg, int64_t seg_bytes,
                                                            int64_t start_lin, int64_t chain_end) {
  constexpr int NSUB = 64 / SL, WINB = 512, NPC = (WINB + 64) / 16;  // pieces per sub-window
  constexpr int NI = (NPC + SL - 1) / SL;                              // DMA instructions per window
  __shared__ uint4 win[NI * 64 + 1];
  const auto W = (const __attribute__((address_space(3))) uint8_t*)win;
  const int lane = threadIdx.x, u = lane / SL, ll = lane % SL;
  const uint64_t umask = (SL == 64 ? ~0ull : ((1ull << SL) - 1)) << (u * SL);
  REC_T_DECL;
  for (int64_t s0 = (int64_t)blockIdx.x * NSUB; s0 < nseg; s0 += (int64_t)gridDim.x * NSUB) {
    const int64_t s = s0 + u;
    const int64_t sb = start_lin + s * seg_bytes;
    const int64_t se = s < nseg ? min(chain_end, sb + seg_bytes) : sb;
    int64_t best = INT64_MAX;
    if (s == 0) best = start_lin;
    int64_t v0 = sb;
    bool searching = s != 0 && s < nseg && v0 < se;
    while (__any(searching)) {
      const int64_t wb = v0 & ~(int64_t)15;
      const int64_t vend = min(se, wb + WINB);
      const int np = searching ? (int)max((int64_t)0, min((int64_t)NPC, (ulen - wb) / 16)) : 0;
      const uint4* src = reinterpret_cast<const uint4*>(U + wb);
#pragma unroll
      for (int c = 0; c < NI; c++)
        if (c * SL + ll < np)
          __builtin_amdgcn_global_load_lds(static_cast<const void*>(src + c * SL + ll),
                                           (__attribute__((address_space(3))) void*)(win + c * 64), 16, 0, 0);
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      REC_T(0);
      // sub-window byte o -> LDS byte (SB bytes of each sub-window per DMA instruction)
      constexpr int SB = SL * 16;
      const int ub = u * SB;
      auto ldw = [&](int o) -> uint32_t {  // the dword at sub-window byte o (o % 4 == 0)
        return *(const __attribute__((address_space(3))) uint32_t*)(W + (o / SB) * 1024 + ub + (o % SB));
      };
      bool scan = searching;
      for (int64_t b = v0; __any(scan); b += SL) {
        const int64_t v = b + ll;
        bool hit = false;
        if (scan && v < vend) {
          const int o = (int)(v - wb), avail = 16 * np;
          bool pass = true;
          if (o + 36 <= avail) {
            if (v + 36 > ulen) {
              pass = false;
            } else {
              const uint32_t sh = (uint32_t)(o & 3);
              const int o4 = o & ~3;
              uint32_t w[9], f[8];
#pragma unroll
              for (int k = 0; k < 9; k++) w[k] = ldw(o4 + 4 * k);
#pragma unroll
              for (int k = 0; k < 8; k++) f[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
              const int32_t remaining = (int32_t)f[0], id = (int32_t)f[1], pos = (int32_t)f[2];
              const int32_t nid = (int32_t)f[6], npos = (int32_t)f[7];
              const int32_t name_len = (int32_t)(f[3] & 0xff);
              const int32_t flags = (int32_t)(f[4] >> 16), n_cig = (int32_t)(f[4] & 0xffff);
              const int32_t cig_len = (int32_t)((uint32_t)n_cig * 4u);
              const int32_t l_seq = (int32_t)f[5];
              const int32_t seq_len =
                  (int32_t)((uint32_t)l_seq + (uint32_t)((int32_t)((uint32_t)l_seq + 1u) / 2));
              const int32_t zero_min =
                  (int32_t)((uint32_t)32 + (uint32_t)name_len + (uint32_t)cig_len + (uint32_t)seq_len);
              pass = !(id < -1 || id >= n_ref || pos < -1) && !(nid < -1 || nid >= n_ref || npos < -1) &&
                     name_len >= 2 && !((flags & 4) == 0 && (seq_len == 0 || n_cig == 0)) &&
                     v + 36 + name_len <= ulen && remaining >= zero_min;
              if (pass) {
                const int t = o + 36 + name_len - 1;  // the name's NUL
                if (t < avail && ((ldw(t & ~3) >> (8 * (t & 3))) & 0xff) != 0) pass = false;
              }
              if (pass && id >= 0 && pos > ref_len[id]) pass = false;
              if (pass && nid >= 0 && npos > ref_len[nid]) pass = false;
            }
          }
          REC_T(1);
#ifdef DQ_REC_TIMING
          rt_[3] += __any(pass) ? 1 : 0;
          rt_[7] += __popcll(__ballot(pass));
#endif
          if (pass) hit = check_record_start<3>(U, ulen, u_is_eof, ref_len, n_ref, v) == 1;
          REC_T(2);
        }
        const uint64_t m = __ballot(hit) & umask;
        if (scan && m) {
          best = b + (__builtin_ctzll(m) - u * SL);
          scan = false;
          searching = false;
        }
        if (b + SL >= vend) scan = false;  // this window is done
      }
      if (searching) {
        v0 = vend;
        searching = v0 < se;
      }
      __syncthreads();  // every lane is done with the windows before they are restaged
    }
    if (ll == 0 && s < nseg) {
      Seg g;
      g.exact = s == 0;
      g.status = 0;
      g.start = best == INT64_MAX ? -1 : best;
      g.exit = -1;
      g.count = 0;
      segs[s] = g;
    }
  }
  REC_T_FLUSH;
}

#ifdef DQ_CHECKED
__global__ void spec_cmp_kernel(const Seg* __restrict__ a, const Seg* __restrict__ b, int64_t n) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s < n) DQ_CHK(a[s].start == b[s].start, CHK_K3_SPEC);
}
#endif

// The walks of all segments, one lane each (a walk is a chain of dependent loads: many walks per
// wave keep many in flight).  With `offs` (64 KiB segments), the walk also records its record
// starts as 16-bit offsets from the segment start, four per 8-byte store, so that seg_emit copies
// them instead of walking the chain a second time (round 5: the re-walk fetched a line of U per
// record again, 2.9 ms of the 12.5 GB file's 214 ms step).
__global__ __launch_bounds__(256) void seg_walk_kernel(const uint8_t* __restrict__ U, int64_t ulen,
                                                       int32_t u_is_eof, Seg* __restrict__ segs,
                                                       int64_t nseg, int64_t seg_bytes,
                                                       int64_t start_lin, int64_t chain_end,
                                                       uint16_t* __restrict__ offs) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nseg) return;
  Seg g = segs[s];
  if (g.start < 0) return;
  const int64_t sb = start_lin + s * seg_bytes;
  const int64_t se = min(chain_end, sb + seg_bytes);
  int64_t ex = 0, cnt = 0;
  int r;
  if (offs) {
    uint64_t* const o64 = reinterpret_cast<uint64_t*>(offs + s * SEG_OFF_CAP);
    int64_t p = g.start, n = 0;
    uint64_t acc = 0;
    r = 0;
    for (;;) {
      if (p >= se) {
        ex = p;
        break;
      }
      if (p + 4 > ulen) {
        if (u_is_eof) {
          ex = END_CHAIN;
          break;
        }
        r = 4;
        break;
      }
      const int32_t bs = ld32(U, p);
      if (bs < 32) {
        r = ST_BAD_CODE;
        break;
      }
      acc |= (uint64_t)(uint16_t)(p - sb) << (16 * (n & 3));
      if ((n & 3) == 3 && n < SEG_OFF_CAP) {
        o64[n >> 2] = acc;
        acc = 0;
      }
      n++;
      p += 4 + (int64_t)bs;
    }
    if (r == 0 && (n & 3) && n <= SEG_OFF_CAP) o64[n >> 2] = acc;
    cnt = n;
    g.exact = (g.exact & 1) | (r == 0 && n <= SEG_OFF_CAP ? 2 : 0);
  } else {
    r = walk(U, ulen, u_is_eof, g.start, se, &ex, &cnt);
  }
  g.status = r;
  if (r == 0) {
    g.exit = ex;
    g.count = cnt;
  }
  segs[s] = g;
}

// Serial link check + repair (one lane), run only when seg_link found a broken link (a guesser
// false positive): each link is O(1) unless a speculation was wrong, in which case that segment is
// re-walked from the exact incoming position.
__global__ void seg_fix_kernel(const uint8_t* __restrict__ U, int64_t ulen, int32_t u_is_eof,
                               Seg* __restrict__ segs, int64_t nseg, int64_t seg_bytes,
                               int64_t start_lin, int64_t chain_end, int32_t* d_status) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int64_t in = segs[0].exit;
  if (segs[0].status) {
    *d_status = segs[0].status;
    return;
  }
  for (int64_t s = 1; s < nseg; s++) {
    Seg& g = segs[s];
    const int64_t sb = start_lin + s * seg_bytes;
    const int64_t se = min(chain_end, sb + seg_bytes);
    if (in == END_CHAIN || in >= se) {  // no record starts inside this segment
      g.start = in;
      g.exit = in;
      g.count = 0;
      g.exact = 1;
      g.status = 0;
      continue;
    }
    if (g.start != in || g.status != 0) {
      int64_t ex = -1, cnt = 0;
      int r = walk(U, ulen, u_is_eof, in, se, &ex, &cnt);
      g.exact = 0;  // the recorded starts were another walk's
      g.start = in;
      g.status = r;
      g.exit = ex;
      g.count = cnt;
      if (r) {
        *d_status = r;
        return;
      }
    }
    g.exact |= 1;
    in = g.exit;
  }
}

// Parallel link check: segment s is consistent when the exit of the last earlier segment that
// has a start equals s's speculated start (or passes beyond s when s has none).
__global__ void seg_link_kernel(const Seg* __restrict__ segs, int64_t nseg, int64_t seg_bytes,
                                int64_t start_lin, int64_t ulen, int32_t* d_broken) {
  int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nseg) return;
  const Seg g = segs[s];
  if (g.status != 0) {
    *d_broken = 1;
    return;
  }
  if (s == 0) return;
  int64_t t = s - 1;
  while (t > 0 && segs[t].start < 0) t--;
  const int64_t in = segs[t].exit;
  const int64_t se = min(ulen, start_lin + (s + 1) * seg_bytes);
  bool ok = g.start < 0 ? (in == END_CHAIN || in >= se) : (in == g.start);
  if (!ok) *d_broken = 1;
}

__global__ void seg_counts_kernel(const Seg* __restrict__ segs, int64_t nseg, int64_t* counts) {
  int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s < nseg) counts[s] = segs[s].count;
}

// One lane per segment walks its chain again and writes the record starts.  The walk goes in
// rounds of EMIT_R records into an LDS buffer per lane; the wave then writes each lane's run with
// consecutive lanes on consecutive entries (coalesced), instead of 64 lanes storing 64 scattered
// 8-byte entries per instruction.
constexpr int EMIT_R = 32;
__global__ __launch_bounds__(64) void seg_emit_kernel(const uint8_t* __restrict__ U,
                                                      const Seg* __restrict__ segs,
                                                      const int64_t* __restrict__ base, int64_t nseg,
                                                      int64_t* __restrict__ rec_lin) {
  __shared__ int64_t buf[64][EMIT_R + 1];
  const int lane = threadIdx.x;
  const int64_t s = (int64_t)blockIdx.x * 64 + lane;
  int64_t p = 0, o = 0, left = 0;
  if (s < nseg) {
    const Seg g = segs[s];
    p = g.start;
    o = base[s];
    left = (g.exact & 2) ? 0 : g.count;  // recorded by the walk: seg_copy_kernel writes them
  }
  for (;;) {
    const int n = (int)min(left, (int64_t)EMIT_R);
    if (!__any(n > 0)) break;
    for (int k = 0; k < n; k++) {
      buf[lane][k] = p;
      p += 4 + (int64_t)ld32(U, p);
    }
    // publish (n, o) of every lane, then write lane l's n entries with lanes 0..n-1
    const int64_t my_o = o;
    for (int l = 0; l < 64; l++) {
      const int nl = __shfl(n, l, 64);
      if (nl == 0) continue;  // uniform
      const int64_t ol = __shfl(my_o, l, 64);
      if (lane < nl) rec_lin[ol + lane] = buf[l][lane];
    }
    o += n;
    left -= n;
  }
}

// The record starts the walk recorded (Seg.exact bit 1): one wave per segment copies them to
// rec_lin, consecutive lanes on consecutive entries (grid-stride over the segments).
__global__ __launch_bounds__(64) void seg_copy_kernel(const Seg* __restrict__ segs,
                                                      const int64_t* __restrict__ base, int64_t nseg,
                                                      const uint16_t* __restrict__ offs,
                                                      int64_t seg_bytes, int64_t start_lin,
                                                      int64_t* __restrict__ rec_lin) {
  for (int64_t s = blockIdx.x; s < nseg; s += gridDim.x) {
    const int32_t ex = segs[s].exact;
    if (!(ex & 2)) continue;
    const int64_t cnt = segs[s].count, o = base[s], sb = start_lin + s * seg_bytes;
    const uint16_t* of = offs + s * SEG_OFF_CAP;
    for (int64_t k = threadIdx.x; k < cnt; k += 64) rec_lin[o + k] = sb + (int64_t)of[k];
  }
}

// ------------------------------------------------------------------ decode + hash
// Page table for block_of: pt[g] = the last block whose first byte is <= g * 64 KiB, so the block
// of a record start is pt[p >> 16] plus a short forward walk (htsjdk blocks hold <= 64 KiB).
__global__ void block_pages_kernel(const int64_t* __restrict__ uoff, int64_t nblk, int32_t* pt,
                                   int64_t npages) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g < npages) pt[g] = (int32_t)block_of(uoff, nblk, g << 16);
}

__device__ inline uint32_t funnel(uint32_t lo, uint32_t hi, uint32_t sh) {  // (hi:lo) >> 8 sh
  return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

// One wave per 64 consecutive records (the chain is contiguous in U).  The wave first copies the
// records' bytes into LDS with coalesced 16-byte loads, then lane r decodes record r: fixed fields
// into the SoA, the htsjdk start pointer (block via the page table) and the raw-byte hash
// (8-byte little-endian words, zero padded; DESIGN.md section "hash") from LDS.  Runs of records
// longer than the staging buffer (long reads) are read straight from U.
constexpr int REC_WAVE = 64;      // threads per workgroup (one wave)
// lanes per record (they split its hash words); records per group = 64 / lanes; the staging holds
// one group of short-read records (~330 B each): 2 lanes -> 32 records, 12 KB, 13 waves per CU;
// 4 lanes -> 16 records, 6 KB, 26 waves per CU
#ifndef DQ_REC_LANES
#define DQ_REC_LANES 2
#endif
constexpr int REC_LANES = DQ_REC_LANES;
static_assert(REC_LANES == 2 || REC_LANES == 4, "2 or 4 lanes per record");
constexpr int REC_GROUP = REC_WAVE / REC_LANES;
constexpr int REC_STAGE = REC_GROUP * 384;

// Lane work of decode_group: record i (start p, n = 4 + block_size bytes) read through W, a
// dword view in which the record starts at byte `off` (LDS staging or U itself).  Lane part 0
// decodes the fixed fields; the REC_LANES parts hash the record's 8-byte words k = part mod
// REC_LANES (the word sum is order-free) and return the partial sum.
// SoA stores: non-temporal (the rows are not read again by this pass; 2 % faster records stage,
// profiles/r6o_records_window_nt.txt); DQ_REC_NT=0: plain stores
#ifndef DQ_REC_NT
#define DQ_REC_NT 1
#endif
#if DQ_REC_NT
#define REC_ST(dst, v) __builtin_nontemporal_store((v), &(dst))
#else
#define REC_ST(dst, v) ((dst) = (v))
#endif
struct BlockOf {  // the htsjdk block of a record start: loaded before the staging wait
  int64_t j, u0, u1, bp;
};

template <typename WP>
__device__ __attribute__((always_inline)) inline uint64_t decode_one(
    WP W, int64_t off, int64_t p, int32_t bs, int64_t n, int64_t i, int half,
    const int64_t* __restrict__ blk_pos, const int64_t* __restrict__ uoff, int64_t nblk,
    BlockOf bo, const RecSoA& soa, bool hash = true) {
  const int64_t wi0 = off >> 2;
  const uint32_t sh = (uint32_t)(off & 3);
  if (half == 0) {
    uint32_t f[10];
    {
      uint32_t w[10];
#pragma unroll
      for (int k = 0; k < 10; k++) w[k] = W[wi0 + k];
#pragma unroll
      for (int k = 0; k < 9; k++) f[k] = funnel(w[k], w[k + 1], sh);
    }
    REC_ST(soa.block_size[i], bs);
    REC_ST(soa.ref_id[i], (int32_t)f[1]);
    REC_ST(soa.pos[i], (int32_t)f[2]);
    REC_ST(soa.l_read_name[i], (uint8_t)(f[3] & 0xff));
    REC_ST(soa.mapq[i], (uint8_t)((f[3] >> 8) & 0xff));
    REC_ST(soa.bin[i], (uint16_t)(f[3] >> 16));
    REC_ST(soa.n_cigar[i], (uint16_t)(f[4] & 0xffff));
    REC_ST(soa.flag[i], (uint16_t)(f[4] >> 16));
    REC_ST(soa.l_seq[i], (int32_t)f[5]);
    REC_ST(soa.next_ref_id[i], (int32_t)f[6]);
    REC_ST(soa.next_pos[i], (int32_t)f[7]);
    REC_ST(soa.tlen[i], (int32_t)f[8]);
    while (bo.j + 1 < nblk && bo.u1 <= p) {  // rare: the page's first block ends before p
      bo.j++;
      bo.u0 = bo.u1;
      bo.u1 = bo.j + 1 < nblk ? uoff[bo.j + 1] : INT64_MAX;
      bo.bp = blk_pos[bo.j];
    }
    REC_ST(soa.voffset[i], ((uint64_t)bo.bp << 16) | (uint64_t)(p - bo.u0));
  }
  // hash words k = half, half + REC_LANES, ... (a long record's words: long_hash_kernel): the
  // whole words first, with no mask and 32-bit counters, then the partial last word by the lane
  // whose word it is (round 5 computed the partial-word mask and 64-bit counters for every word:
  // 36 VALU per word, 7 of them the mask)
  uint64_t part = 0;
#ifdef DQ_REC_NOHASH  // dev experiment: the decode without the hash (wrong hashes)
  hash = false;
#endif
  if (hash) {
    const int nfull = (int)(n >> 3), nw = (int)((n + 7) >> 3);
    uint64_t kk = (uint64_t)(half + 1) * DQ_K_WORD;  // (k + 1) K_WORD
    for (int k = half; k < nfull; k += REC_LANES) {
      const int64_t wi = wi0 + 2 * k;
      const uint32_t w0 = W[wi], w1 = W[wi + 1], w2 = W[wi + 2];
      const uint64_t w = ((uint64_t)funnel(w1, w2, sh) << 32) | funnel(w0, w1, sh);
      part += dq_mix64(w ^ kk);
      kk += (uint64_t)REC_LANES * DQ_K_WORD;
    }
    if (nfull < nw && (nfull - half) % REC_LANES == 0) {
      const int64_t wi = wi0 + 2 * nfull;
      const uint32_t w0 = W[wi], w1 = W[wi + 1], w2 = W[wi + 2];
      uint64_t w = ((uint64_t)funnel(w1, w2, sh) << 32) | funnel(w0, w1, sh);
      w &= (1ull << (8 * (n - 8 * (int64_t)nfull))) - 1;
      part += dq_mix64(w ^ ((uint64_t)(nfull + 1) * DQ_K_WORD));
    }
  }
  return part;
}

// Long records (long reads: 10 kb - 2 Mb, records of 15 KB - 3 MB) are hashed by many threads:
// two lanes walking a record of ~100 KB word by word made the records stage 2x the inflate on a
// long-read file.  decode_group appends every PIECE-byte piece of a record longer than LONG_N to a
// list and writes 0 to its hash; long_hash_kernel adds each piece's word sum (the sum is
// order-free) into the hash slot; long_hash_final_kernel applies the length term and mix64.
constexpr int64_t LONG_N = 2048;
constexpr int64_t LONG_PIECE = 32768;
struct LongList {
  uint64_t* ent;                // record index << 16 | piece
  int64_t cap;
  unsigned long long* cnt;      // entries appended
};

__device__ void decode_group(const uint8_t* __restrict__ U, int64_t ulen,
                             const int64_t* __restrict__ rec_lin, int64_t nrec,
                             const int64_t* __restrict__ blk_pos, const int64_t* __restrict__ uoff,
                             int64_t nblk, const int32_t* __restrict__ pt, const RecSoA& soa,
                             int32_t* d_status, int64_t i0, uint4* stage4, LongList ll REC_T_PARAM) {
  const int lane = threadIdx.x, r = lane & (REC_GROUP - 1), half = lane / REC_GROUP;
  const int nact = (int)min((int64_t)REC_GROUP, nrec - i0);
  const int64_t i = i0 + r;
  const bool act = r < nact;
  const int64_t p = act ? rec_lin[i] : rec_lin[i0];
  // block_size of every record: two aligned dwords (U is padded by 256 zero bytes)
  const uint32_t* U32 = reinterpret_cast<const uint32_t*>(U);
  const int32_t bs = (int32_t)funnel(U32[p >> 2], U32[(p >> 2) + 1], (uint32_t)(p & 3));
  const int64_t n = 4 + (int64_t)bs;
  const bool bad = act && p + n > ulen;
  if (__any(bad)) {
    if (bad) *d_status = ST_SHORT;
    return;
  }
  // the block lookups of the voffset, issued now so their latency overlaps the staging
  BlockOf bo;
  bo.j = pt[p >> 16];
  bo.u0 = uoff[bo.j];
  bo.u1 = bo.j + 1 < nblk ? uoff[bo.j + 1] : INT64_MAX;
  bo.bp = blk_pos[bo.j];
  const int64_t first = rec_lin[i0];
  const int64_t lastp = rec_lin[i0 + nact - 1];
  const int32_t lastbs = (int32_t)funnel(U32[lastp >> 2], U32[(lastp >> 2) + 1], (uint32_t)(lastp & 3));
  const int64_t base = first & ~(int64_t)15;
  const int64_t len = lastp + 4 + (int64_t)lastbs - base;
  uint64_t part = 0;
  bool lng = false;
  REC_T(4);
  if (len + 32 <= REC_STAGE) {  // the hash reads up to 12 bytes past the last record
    // LDS-DMA: every 16-byte piece in flight at once (a register-staged loop waits per piece)
    const uint4* src = reinterpret_cast<const uint4*>(U + base);
    const int npiece = (int)((len + 31) / 16);
    // the staged pieces, the fixed-field words and the last hash word read stay in the staging
    DQ_CHK(npiece * 16 <= REC_STAGE && (p - base) + 4 * 10 <= REC_STAGE &&
               (p - base) + 8 * ((n + 7) / 8) + 4 <= REC_STAGE, CHK_K3_STAGE);
    for (int c0 = 0; c0 < npiece; c0 += REC_WAVE)
      if (c0 + lane < npiece)
        __builtin_amdgcn_global_load_lds(
            static_cast<const void*>(src + c0 + lane),
            (__attribute__((address_space(3))) void*)(stage4 + c0), 16, 0, 0);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    REC_T(5);
    if (act)  // DS reads from the staging buffer (a pointer that may be either would be flat)
      part = decode_one((const __attribute__((address_space(3))) uint32_t*)stage4, p - base, p, bs,
                        n, i, half, blk_pos, uoff, nblk, bo, soa);
  } else if (act) {
    lng = n > LONG_N;
    part = decode_one(U32, p, p, bs, n, i, half, blk_pos, uoff, nblk, bo, soa, !lng);
    if (lng && half == 0) {  // its pieces go to long_hash_kernel
      const int64_t np = (n + LONG_PIECE - 1) / LONG_PIECE;
      const int64_t e0 = (int64_t)atomicAdd(ll.cnt, (unsigned long long)np);
      for (int64_t j = 0; j < np && e0 + j < ll.cap; j++) ll.ent[e0 + j] = (uint64_t)i << 16 | (uint64_t)j;
    }
  }
  // the parts' word sums (all lanes take part in the shuffles)
#pragma unroll
  for (int o = REC_GROUP; o < REC_WAVE; o <<= 1) {
    const uint32_t plo = (uint32_t)part, phi = (uint32_t)(part >> 32);
    part += ((uint64_t)(uint32_t)__shfl_xor((int)phi, o, 64) << 32) |
            (uint32_t)__shfl_xor((int)plo, o, 64);
  }
  if (act && half == 0) REC_ST(soa.hash[i], lng ? 0ull : dq_mix64((uint64_t)n * DQ_K_LEN + part));
  REC_T(6);
}

// decode_group without the block-size loads before the staging (DQ_REC_HINT): records ascend and do
// not overlap, so a group's bytes end at or before the next group's first record start, which
// rec_lin already holds; the staging copies [first, that start) and each lane then reads its
// block_size from LDS.  The dependent round trip to U (the first touch of the records' header
// lines, an HBM miss) that sized the staging is gone; a lane whose record does not end inside the
// staged bytes (rec_lin not ascending, e.g. a record listed twice) sends the group down the
// unstaged path, which reads the block sizes from U as decode_group does.
// The group's lane work given its record starts: lane r's start p (the group's first for inactive
// lanes), `nact` records, the first start and an end bound (`end` < 0: the last record's block size
// is loaded to find it).
__device__ void decode_group_core(const uint8_t* __restrict__ U, int64_t ulen, int64_t p, int nact,
                                  int64_t first, int64_t end,
                                  const int64_t* __restrict__ blk_pos, const int64_t* __restrict__ uoff,
                                  int64_t nblk, const int32_t* __restrict__ pt, const RecSoA& soa,
                                  int32_t* d_status, int64_t i0, uint4* stage4, LongList ll REC_T_PARAM) {
  const int lane = threadIdx.x, r = lane & (REC_GROUP - 1), half = lane / REC_GROUP;
  const int64_t i = i0 + r;
  const bool act = r < nact;
  const uint32_t* U32 = reinterpret_cast<const uint32_t*>(U);
  if (end < 0) {  // the chain's last group: its last record's block size
    const int64_t lastp = __shfl(p, nact - 1, 64);
    end = lastp + 4 + (int64_t)(int32_t)funnel(U32[lastp >> 2], U32[(lastp >> 2) + 1], (uint32_t)(lastp & 3));
  }
  // the block lookups of the voffset, issued now so their latency overlaps the staging
  BlockOf bo;
  bo.j = pt[p >> 16];
  bo.u0 = uoff[bo.j];
  bo.u1 = bo.j + 1 < nblk ? uoff[bo.j + 1] : INT64_MAX;
  bo.bp = blk_pos[bo.j];
  const int64_t base = first & ~(int64_t)15;
  const int64_t len = end - base;
  bool staged = len >= 0 && len + 32 <= REC_STAGE && end <= ulen;
  int32_t bs = 0;
  REC_T(4);
  const auto S = (const __attribute__((address_space(3))) uint32_t*)stage4;
  if (staged) {
    const uint4* src = reinterpret_cast<const uint4*>(U + base);
    const int npiece = (int)((len + 31) / 16);
    for (int c0 = 0; c0 < npiece; c0 += REC_WAVE)
      if (c0 + lane < npiece)
        __builtin_amdgcn_global_load_lds(
            static_cast<const void*>(src + c0 + lane),
            (__attribute__((address_space(3))) void*)(stage4 + c0), 16, 0, 0);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    const int64_t o = p - base;
    const bool inb = o >= 0 && o + 8 <= 16 * (int64_t)npiece;
    bs = inb ? (int32_t)funnel(S[o >> 2], S[(o >> 2) + 1], (uint32_t)(o & 3)) : 0;
    const bool fit = !act || (inb && bs >= 0 && p + 4 + (int64_t)bs <= end);
    if (__any(!fit)) staged = false;
    DQ_CHK(!staged || !act || (o + 4 * 10 <= REC_STAGE && o + 8 * ((4 + (int64_t)bs + 7) / 8) + 4 <= REC_STAGE),
           CHK_K3_STAGE);
  }
  REC_T(5);
  if (!staged) bs = (int32_t)funnel(U32[p >> 2], U32[(p >> 2) + 1], (uint32_t)(p & 3));
  const int64_t n = 4 + (int64_t)bs;
  const bool bad = act && p + n > ulen;
  if (__any(bad)) {
    if (bad) *d_status = ST_SHORT;
    return;
  }
  uint64_t part = 0;
  bool lng = false;
  if (staged) {
    if (act) part = decode_one(S, p - base, p, bs, n, i, half, blk_pos, uoff, nblk, bo, soa);
  } else if (act) {
    lng = n > LONG_N;
    part = decode_one(U32, p, p, bs, n, i, half, blk_pos, uoff, nblk, bo, soa, !lng);
    if (lng && half == 0) {  // its pieces go to long_hash_kernel
      const int64_t np = (n + LONG_PIECE - 1) / LONG_PIECE;
      const int64_t e0 = (int64_t)atomicAdd(ll.cnt, (unsigned long long)np);
      for (int64_t j = 0; j < np && e0 + j < ll.cap; j++) ll.ent[e0 + j] = (uint64_t)i << 16 | (uint64_t)j;
    }
  }
#pragma unroll
  for (int o = REC_GROUP; o < REC_WAVE; o <<= 1) {
    const uint32_t plo = (uint32_t)part, phi = (uint32_t)(part >> 32);
    part += ((uint64_t)(uint32_t)__shfl_xor((int)phi, o, 64) << 32) |
            (uint32_t)__shfl_xor((int)plo, o, 64);
  }
  if (act && half == 0) REC_ST(soa.hash[i], lng ? 0ull : dq_mix64((uint64_t)n * DQ_K_LEN + part));
  REC_T(6);
}
__device__ void decode_group_hint(const uint8_t* __restrict__ U, int64_t ulen,
                                  const int64_t* __restrict__ rec_lin, int64_t nrec,
                                  const int64_t* __restrict__ blk_pos, const int64_t* __restrict__ uoff,
                                  int64_t nblk, const int32_t* __restrict__ pt, const RecSoA& soa,
                                  int32_t* d_status, int64_t i0, uint4* stage4, LongList ll REC_T_PARAM) {
  const int r = threadIdx.x & (REC_GROUP - 1);
  const int nact = (int)min((int64_t)REC_GROUP, nrec - i0);
  const int64_t p = r < nact ? rec_lin[i0 + r] : rec_lin[i0];
  const int64_t end = i0 + nact < nrec ? rec_lin[i0 + nact] : -1;
  decode_group_core(U, ulen, p, nact, rec_lin[i0], end, blk_pos, uoff, nblk, pt, soa, d_status, i0, stage4,
                    ll REC_T_ARG);
}
#ifndef DQ_REC_HINT
#define DQ_REC_HINT 1
#endif

// One workgroup per piece of a long record (grid-stride over the list): thread t sums the words
// of pairs t, t + 256, ... of the piece (five dword loads per pair, consecutive lanes on
// consecutive pairs), a workgroup reduction, one 64-bit atomic add into the record's hash slot.
constexpr int LH_THREADS = 256;
__global__ __launch_bounds__(LH_THREADS) void long_hash_kernel(
    const uint8_t* __restrict__ U, const int64_t* __restrict__ rec_lin, const uint64_t* __restrict__ ent,
    const unsigned long long* __restrict__ cnt, int64_t cap, uint64_t* __restrict__ hash) {
  __shared__ uint64_t wsum[LH_THREADS / 64];
  const int64_t ne = min((int64_t)*cnt, cap);
  const uint32_t* U32 = reinterpret_cast<const uint32_t*>(U);
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  for (int64_t e = blockIdx.x; e < ne; e += gridDim.x) {
    const uint64_t x = ent[e];
    const int64_t i = (int64_t)(x >> 16), j = (int64_t)(x & 0xffff);
    const int64_t p = rec_lin[i];
    const uint32_t sh = (uint32_t)(p & 3);
    const int32_t bs = (int32_t)funnel(U32[p >> 2], U32[(p >> 2) + 1], sh);
    const int64_t n = 4 + (int64_t)bs, nw = (n + 7) / 8;
    const int64_t k0 = j * (LONG_PIECE / 8), k1 = min(nw, k0 + LONG_PIECE / 8);
    uint64_t part = 0;
    // whole word pairs without masks, then (one thread) the piece's odd or partial last words
    const int64_t kf = min(k1, n >> 3);  // words with 8 valid bytes end here
    const int64_t kp = k0 + ((kf - k0) & ~(int64_t)1);  // whole pairs [k0, kp)
#pragma unroll 4
    for (int64_t k = k0 + 2 * t; k < kp; k += 2 * LH_THREADS) {
      const int64_t wi = (p >> 2) + 2 * k;
      const uint32_t w0 = U32[wi], w1 = U32[wi + 1], w2 = U32[wi + 2], w3 = U32[wi + 3], w4 = U32[wi + 4];
      const uint64_t a = ((uint64_t)funnel(w1, w2, sh) << 32) | funnel(w0, w1, sh);
      const uint64_t b = ((uint64_t)funnel(w3, w4, sh) << 32) | funnel(w2, w3, sh);
      part += dq_mix64(a ^ ((uint64_t)(k + 1) * DQ_K_WORD)) + dq_mix64(b ^ ((uint64_t)(k + 2) * DQ_K_WORD));
    }
    if (t == 0)
      for (int64_t k = kp; k < k1; k++) {  // at most one whole word and one partial one
        const int64_t wi = (p >> 2) + 2 * k;
        uint64_t a = ((uint64_t)funnel(U32[wi + 1], U32[wi + 2], sh) << 32) | funnel(U32[wi], U32[wi + 1], sh);
        const int64_t ra = n - 8 * k;
        if (ra < 8) a &= (1ull << (8 * ra)) - 1;
        part += dq_mix64(a ^ ((uint64_t)(k + 1) * DQ_K_WORD));
      }
    for (int o = 32; o >= 1; o >>= 1) {
      const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)part, o, 64);
      const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(part >> 32), o, 64);
      part += ((uint64_t)hi << 32) | lo;
    }
    if (lane == 0) wsum[wv] = part;
    __syncthreads();
    if (t == 0) {
      uint64_t s = 0;
      for (int w = 0; w < LH_THREADS / 64; w++) s += wsum[w];
      atomicAdd((unsigned long long*)&hash[i], (unsigned long long)s);
    }
    __syncthreads();
  }
}

// Per-run block statistics without copying the block table to the host: out[0] += sum of the
// DEFLATE payload bytes (csize - 26) over the blocks; block 0 also writes out[1] = uoff of the
// first block whose start is > x (upper bound; ulen past the last), out[2] = the same for >= x
// (lower bound).  out[0] must be zero on entry.
__global__ __launch_bounds__(256) void block_stats_kernel(const int64_t* __restrict__ blk_pos,
                                                          const int32_t* __restrict__ blk_cs,
                                                          const int64_t* __restrict__ uoff, int64_t nblk,
                                                          int64_t ulen, int64_t x, uint64_t* out) {
  uint64_t acc = 0;
  for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nblk;
       b += (int64_t)gridDim.x * blockDim.x)
    acc += (uint64_t)(int64_t)(blk_cs[b] - 26);
  for (int o = 32; o >= 1; o >>= 1) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)acc, o, 64);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(acc >> 32), o, 64);
    acc += ((uint64_t)hi << 32) | lo;
  }
  if ((threadIdx.x & 63) == 0 && acc) atomicAdd((unsigned long long*)out, (unsigned long long)acc);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    int64_t lo = 0, hi = nblk;  // first blk_pos > x
    while (lo < hi) {
      const int64_t m = (lo + hi) >> 1;
      if (blk_pos[m] <= x) lo = m + 1;
      else hi = m;
    }
    out[1] = (uint64_t)(lo < nblk ? uoff[lo] : ulen);
    out[3] = (uint64_t)lo;
    lo = 0, hi = nblk;  // first blk_pos >= x
    while (lo < hi) {
      const int64_t m = (lo + hi) >> 1;
      if (blk_pos[m] < x) lo = m + 1;
      else hi = m;
    }
    out[2] = (uint64_t)(lo < nblk ? uoff[lo] : ulen);
  }
}

__global__ void long_hash_final_kernel(const uint8_t* __restrict__ U, const int64_t* __restrict__ rec_lin,
                                       const uint64_t* __restrict__ ent,
                                       const unsigned long long* __restrict__ cnt, int64_t cap,
                                       uint64_t* __restrict__ hash) {
  const int64_t ne = min((int64_t)*cnt, cap);
  const uint32_t* U32 = reinterpret_cast<const uint32_t*>(U);
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < ne;
       e += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t x = ent[e];
    if (x & 0xffff) continue;  // one entry per record: its first piece
    const int64_t i = (int64_t)(x >> 16), p = rec_lin[i];
    const int32_t bs = (int32_t)funnel(U32[p >> 2], U32[(p >> 2) + 1], (uint32_t)(p & 3));
    hash[i] = dq_mix64((uint64_t)(4 + (int64_t)bs) * DQ_K_LEN + hash[i]);
  }
}

// Grid-stride over groups of 32 records: a few thousand resident waves, not one dispatch per group.
__global__ __launch_bounds__(64) void decode_records_kernel(
    const uint8_t* __restrict__ U, int64_t ulen, const int64_t* __restrict__ rec_lin, int64_t nrec,
    const int64_t* __restrict__ blk_pos, const int64_t* __restrict__ uoff, int64_t nblk,
    const int32_t* __restrict__ pt, RecSoA soa, int32_t* d_status, LongList ll) {
  __shared__ uint4 stage4[REC_STAGE / 16 + 1];
  REC_T_DECL;
  for (int64_t g = blockIdx.x; g * REC_GROUP < nrec; g += gridDim.x) {
    if (DQ_REC_HINT)
      decode_group_hint(U, ulen, rec_lin, nrec, blk_pos, uoff, nblk, pt, soa, d_status, g * REC_GROUP,
                        stage4, ll REC_T_ARG);
    else
      decode_group(U, ulen, rec_lin, nrec, blk_pos, uoff, nblk, pt, soa, d_status, g * REC_GROUP,
                   stage4, ll REC_T_ARG);
    __syncthreads();  // this group is done with the staging buffer
  }
  REC_T_FLUSH;
}

// ------------------------------------------------------------------ partitions
// BAMFileIndexIterator over Chunk(vstart, vend): records from the guesser's start while the
// start pointer < vend (H/BAMFileReader2.java:1082-1095).
__global__ void partition_ranges_kernel(const SplitPlan* __restrict__ plans, int64_t nsplit,
                                        const int64_t* __restrict__ rec_lin,
                                        const uint64_t* __restrict__ voffset, int64_t nrec,
                                        PartRange* __restrict__ parts, int32_t* d_status) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nsplit) return;
  const SplitPlan P = plans[i];
  PartRange r;
  r.begin = r.end = 0;
  r.digest = 0;
  if (P.rec_lin >= 0 && P.first_blk == SPLIT_FROM_SBI) {  // .sbi chunk: both ends are pointers
    const int64_t b = lower_bound_u64(voffset, nrec, P.vstart);
    if (b >= nrec || voffset[b] != P.vstart) {
      atomicCAS(d_status, 0, 102);  // indexed offset is not a record start (a short record wins)
    } else {
      const int64_t e = lower_bound_u64(voffset, nrec, P.vend);
      r.begin = b;
      r.end = e < b ? b : e;
    }
  } else if (P.rec_lin >= 0) {
    int64_t b = lower_bound_i64(rec_lin, nrec, P.rec_lin);
    if (b >= nrec || rec_lin[b] != P.rec_lin) {
      atomicCAS(d_status, 0, 101);  // guesser start not on the record chain (misfire)
    } else {
      int64_t e = lower_bound_u64(voffset, nrec, P.vend);
      r.begin = b;
      r.end = e < b ? b : e;
    }
  }
  parts[i] = r;
}

// .sbi entries (SBIIndexWriter.processRecord, M/htsjdk/samtools/SBIIndexWriter.java:84-88):
// the virtual offset of every g-th record, counted from the first
__global__ __launch_bounds__(256) void sbi_sample_kernel(const uint64_t* __restrict__ voffset,
                                                         int64_t nrec, int64_t g,
                                                         uint64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i * g < nrec) out[i] = voffset[i * g];
}

// grid (partition, DIG_SPLIT): block y of partition x sums every DIG_SPLIT-th group of 256 records
// and adds its sum to the partition digest (zeroed by partition_ranges_kernel)
constexpr int DIG_SPLIT = 64;
__global__ __launch_bounds__(256) void partition_digest_kernel(const uint64_t* __restrict__ hash,
                                                               PartRange* __restrict__ parts,
                                                               int64_t nparts) {
  __shared__ uint64_t red[256];
  const int64_t i = blockIdx.x;
  if (i >= nparts) return;
  const PartRange r = parts[i];
  uint64_t acc = 0;
  for (int64_t k = r.begin + (int64_t)blockIdx.y * 256 + threadIdx.x; k < r.end;
       k += 256 * DIG_SPLIT)
    acc += dq_mix64(hash[k] + (uint64_t)(k - r.begin + 1) * DQ_K_LEN);
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0 && red[0]) atomicAdd(reinterpret_cast<unsigned long long*>(&parts[i].digest),
                                            (unsigned long long)red[0]);
}

// ------------------------------------------------------------------ Kernel 4: interval filter
// BAMQueryMultipleIntervalsIteratorFilter.compareIntervalToRecord with contained=false on
// optimized (sorted, merged) QueryIntervals: a record matches iff an interval on its reference
// has start <= alignmentEnd and end >= alignmentStart.  alignmentEnd = pos + refLen(CIGAR
// M/D/N/=/X) for mapped reads, alignmentStart for unmapped reads with a position, 0 otherwise.
__global__ __launch_bounds__(256) void interval_filter_kernel(
    const uint8_t* __restrict__ U, const int64_t* __restrict__ rec_lin, RecSoA soa,
    const int64_t* __restrict__ idx, int64_t n, const int32_t* __restrict__ iv_ref,
    const int32_t* __restrict__ iv_start, const int32_t* __restrict__ iv_end,
    const int32_t* __restrict__ ref_iv_begin, int32_t n_ref, uint8_t* __restrict__ keep) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const int64_t i = idx ? idx[t] : t;
  const int32_t ref = soa.ref_id[i];
  uint8_t k = 0;
  if (ref >= 0 && ref < n_ref) {
    const int32_t astart = soa.pos[i] + 1;
    const uint16_t flag = soa.flag[i];
    int32_t aend;
    if (flag & 4) {
      aend = astart != 0 ? astart : 0;
    } else {
      const int64_t p = rec_lin[i];
      const int64_t cp = p + 36 + soa.l_read_name[i];
      const int nc = soa.n_cigar[i];
      int32_t rl = 0;
      if (32 + (int64_t)soa.l_read_name[i] + 4 * (int64_t)nc <= soa.block_size[i]) {
        for (int c = 0; c < nc; c++) {
          uint32_t op = (uint32_t)ld32(U, cp + 4 * c);
          uint32_t o = op & 0xf;
          if (o == 0 || o == 2 || o == 3 || o == 7 || o == 8) rl += (int32_t)(op >> 4);
        }
      }
      aend = astart + rl - 1;
    }
    int32_t lo = ref_iv_begin[ref], hi = ref_iv_begin[ref + 1];
    // last interval with start <= aend (intervals on one reference are sorted and disjoint)
    int32_t a = lo, b = hi;
    while (a < b) {
      int32_t m = (a + b) >> 1;
      if (iv_start[m] <= aend) a = m + 1;
      else b = m;
    }
    if (a > lo) {
      int32_t e = iv_end[a - 1];
      if (e <= 0) e = INT32_MAX;
      if (e >= astart) k = 1;
    }
  }
  keep[t] = k;
}

// ------------------------------------------------------------------ windowed record chains
// Sparse runs (an interval traversal's .bai spans, AbstractBinarySamSource.java:102-112) inflate
// only some blocks, in the whole-file U layout: each window is a run of inflated bytes whose first
// record start is exact (a span chunk start).  The segmented chain of Kernel 3 runs inside every
// window at once; a window's reads stop at its inflated end (status 4: needs more blocks).
__device__ inline int64_t win_of(const Win* __restrict__ w, int64_t nwin, int64_t s) {
  int64_t lo = 0, hi = nwin - 1;  // last window with seg0 <= s
  while (lo < hi) {
    const int64_t mid = (lo + hi + 1) >> 1;
    if (w[mid].seg0 <= s) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__global__ __launch_bounds__(64) void wseg_spec_kernel(const uint8_t* __restrict__ U,
                                                       const int32_t* __restrict__ ref_len,
                                                       int32_t n_ref, const Win* __restrict__ wins,
                                                       int64_t nwin, Seg* __restrict__ segs,
                                                       int64_t nseg, int64_t seg_bytes) {
  for (int64_t s = blockIdx.x; s < nseg; s += gridDim.x) {
    const Win w = wins[win_of(wins, nwin, s)];
    const int64_t k = s - w.seg0;
    const int64_t sb = w.u_start + k * seg_bytes;
    const int64_t se = min(w.u_chain_end, sb + seg_bytes);
    int64_t best = INT64_MAX;
    if (k == 0) {
      best = w.u_start;
    } else {
      for (int64_t b = sb; b < se; b += 64) {
        const int64_t v = b + threadIdx.x;
        const bool hit =
            v < se && check_record_start<3>(U, w.u_limit, w.at_eof, ref_len, n_ref, v) == 1;
        const uint64_t m = __ballot(hit);
        if (m) {
          best = b + __builtin_ctzll(m);
          break;
        }
      }
    }
    if (threadIdx.x == 0) {
      Seg g;
      g.exact = k == 0;
      g.status = 0;
      g.start = best == INT64_MAX ? -1 : best;
      g.exit = -1;
      g.count = 0;
      segs[s] = g;
    }
  }
}

__global__ __launch_bounds__(256) void wseg_walk_kernel(const uint8_t* __restrict__ U,
                                                        const Win* __restrict__ wins, int64_t nwin,
                                                        Seg* __restrict__ segs, int64_t nseg,
                                                        int64_t seg_bytes) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nseg) return;
  Seg g = segs[s];
  if (g.start < 0) return;
  const Win w = wins[win_of(wins, nwin, s)];
  const int64_t se = min(w.u_chain_end, w.u_start + (s - w.seg0 + 1) * seg_bytes);
  int64_t ex = -1, cnt = 0;
  const int r = walk_win(U, w.u_limit, w.at_eof, g.start, se, &ex, &cnt);
  g.status = r;
  if (r == 0) {
    g.exit = ex;
    g.count = cnt;
  }
  segs[s] = g;
}

__global__ void wseg_link_kernel(const Seg* __restrict__ segs, const Win* __restrict__ wins,
                                 int64_t nwin, int64_t nseg, int64_t seg_bytes,
                                 int32_t* d_broken) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nseg) return;
  const Seg g = segs[s];
  if (g.status != 0) {
    *d_broken = 1;
    return;
  }
  const Win w = wins[win_of(wins, nwin, s)];
  if (s == w.seg0) return;
  int64_t t = s - 1;
  while (t > w.seg0 && segs[t].start < 0) t--;
  const int64_t in = segs[t].exit;
  const int64_t se = min(w.u_chain_end, w.u_start + (s - w.seg0 + 1) * seg_bytes);
  const bool ok = g.start < 0 ? (in == END_CHAIN || in >= se) : (in == g.start);
  if (!ok) *d_broken = 1;
}

// Serial link check + repair, one lane per window (as seg_fix_kernel, inside each window).
__global__ void wseg_fix_kernel(const uint8_t* __restrict__ U, Seg* __restrict__ segs,
                                const Win* __restrict__ wins, int64_t nwin, int64_t nseg,
                                int64_t seg_bytes, int32_t* d_status) {
  const int64_t wi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (wi >= nwin) return;
  const Win w = wins[wi];
  const int64_t s1 = wi + 1 < nwin ? wins[wi + 1].seg0 : nseg;
  if (s1 <= w.seg0) return;
  if (segs[w.seg0].status) {
    atomicMax(d_status, segs[w.seg0].status);
    return;
  }
  int64_t in = segs[w.seg0].exit;
  for (int64_t s = w.seg0 + 1; s < s1; s++) {
    Seg& g = segs[s];
    const int64_t sb = w.u_start + (s - w.seg0) * seg_bytes;
    const int64_t se = min(w.u_chain_end, sb + seg_bytes);
    if (in == END_CHAIN || in >= se) {
      g.start = in;
      g.exit = in;
      g.count = 0;
      g.exact = 1;
      g.status = 0;
      continue;
    }
    if (g.start != in || g.status != 0) {
      int64_t ex = -1, cnt = 0;
      const int r = walk_win(U, w.u_limit, w.at_eof, in, se, &ex, &cnt);
      g.start = in;
      g.status = r;
      g.exit = ex;
      g.count = cnt;
      if (r) {
        atomicMax(d_status, r);
        return;
      }
    }
    g.exact = 1;
    in = g.exit;
  }
}

// Records of the span chunks, in partition order: chunk j selects the records whose start pointer
// is in [beg_j, end_j) (BAMFileIndexIterator over the chunk list, H/BAMFileReader2.java:1082-1095).
__global__ __launch_bounds__(256) void span_ranges_kernel(const uint64_t* __restrict__ voffset,
                                                          int64_t nrec,
                                                          const uint64_t* __restrict__ cbeg,
                                                          const uint64_t* __restrict__ cend,
                                                          int64_t nchunk, int64_t* __restrict__ first,
                                                          int64_t* __restrict__ count) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nchunk) return;
  const int64_t a = lower_bound_u64(voffset, nrec, cbeg[j]);
  const int64_t b = lower_bound_u64(voffset, nrec, cend[j]);
  first[j] = a;
  count[j] = b > a ? b - a : 0;
}

// kept[off[i]] = idx[i] for every kept record (off = exclusive scan of keep).
__global__ __launch_bounds__(256) void compact_kept_kernel(const int64_t* __restrict__ idx,
                                                           const uint8_t* __restrict__ keep,
                                                           const int64_t* __restrict__ off, int64_t n,
                                                           int64_t* __restrict__ kept) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && keep[i]) kept[off[i]] = idx ? idx[i] : i;
}

__global__ __launch_bounds__(256) void keep_to_i32_kernel(const uint8_t* __restrict__ keep, int64_t n,
                                                          int32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = keep[i];
}

// Partition digests over an index list: partition p = kept[begin_p, end_p) (same definition as
// partition_digest_kernel: sum of mix64(hash + (k + 1) * K_LEN) in order).
__global__ __launch_bounds__(256) void partition_digest_idx_kernel(const uint64_t* __restrict__ hash,
                                                                   const int64_t* __restrict__ kept,
                                                                   PartRange* __restrict__ parts,
                                                                   int64_t nparts) {
  __shared__ uint64_t red[256];
  const int64_t i = blockIdx.x;
  if (i >= nparts) return;
  const PartRange r = parts[i];
  uint64_t acc = 0;
  for (int64_t k = r.begin + (int64_t)blockIdx.y * 256 + threadIdx.x; k < r.end; k += 256 * 64)
    acc += dq_mix64(hash[kept[k]] + (uint64_t)(k - r.begin + 1) * DQ_K_LEN);
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0 && red[0])
    atomicAdd(reinterpret_cast<unsigned long long*>(&parts[i].digest), (unsigned long long)red[0]);
}

__global__ __launch_bounds__(256) void gather_i64_kernel(const int64_t* __restrict__ src,
                                                         const int64_t* __restrict__ pos, int64_t n,
                                                         int64_t* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[pos[i]];
}

// ------------------------------------------------------------------ record export (gathers)
// idx[o_r + k] = begin_r + k for record-index ranges r (one block per range).
__global__ __launch_bounds__(256) void ranges_to_idx_kernel(const int64_t* __restrict__ begin,
                                                            const int64_t* __restrict__ out_off,
                                                            int64_t nranges, int64_t* __restrict__ idx) {
  const int64_t r = blockIdx.x;
  if (r >= nranges) return;
  const int64_t b = begin[r], o = out_off[r], n = out_off[r + 1] - o;
  for (int64_t k = threadIdx.x; k < n; k += blockDim.x) idx[o + k] = b + k;
}

// dst row t = src row idx[t] for every SoA field (the batch a Spark task receives, compacted on
// the device so only the selected records cross PCIe).
__global__ __launch_bounds__(256) void gather_soa_kernel(const int64_t* __restrict__ idx, int64_t n,
                                                         RecSoA src, RecSoA dst) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const int64_t i = idx[t];
  dst.voffset[t] = src.voffset[i];
  dst.block_size[t] = src.block_size[i];
  dst.ref_id[t] = src.ref_id[i];
  dst.pos[t] = src.pos[i];
  dst.l_seq[t] = src.l_seq[i];
  dst.next_ref_id[t] = src.next_ref_id[i];
  dst.next_pos[t] = src.next_pos[i];
  dst.tlen[t] = src.tlen[i];
  dst.flag[t] = src.flag[i];
  dst.bin[t] = src.bin[i];
  dst.n_cigar[t] = src.n_cigar[i];
  dst.mapq[t] = src.mapq[i];
  dst.l_read_name[t] = src.l_read_name[i];
  dst.hash[t] = src.hash[i];
}

// The raw bytes (4 + block_size) of record idx[t] (or first + t when idx is null) to
// out[out_off[t] ...]: one wave per record.
__global__ __launch_bounds__(256) void gather_raw_kernel(const uint8_t* __restrict__ U,
                                                         const int64_t* __restrict__ rec_lin,
                                                         const int32_t* __restrict__ block_size,
                                                         const int64_t* __restrict__ idx,
                                                         int64_t first, int64_t n,
                                                         const int64_t* __restrict__ out_off,
                                                         uint8_t* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= n) return;
  const int lane = threadIdx.x & 63;
  const int64_t i = idx ? idx[t] : first + t;
  const int64_t src = rec_lin[i], len = 4 + (int64_t)block_size[i], o = out_off[t];
  for (int64_t k = lane; k < len; k += 64) out[o + k] = U[src + k];
}

}  // namespace

// ------------------------------------------------------------------ launchers
void launch_bgzf_scan(const uint8_t* C, int64_t n, int64_t L, Cand* slots_out, int64_t cap,
                      int32_t* chunk_counts, int64_t n_chunks, int64_t* d_count,
                      int32_t* over_list, hipStream_t s) {
  (void)cap;
  (void)d_count;
  if (n_chunks <= 0) return;
  hipLaunchKernelGGL((bgzf_scan_kernel<SCAN_CAP, false>), dim3((unsigned)n_chunks), dim3(256), 0, s,
                     C, n, L, slots_out, chunk_counts, over_list, nullptr);
}

void launch_bgzf_scan_listed(const uint8_t* C, int64_t n, int64_t L, Cand* big, int64_t n_over,
                             int32_t* chunk_counts, int32_t* over_list, int32_t* over_map,
                             hipStream_t s) {
  if (n_over <= 0) return;
  hipLaunchKernelGGL((bgzf_scan_kernel<SCAN_CAP_BIG, true>), dim3((unsigned)n_over), dim3(256), 0,
                     s, C, n, L, big, chunk_counts, over_list, over_map);
}

void launch_gather_slots(const Cand* slots, const int32_t* counts, const int64_t* offs,
                         int64_t nchunks, Cand* out, int64_t cap, const int32_t* over_map,
                         const Cand* big, hipStream_t s) {
  hipLaunchKernelGGL(gather_slots_kernel, dim3((unsigned)nchunks), dim3(64), 0, s, slots, counts,
                     offs, nchunks, out, cap, over_map, big);
}

void launch_exclusive_scan_i32(const int32_t* in, int64_t* out, int64_t n, int64_t* tmp,
                               hipStream_t s) {
  exclusive_scan<int32_t>(in, out, n, tmp, s);
}
void launch_exclusive_scan_i64(const int64_t* in, int64_t* out, int64_t n, int64_t* tmp,
                               hipStream_t s) {
  exclusive_scan<int64_t>(in, out, n, tmp, s);
}

void launch_valid_flags(const Cand* cand, const int64_t* ncand, int64_t cap, int32_t* flags,
                        hipStream_t s) {
  hipLaunchKernelGGL(valid_flags_kernel, dim3((unsigned)((cap + 255) / 256)), dim3(256), 0, s,
                     cand, ncand, flags);
}

void launch_chain2(const uint8_t* C, int64_t L, const Cand* cand, const int64_t* ncand, int64_t cap,
                   const int64_t* voff, int64_t* blk_pos, int32_t* blk_csize, int32_t* blk_usize,
                   int64_t blk_cap, int64_t* d_nblk, int32_t* d_broken, int32_t eof_in_buf,
                   hipStream_t s) {
  hipLaunchKernelGGL(chain_kernel, dim3((unsigned)((cap + 255) / 256)), dim3(256), 0, s, C, L, cand,
                     ncand, voff, blk_pos, blk_csize, blk_usize, blk_cap, d_nblk, d_broken,
                     eof_in_buf);
}

// Chain start of a shard (the first valid candidate: the guesser's first block of its first
// split) as a device min-reduction, plus a copy of the chain's first block position, so the host
// reads both with the block count in one small copy.  out[0] = min valid pos (initialised to
// all ones by the caller), out[1] = blk_pos[0].
__global__ void chain_check_kernel(const Cand* __restrict__ cand, const int64_t* __restrict__ ncand,
                                   const int64_t* __restrict__ blk_pos, const int64_t* __restrict__ d_nblk,
                                   unsigned long long* __restrict__ out) {
  const int64_t n = *ncand;
  unsigned long long best = ~0ull;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (cand[i].valid == 1) best = min(best, (unsigned long long)cand[i].pos);
  for (int o = 32; o >= 1; o >>= 1) best = min(best, (unsigned long long)__shfl_xor(best, o, 64));
  if ((threadIdx.x & 63) == 0 && best != ~0ull) atomicMin(&out[0], best);
  if (blockIdx.x == 0 && threadIdx.x == 0) out[1] = *d_nblk > 0 ? (unsigned long long)blk_pos[0] : ~0ull;
}

// First block whose status is not ST_OK: a device min-reduction of the block index into out[0]
// (initialised to all ones by the caller); the host reads one word instead of the status array.
__global__ void first_bad_kernel(const int32_t* __restrict__ status, const int32_t* __restrict__ sel,
                                 int64_t n, unsigned long long* __restrict__ out) {
  unsigned long long best = ~0ull;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = sel ? (int64_t)sel[i] : i;
    if (status[b] != 0) best = min(best, (unsigned long long)b);
  }
  for (int o = 32; o >= 1; o >>= 1) best = min(best, (unsigned long long)__shfl_xor(best, o, 64));
  if ((threadIdx.x & 63) == 0 && best != ~0ull) atomicMin(out, best);
}

void launch_chain_check(const Cand* cand, const int64_t* d_ncand, int64_t cap, const int64_t* blk_pos,
                        const int64_t* d_nblk, unsigned long long* out, hipStream_t s) {
  const unsigned g = (unsigned)std::min<int64_t>(1024, std::max<int64_t>(1, (cap + 255) / 256));
  hipLaunchKernelGGL(chain_check_kernel, dim3(g), dim3(256), 0, s, cand, d_ncand, blk_pos, d_nblk, out);
}

void launch_first_bad(const int32_t* status, const int32_t* sel, int64_t n, unsigned long long* out,
                      hipStream_t s) {
  if (n <= 0) return;
  const unsigned g = (unsigned)std::min<int64_t>(1024, (n + 255) / 256);
  hipLaunchKernelGGL(first_bad_kernel, dim3(g), dim3(256), 0, s, status, sel, n, out);
}

void launch_chain_serial(const uint8_t* C, int64_t clen, int64_t start, int64_t* blk_pos,
                         int32_t* blk_csize, int32_t* blk_usize, int64_t cap, int64_t* d_nblk,
                         int32_t* d_status, hipStream_t s) {
  hipLaunchKernelGGL(chain_serial_kernel, dim3(1), dim3(64), 0, s, C, clen, start, blk_pos,
                     blk_csize, blk_usize, cap, d_nblk, d_status);
}

void launch_plan_blocks(const Cand* cand, const int64_t* d_ncand, const int64_t* blk_pos,
                        const int32_t* blk_usize, const int64_t* uoff, const int64_t* d_nblk,
                        SplitPlan* plans, int64_t nsplit, hipStream_t s) {
  if (nsplit <= 0) return;
  hipLaunchKernelGGL(plan_blocks_kernel, dim3((unsigned)((nsplit + 63) / 64)), dim3(64), 0, s,
                     cand, d_ncand, blk_pos, blk_usize, uoff, d_nblk, plans, nsplit);
}

// Guesser at every position of the resident stream (BamRecordGuesserChecker's exhaustive check,
// D/impl/formats/bam/BamRecordGuesserChecker.java:104-120): flag[x] = checkRecordStart(x).
__global__ void guess_all_kernel(const uint8_t* U, int64_t ulen, int32_t u_is_eof,
                                 const int32_t* ref_len, int32_t n_ref, uint8_t* flag) {
  const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= ulen) return;
  flag[x] = (uint8_t)check_record_start(U, ulen, u_is_eof, ref_len, n_ref, x);
}

void launch_guess_all(const uint8_t* U, int64_t ulen, int32_t u_is_eof, const int32_t* ref_len,
                      int32_t n_ref, uint8_t* flag, hipStream_t s) {
  if (ulen <= 0) return;
  hipLaunchKernelGGL(guess_all_kernel, dim3((unsigned)((ulen + 255) / 256)), dim3(256), 0, s, U,
                     ulen, u_is_eof, ref_len, n_ref, flag);
}

void launch_first_record(const uint8_t* U, int64_t ulen, int32_t u_is_eof, const int32_t* ref_len,
                         int32_t n_ref, const int64_t* blk_pos, const int64_t* uoff,
                         const int64_t* d_nblk, SplitPlan* plans, int64_t nsplit,
                         unsigned long long* best, hipStream_t s) {
  if (nsplit <= 0) return;
  (void)hipMemsetAsync(best, 0xff, 8 * (size_t)nsplit, s);       // minima: all ones
  (void)hipMemsetAsync(best + nsplit, 0, 8 * (size_t)nsplit, s);  // "need more data" flags
  hipLaunchKernelGGL(first_record_kernel, dim3((unsigned)(nsplit * FR_K)), dim3(256), 0, s, U, ulen,
                     u_is_eof, ref_len, n_ref, plans, nsplit, best);
  hipLaunchKernelGGL(first_record_final_kernel, dim3((unsigned)((nsplit + 63) / 64)), dim3(64), 0, s,
                     U, ulen, u_is_eof, ref_len, n_ref, blk_pos, uoff, d_nblk, plans, nsplit, best);
}

void launch_seg_spec(const uint8_t* U, int64_t ulen, int32_t u_is_eof, int64_t chain_end,
                     const int32_t* ref_len,
                     int32_t n_ref, Seg* segs, int64_t nseg, int64_t seg_bytes, int64_t start_lin,
                     uint16_t* offs, hipStream_t s) {
  if (nseg <= 0) return;
  if (seg_bytes > 64 * 1024)  // long records (segments sized from the guesser's record span)
    hipLaunchKernelGGL(seg_spec_kernel<256>, dim3((unsigned)std::min<int64_t>(nseg, 16384)), dim3(256), 0, s, U,
                       ulen, u_is_eof, ref_len, n_ref, segs, nseg, seg_bytes, start_lin, chain_end);
  else if (DQ_SPEC_LDS == 2)
    hipLaunchKernelGGL(seg_spec_split_kernel<DQ_SPEC_SL>, dim3((unsigned)std::min<int64_t>((nseg + 64 / DQ_SPEC_SL - 1) / (64 / DQ_SPEC_SL), 16384)),
                       dim3(64), 0, s, U, ulen, u_is_eof, ref_len, n_ref, segs, nseg, seg_bytes, start_lin, chain_end);
  else if (DQ_SPEC_LDS == 1)
    hipLaunchKernelGGL(seg_spec_lds_kernel, dim3((unsigned)std::min<int64_t>(nseg, 16384)), dim3(64), 0, s, U,
                       ulen, u_is_eof, ref_len, n_ref, segs, nseg, seg_bytes, start_lin, chain_end);
  else
    hipLaunchKernelGGL(seg_spec_kernel<64>, dim3((unsigned)std::min<int64_t>(nseg, 16384)), dim3(64), 0, s, U,
                       ulen, u_is_eof, ref_len, n_ref, segs, nseg, seg_bytes, start_lin, chain_end);
#ifdef DQ_CHECKED
  if (seg_bytes <= 64 * 1024 && DQ_SPEC_LDS) {  // the filtered search finds seg_spec_kernel<64>'s starts
    Seg* ref = nullptr;
    if (hipMalloc(&ref, sizeof(Seg) * (size_t)nseg) == hipSuccess) {
      hipLaunchKernelGGL(seg_spec_kernel<64>, dim3((unsigned)std::min<int64_t>(nseg, 16384)), dim3(64), 0, s, U,
                         ulen, u_is_eof, ref_len, n_ref, ref, nseg, seg_bytes, start_lin, chain_end);
      hipLaunchKernelGGL(spec_cmp_kernel, dim3((unsigned)((nseg + 255) / 256)), dim3(256), 0, s, segs, ref, nseg);
      (void)hipStreamSynchronize(s);
      (void)hipFree(ref);
    }
  }
#endif
#ifdef DQ_REC_TIMING
  {
    unsigned long long h[8] = {0};
    (void)hipStreamSynchronize(s);
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_rec_tim), sizeof(h));
    fprintf(stderr, "[dq] seg_spec cycles summed over waves: staging=%.3g prefilter=%.3g full_checks=%.3g; "
            "steps with a full check %.3g, candidates passing the prefilter %.3g, segments %lld\n",
            (double)h[0], (double)h[1], (double)h[2], (double)h[3], (double)h[7], (long long)nseg);
    const unsigned long long z[8] = {0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_rec_tim), z, sizeof(z));
  }
#endif
  hipLaunchKernelGGL(seg_walk_kernel, dim3((unsigned)((nseg + 255) / 256)), dim3(256), 0, s, U, ulen,
                     u_is_eof, segs, nseg, seg_bytes, start_lin, chain_end,
                     seg_bytes <= 65536 ? offs : nullptr);
}

void launch_seg_fix2(const uint8_t* U, int64_t ulen, int32_t u_is_eof, int64_t chain_end,
                     Seg* segs, int64_t nseg, int64_t seg_bytes, int64_t start_lin,
                     int32_t* d_status, hipStream_t s) {
  hipLaunchKernelGGL(seg_fix_kernel, dim3(1), dim3(64), 0, s, U, ulen, u_is_eof, segs, nseg,
                     seg_bytes, start_lin, chain_end, d_status);
}

void launch_seg_link(const Seg* segs, int64_t nseg, int64_t seg_bytes, int64_t start_lin,
                     int64_t ulen, int32_t* d_broken, hipStream_t s) {
  if (nseg <= 0) return;
  hipLaunchKernelGGL(seg_link_kernel, dim3((unsigned)((nseg + 255) / 256)), dim3(256), 0, s, segs,
                     nseg, seg_bytes, start_lin, ulen, d_broken);
}

void launch_seg_counts(const Seg* segs, int64_t nseg, int64_t* counts, hipStream_t s) {
  hipLaunchKernelGGL(seg_counts_kernel, dim3((unsigned)((nseg + 255) / 256)), dim3(256), 0, s,
                     segs, nseg, counts);
}

void launch_seg_emit2(const uint8_t* U, int64_t, const Seg* segs, const int64_t* base,
                      int64_t nseg, int64_t* rec_lin, hipStream_t s, const uint16_t* offs,
                      int64_t seg_bytes, int64_t start_lin) {
  hipLaunchKernelGGL(seg_emit_kernel, dim3((unsigned)((nseg + 63) / 64)), dim3(64), 0, s, U, segs,
                     base, nseg, rec_lin);
  if (offs && seg_bytes <= 65536)
    hipLaunchKernelGGL(seg_copy_kernel, dim3((unsigned)std::min<int64_t>(nseg, 32768)), dim3(64), 0, s,
                       segs, base, nseg, offs, seg_bytes, start_lin, rec_lin);
}

void launch_block_stats(const int64_t* blk_pos, const int32_t* blk_cs, const int64_t* uoff,
                        int64_t nblk, int64_t ulen, int64_t x, uint64_t* out, hipStream_t s) {
  (void)hipMemsetAsync(out, 0, 4 * sizeof(uint64_t), s);
  const int64_t g = std::max<int64_t>(1, std::min<int64_t>(1024, (nblk + 255) / 256));
  hipLaunchKernelGGL(block_stats_kernel, dim3((unsigned)g), dim3(256), 0, s, blk_pos, blk_cs, uoff,
                     nblk, ulen, x, out);
}

int64_t long_list_cap(int64_t ulen, int64_t nrec) {
  return ulen / LONG_PIECE + std::min(nrec, ulen / LONG_N) + 1;
}

void launch_decode_records(const uint8_t* U, int64_t ulen, const int64_t* rec_lin, int64_t nrec,
                           const int64_t* blk_pos, const int64_t* uoff, int64_t nblk, int32_t* pt,
                           RecSoA soa, int32_t* d_status, uint64_t* long_ent, int64_t long_cap,
                           unsigned long long* long_cnt, hipStream_t s) {
  if (nrec <= 0 || nblk <= 0) return;
  const int64_t npages = (ulen >> 16) + 1;
  hipLaunchKernelGGL(block_pages_kernel, dim3((unsigned)((npages + 255) / 256)), dim3(256), 0, s,
                     uoff, nblk, pt, npages);
  (void)hipMemsetAsync(long_cnt, 0, sizeof(unsigned long long), s);
  const LongList ll{long_ent, long_cap, long_cnt};
  const int64_t ngroup = (nrec + REC_GROUP - 1) / REC_GROUP;
  hipLaunchKernelGGL(decode_records_kernel, dim3((unsigned)std::min<int64_t>(ngroup, 16384)),
                     dim3(REC_WAVE), 0, s, U, ulen, rec_lin, nrec, blk_pos, uoff, nblk, pt, soa,
                     d_status, ll);
#ifdef DQ_REC_TIMING
  {
    unsigned long long h[8] = {0};
    (void)hipStreamSynchronize(s);
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_rec_tim), sizeof(h));
    fprintf(stderr, "[dq] decode_records cycles summed over waves: index=%.3g staging=%.3g decode=%.3g\n",
            (double)h[4], (double)h[5], (double)h[6]);
    const unsigned long long z[8] = {0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_rec_tim), z, sizeof(z));
  }
#endif
  // the long records' pieces (an empty list costs two tiny launches that read the count)
  hipLaunchKernelGGL(long_hash_kernel, dim3(2048), dim3(LH_THREADS), 0, s, U, rec_lin, long_ent,
                     long_cnt, long_cap, soa.hash);
  hipLaunchKernelGGL(long_hash_final_kernel, dim3(64), dim3(256), 0, s, U, rec_lin, long_ent,
                     long_cnt, long_cap, soa.hash);
}

void launch_partition_ranges(const SplitPlan* plans, int64_t nsplit, const int64_t* rec_lin,
                             const uint64_t* voffset, int64_t nrec, PartRange* parts,
                             int32_t* d_status, hipStream_t s) {
  if (nsplit <= 0) return;
  hipLaunchKernelGGL(partition_ranges_kernel, dim3((unsigned)((nsplit + 63) / 64)), dim3(64), 0, s,
                     plans, nsplit, rec_lin, voffset, nrec, parts, d_status);
}

// Batch export helpers: 4 + block_size of each record (the raw-offset scan's input), and voffsets
// translated by a shard's base.
__global__ void bs_plus4_kernel(const int32_t* __restrict__ bs, int64_t n, int32_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = 4 + bs[i];
}
__global__ void add_u64_kernel(const uint64_t* __restrict__ in, int64_t n, uint64_t add,
                               uint64_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = in[i] + add;
}
void launch_bs_plus4(const int32_t* bs, int64_t n, int32_t* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(bs_plus4_kernel, dim3((unsigned)std::min<int64_t>(4096, (n + 255) / 256)),
                     dim3(256), 0, s, bs, n, out);
}
void launch_add_u64(const uint64_t* in, int64_t n, uint64_t add, uint64_t* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(add_u64_kernel, dim3((unsigned)std::min<int64_t>(4096, (n + 255) / 256)),
                     dim3(256), 0, s, in, n, add, out);
}

void launch_partition_digest2(const uint64_t* hash, PartRange* parts, int64_t nparts, hipStream_t s) {
  if (nparts <= 0) return;
  hipLaunchKernelGGL(partition_digest_kernel, dim3((unsigned)nparts, DIG_SPLIT), dim3(256), 0, s,
                     hash, parts, nparts);
}

void launch_interval_filter(const uint8_t* U, const int64_t* rec_lin, const RecSoA soa,
                            const int64_t* idx, int64_t n, const int32_t* iv_ref,
                            const int32_t* iv_start, const int32_t* iv_end,
                            const int32_t* ref_iv_begin, int32_t n_ref, uint8_t* keep,
                            hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(interval_filter_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, U,
                     rec_lin, soa, idx, n, iv_ref, iv_start, iv_end, ref_iv_begin, n_ref, keep);
}

void launch_sbi_sample(const uint64_t* voffset, int64_t nrec, int64_t g, uint64_t* out,
                       hipStream_t s) {
  const int64_t n = (nrec + g - 1) / g;
  if (n <= 0) return;
  hipLaunchKernelGGL(sbi_sample_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, voffset,
                     nrec, g, out);
}

void launch_ranges_to_idx(const int64_t* begin, const int64_t* out_off, int64_t nranges,
                          int64_t* idx, hipStream_t s) {
  if (nranges <= 0) return;
  hipLaunchKernelGGL(ranges_to_idx_kernel, dim3((unsigned)nranges), dim3(256), 0, s, begin, out_off,
                     nranges, idx);
}

void launch_gather_soa(const int64_t* idx, int64_t n, const RecSoA src, RecSoA dst, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(gather_soa_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, idx, n,
                     src, dst);
}

void launch_gather_raw(const uint8_t* U, const int64_t* rec_lin, const int32_t* block_size,
                       const int64_t* idx, int64_t first, int64_t n, const int64_t* out_off,
                       uint8_t* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(gather_raw_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, U, rec_lin,
                     block_size, idx, first, n, out_off, out);
}

void launch_wseg(const uint8_t* U, const int32_t* ref_len, int32_t n_ref, const Win* wins,
                 int64_t nwin, Seg* segs, int64_t nseg, int64_t seg_bytes, int32_t* d_broken,
                 hipStream_t s) {
  if (nseg <= 0) return;
  hipLaunchKernelGGL(wseg_spec_kernel, dim3((unsigned)std::min<int64_t>(nseg, 16384)), dim3(64), 0, s,
                     U, ref_len, n_ref, wins, nwin, segs, nseg, seg_bytes);
  hipLaunchKernelGGL(wseg_walk_kernel, dim3((unsigned)((nseg + 255) / 256)), dim3(256), 0, s, U, wins,
                     nwin, segs, nseg, seg_bytes);
  hipLaunchKernelGGL(wseg_link_kernel, dim3((unsigned)((nseg + 255) / 256)), dim3(256), 0, s, segs,
                     wins, nwin, nseg, seg_bytes, d_broken);
}

void launch_wseg_fix(const uint8_t* U, Seg* segs, const Win* wins, int64_t nwin, int64_t nseg,
                     int64_t seg_bytes, int32_t* d_status, hipStream_t s) {
  if (nwin <= 0) return;
  hipLaunchKernelGGL(wseg_fix_kernel, dim3((unsigned)((nwin + 63) / 64)), dim3(64), 0, s, U, segs,
                     wins, nwin, nseg, seg_bytes, d_status);
}

void launch_span_ranges(const uint64_t* voffset, int64_t nrec, const uint64_t* cbeg,
                        const uint64_t* cend, int64_t nchunk, int64_t* first, int64_t* count,
                        hipStream_t s) {
  if (nchunk <= 0) return;
  hipLaunchKernelGGL(span_ranges_kernel, dim3((unsigned)((nchunk + 255) / 256)), dim3(256), 0, s,
                     voffset, nrec, cbeg, cend, nchunk, first, count);
}

// The unplaced-unmapped tail of a span run (BAMFileIndexUnmappedIterator, H/BAMFileReader2.java:
// 1199-1206, after queryUnmapped's seek to the start of the last linear bin): of the records
// idx[off[k]], .. idx[off[k+1]-1] of the tail chunk k, skip until the first with refID == -1 and
// keep every one from there.  Pass 1: the first such entry (min-reduction into *first, initialised
// to all ones); pass 2: the keep flags of the chunk's entries.
__global__ void tail_first_kernel(const int64_t* __restrict__ idx, const int64_t* __restrict__ off, int k,
                                  const int32_t* __restrict__ ref, unsigned long long* __restrict__ first) {
  const int64_t a = off[k], b = off[k + 1];
  unsigned long long best = ~0ull;
  for (int64_t i = a + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < b; i += (int64_t)gridDim.x * blockDim.x)
    if (ref[idx[i]] == -1) best = min(best, (unsigned long long)i);
  for (int o = 32; o >= 1; o >>= 1) best = min(best, (unsigned long long)__shfl_xor(best, o, 64));
  if ((threadIdx.x & 63) == 0 && best != ~0ull) atomicMin(first, best);
}
__global__ void tail_keep_kernel(const int64_t* __restrict__ off, int k,
                                 const unsigned long long* __restrict__ first, uint8_t* __restrict__ keep) {
  const int64_t a = off[k], b = off[k + 1];
  const unsigned long long f = *first;
  for (int64_t i = a + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < b; i += (int64_t)gridDim.x * blockDim.x)
    keep[i] = (unsigned long long)i >= f ? 1 : 0;
}
void launch_tail_keep(const int64_t* idx, const int64_t* off, int k, const int32_t* ref,
                      unsigned long long* first, uint8_t* keep, int64_t max_n, hipStream_t s) {
  const unsigned g = (unsigned)std::min<int64_t>(1024, std::max<int64_t>(1, (max_n + 255) / 256));
  hipLaunchKernelGGL(tail_first_kernel, dim3(g), dim3(256), 0, s, idx, off, k, ref, first);
  hipLaunchKernelGGL(tail_keep_kernel, dim3(g), dim3(256), 0, s, off, k, first, keep);
}

void launch_keep_to_i32(const uint8_t* keep, int64_t n, int32_t* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(keep_to_i32_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, keep, n,
                     out);
}

void launch_compact_kept(const int64_t* idx, const uint8_t* keep, const int64_t* off, int64_t n,
                         int64_t* kept, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(compact_kept_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, idx,
                     keep, off, n, kept);
}

void launch_partition_digest_idx(const uint64_t* hash, const int64_t* kept, PartRange* parts,
                                 int64_t nparts, hipStream_t s) {
  if (nparts <= 0) return;
  hipLaunchKernelGGL(partition_digest_idx_kernel, dim3((unsigned)nparts, 64), dim3(256), 0, s, hash,
                     kept, parts, nparts);
}

void launch_gather_i64(const int64_t* src, const int64_t* pos, int64_t n, int64_t* dst,
                       hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(gather_i64_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, pos,
                     n, dst);
}

DQ_CHK_UNIT(kernels)

}  // namespace dq
