// dq_inflate.hip -- Kernel 2: BGZF block inflate (+ CRC32) on gfx950.
//
// Replaces htsjdk BlockCompressedInputStream / BlockGunzipper.unzipBlock (htsjdk 2.16.0, reached
// from D/impl/formats/bam/BamSource.java:172-175) -> java.util.zip.Inflater.
//
// One 64-lane wave per BGZF block (BGZF blocks are independent DEFLATE streams).  Per batch:
//   1. the wave tops up an LDS ring with the block's compressed words (coalesced HBM reads);
//   2. lane 0 Huffman-decodes up to 64 symbols (<= ~1 KiB of output) with zlib-format decode
//      tables held in LDS (9-bit litlen / 6-bit distance roots + sub-tables), writing literal /
//      (length, distance) symbols to LDS;
//   3. all lanes place the batch: a wave prefix-sum gives each symbol's output offset, literals
//      land in an LDS staging buffer in parallel, matches whose source lies before the batch are
//      gathered from the block's own output in HBM in parallel (byte-flattened over lanes),
//      matches whose source reaches into the batch are copied in order from LDS;
//   4. the staged bytes are stored to HBM with one store per 64 bytes.
// Output stops at ISIZE (Inflater.inflate(buf, off, ISIZE) semantics); fewer bytes is an error.
#include "dq_internal.h"

namespace dq {
namespace {

constexpr int LROOT = 9;
constexpr int DROOT = 6;
constexpr int ENOUGH_L = 852;  // zlib ENOUGH_LENS for a 9-bit root, max length 15
constexpr int ENOUGH_D = 592;  // zlib ENOUGH_DISTS for a 6-bit root
constexpr int RING_WORDS = 512;
constexpr int BATCH = 64;
constexpr int BATCH_BYTES = 1024;
constexpr int OBUF = 2048;

enum { T_CODES = 0, T_LENS = 1, T_DISTS = 2 };
enum { M_HEADER = 0, M_STORED = 1, M_CODES = 2, M_DONE = 3 };

__constant__ uint16_t c_lbase[31] = {3,  4,  5,  6,  7,  8,  9,  10,  11,  13,  15,  17,  19,  23, 27, 31,
                                     35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258, 0,  0};
__constant__ uint8_t c_lext[31] = {16, 16, 16, 16, 16, 16, 16, 16, 17, 17, 17, 17, 18, 18, 18, 18,
                                   19, 19, 19, 19, 20, 20, 20, 20, 21, 21, 21, 21, 16, 64, 64};
__constant__ uint16_t c_dbase[32] = {1,    2,    3,    4,    5,    7,     9,     13,    17,  25,   33,
                                     49,   65,   97,   129,  193,  257,   385,   513,   769, 1025, 1537,
                                     2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577, 0,   0};
__constant__ uint8_t c_dext[32] = {16, 16, 16, 16, 17, 17, 18, 18, 19, 19, 20, 20, 21, 21, 22, 22,
                                   23, 23, 24, 24, 25, 25, 26, 26, 27, 27, 28, 28, 29, 29, 64, 64};
__constant__ uint8_t c_clorder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

struct alignas(16) Lds {
  uint32_t lcode[ENOUGH_L];   // litlen table; code-length table while reading a dynamic header
  uint32_t dcode[ENOUGH_D];
  uint32_t ring[RING_WORDS];  // compressed words of the block
  uint32_t sym[BATCH];        // decoded symbols of the batch
  uint32_t fpre[BATCH + 1];   // prefix of far-match lengths
  int32_t dsts[BATCH];        // output offset of each symbol inside the batch
  uint16_t lens[320];
  uint16_t work[320];
  uint16_t count[16];
  uint16_t offs[16];
  uint8_t obuf[OBUF];
  int32_t misc[8];
};

__device__ inline uint32_t mk(uint32_t op, uint32_t bits, uint32_t val) {
  return op | (bits << 8) | (val << 16);
}

// Canonical Huffman decode table construction, zlib inflate_table format: entry = op | bits<<8 |
// val<<16; op 0 literal, 16+e base with e extra bits, 32+64 end-of-block, 64 invalid, 1..15
// sub-table link (op = index bits, val = offset).  Run by one lane.  Returns 0 or -1.
__device__ int build_table(Lds& L, int type, const uint16_t* lens, int n, uint32_t* table,
                           int root_in, int enough, uint32_t* mask_out) {
  uint16_t* count = L.count;
  uint16_t* offs = L.offs;
  uint16_t* work = L.work;
  for (int i = 0; i < 16; i++) count[i] = 0;
  for (int s = 0; s < n; s++) count[lens[s]]++;
  int root = root_in;
  int max;
  for (max = 15; max >= 1; max--)
    if (count[max] != 0) break;
  if (root > max) root = max;
  if (max == 0) {  // no codes: table of invalid entries, decoding any symbol fails
    uint32_t inv = mk(64, 1, 0);
    table[0] = inv;
    table[1] = inv;
    *mask_out = 1;
    return 0;
  }
  int min;
  for (min = 1; min < max; min++)
    if (count[min] != 0) break;
  if (root < min) root = min;
  int left = 1;
  for (int len = 1; len <= 15; len++) {
    left <<= 1;
    left -= count[len];
    if (left < 0) return -1;  // over-subscribed
  }
  if (left > 0 && (type == T_CODES || max != 1)) return -1;  // incomplete
  *mask_out = (1u << root) - 1;  // zlib returns the (possibly reduced) root in *bits
  offs[1] = 0;
  for (int len = 1; len < 15; len++) offs[len + 1] = offs[len] + count[len];
  for (int s = 0; s < n; s++)
    if (lens[s] != 0) work[offs[lens[s]]++] = (uint16_t)s;
  int match;
  if (type == T_CODES) match = 20;
  else if (type == T_LENS) match = 257;
  else match = 0;
  uint32_t huff = 0;
  int sym = 0, len = min, drop = 0, curr = root;
  uint32_t* next = table;
  int low = -1;
  int used = 1 << root;
  uint32_t mask = (uint32_t)used - 1;
  if ((type == T_LENS && used > ENOUGH_L) || (type == T_DISTS && used > ENOUGH_D)) return -1;
  for (;;) {
    uint32_t here;
    int w = work[sym];
    uint32_t hb = (uint32_t)(len - drop);
    if (w + 1 < match) {
      here = mk(0, hb, (uint32_t)w);
    } else if (w >= match) {
      int k = w - match;
      if (type == T_LENS) here = mk(c_lext[k], hb, c_lbase[k]);
      else here = mk(c_dext[k], hb, c_dbase[k]);
    } else {
      here = mk(32 + 64, hb, 0);  // end of block
    }
    uint32_t incr = 1u << (len - drop);
    uint32_t fill = 1u << curr;
    int minfill = (int)fill;
    do {
      fill -= incr;
      next[(huff >> drop) + fill] = here;
    } while (fill != 0);
    incr = 1u << (len - 1);
    while (huff & incr) incr >>= 1;
    if (incr != 0) {
      huff &= incr - 1;
      huff += incr;
    } else {
      huff = 0;
    }
    sym++;
    if (--count[len] == 0) {
      if (len == max) break;
      len = lens[work[sym]];
    }
    if (len > root && (int)(huff & mask) != low) {
      if (drop == 0) drop = root;
      next += minfill;
      curr = len - drop;
      left = 1 << curr;
      while (curr + drop < max) {
        left -= count[curr + drop];
        if (left <= 0) break;
        curr++;
        left <<= 1;
      }
      used += 1 << curr;
      if ((type == T_LENS && used > ENOUGH_L) || (type == T_DISTS && used > ENOUGH_D)) return -1;
      low = (int)(huff & mask);
      table[low] = mk((uint32_t)curr, (uint32_t)root, (uint32_t)(next - table));
    }
  }
  if (huff != 0) next[huff] = mk(64, (uint32_t)(len - drop), 0);
  return 0;
}

// Lane-0 decoder state (lives in lane 0's registers across batches).
struct Dec {
  uint64_t bb;       // bit buffer
  uint32_t bc;       // bits in bb
  uint32_t inw;      // next ring word (absolute word index into the deflate data)
  int32_t mode;
  int32_t last;
  int32_t stored_left;
  int32_t err;
  uint32_t lmask;    // litlen root mask
  uint32_t dmask;    // distance root mask
};

__device__ inline void refill(Dec& d, const Lds& L) {
  if (d.bc < 32) {
    d.bb |= (uint64_t)L.ring[d.inw & (RING_WORDS - 1)] << d.bc;
    d.inw++;
    d.bc += 32;
  }
}
__device__ inline uint32_t take(Dec& d, uint32_t n) {
  uint32_t v = (uint32_t)(d.bb & ((1ull << n) - 1));
  d.bb >>= n;
  d.bc -= n;
  return v;
}

// Decode a table entry for the litlen/dist/code-length alphabets, following sub-table links.
__device__ inline uint32_t lookup(Dec& d, const uint32_t* table, uint32_t rootmask) {
  uint32_t here = table[d.bb & rootmask];
  uint32_t op = here & 0xff;
  if (op != 0 && (op & 0xf0) == 0) {  // sub-table link
    uint32_t bits = (here >> 8) & 0xff;
    uint32_t idx = (here >> 16) + (uint32_t)((d.bb >> bits) & ((1u << op) - 1));
    d.bb >>= bits;
    d.bc -= bits;
    here = table[idx];
  }
  uint32_t b = (here >> 8) & 0xff;
  d.bb >>= b;
  d.bc -= b;
  return here;
}

// Read a dynamic block header and build both tables. Returns 0 or an ST_ code.
__device__ int dynamic_header(Dec& d, Lds& L) {
  refill(d, L);
  uint32_t nlen = take(d, 5) + 257, ndist = take(d, 5) + 1, ncode = take(d, 4) + 4;
  if (nlen > 286 || ndist > 30) return ST_BAD_TABLE;
  for (int i = 0; i < 19; i++) L.lens[i] = 0;
  for (uint32_t i = 0; i < ncode; i++) {
    refill(d, L);
    L.lens[c_clorder[i]] = (uint16_t)take(d, 3);
  }
  uint32_t cmask;
  if (build_table(L, T_CODES, L.lens, 19, L.lcode, 7, ENOUGH_L, &cmask) != 0) return ST_BAD_TABLE;
  uint32_t have = 0, total = nlen + ndist;
  while (have < total) {
    refill(d, L);
    uint32_t here = lookup(d, L.lcode, cmask);
    uint32_t op = here & 0xff, val = here >> 16;
    if (op == 64) return ST_BAD_TABLE;
    if (val < 16) {
      L.lens[have++] = (uint16_t)val;
    } else {
      uint32_t rep, v = 0;
      if (val == 16) {
        if (have == 0) return ST_BAD_TABLE;
        v = L.lens[have - 1];
        rep = 3 + take(d, 2);
      } else if (val == 17) {
        rep = 3 + take(d, 3);
      } else {
        rep = 11 + take(d, 7);
      }
      if (have + rep > total) return ST_BAD_TABLE;
      while (rep--) L.lens[have++] = (uint16_t)v;
    }
  }
  if (L.lens[256] == 0) return ST_BAD_TABLE;
  if (build_table(L, T_LENS, L.lens, (int)nlen, L.lcode, LROOT, ENOUGH_L, &d.lmask) != 0)
    return ST_BAD_TABLE;
  if (build_table(L, T_DISTS, L.lens + nlen, (int)ndist, L.dcode, DROOT, ENOUGH_D, &d.dmask) != 0)
    return ST_BAD_TABLE;
  return 0;
}

__device__ int fixed_tables(Dec& d, Lds& L) {
  for (int s = 0; s < 144; s++) L.lens[s] = 8;
  for (int s = 144; s < 256; s++) L.lens[s] = 9;
  for (int s = 256; s < 280; s++) L.lens[s] = 7;
  for (int s = 280; s < 288; s++) L.lens[s] = 8;
  if (build_table(L, T_LENS, L.lens, 288, L.lcode, LROOT, ENOUGH_L, &d.lmask) != 0)
    return ST_BAD_TABLE;
  for (int s = 0; s < 30; s++) L.lens[s] = 5;
  if (build_table(L, T_DISTS, L.lens, 30, L.dcode, DROOT, ENOUGH_D, &d.dmask) != 0)
    return ST_BAD_TABLE;
  return 0;
}

// Lane 0: decode one batch.  Symbol encoding: literal = byte; match = 0x80000000 | len << 16 |
// dist.  out_before = bytes of this block already produced; cap = ISIZE.
__device__ void decode_batch(Dec& d, Lds& L, int32_t out_before, int32_t cap, int32_t* nsym_out,
                             int32_t* nbytes_out) {
  int nsym = 0, nb = 0;
  int headers = 0;
  while (nsym < BATCH && nb < BATCH_BYTES && d.err == 0) {
    int32_t produced = out_before + nb;
    if (produced >= cap) {
      d.mode = M_DONE;
      break;
    }
    if (d.mode == M_DONE) break;
    if (d.mode == M_HEADER) {
      if (headers) break;  // at most one header per batch (ring look-ahead bound)
      headers++;
      refill(d, L);
      d.last = (int32_t)take(d, 1);
      uint32_t type = take(d, 2);
      if (type == 0) {
        take(d, d.bc & 7);
        refill(d, L);
        uint32_t len = take(d, 16), nlen = take(d, 16);
        if ((len ^ 0xffffu) != nlen) {
          d.err = ST_BAD_STORED;
          break;
        }
        d.stored_left = (int32_t)len;
        d.mode = M_STORED;
      } else if (type == 1) {
        int e = fixed_tables(d, L);
        if (e) { d.err = e; break; }
        d.mode = M_CODES;
      } else if (type == 2) {
        int e = dynamic_header(d, L);
        if (e) { d.err = e; break; }
        d.mode = M_CODES;
      } else {
        d.err = ST_BAD_BLOCKTYPE;
        break;
      }
      continue;
    }
    if (d.mode == M_STORED) {
      if (d.stored_left == 0) {
        d.mode = d.last ? M_DONE : M_HEADER;
        continue;
      }
      refill(d, L);
      L.sym[nsym++] = take(d, 8);
      nb += 1;
      d.stored_left--;
      continue;
    }
    // M_CODES
    refill(d, L);
    uint32_t here = lookup(d, L.lcode, d.lmask);
    uint32_t op = here & 0xff;
    if (op == 0) {
      L.sym[nsym++] = here >> 16;
      nb += 1;
      continue;
    }
    if (op & 16) {
      uint32_t len = (here >> 16) + take(d, op & 15);
      refill(d, L);
      uint32_t dh = lookup(d, L.dcode, d.dmask);
      uint32_t dop = dh & 0xff;
      if (!(dop & 16)) {
        d.err = ST_BAD_CODE;
        break;
      }
      refill(d, L);
      uint32_t dist = (dh >> 16) + take(d, dop & 15);
      if ((int32_t)dist > produced) {
        d.err = ST_BAD_DIST;
        break;
      }
      int32_t room = cap - produced;
      if ((int32_t)len > room) len = (uint32_t)room;  // Inflater stops at ISIZE
      L.sym[nsym++] = 0x80000000u | (len << 16) | dist;
      nb += (int)len;
      continue;
    }
    if (op & 32) {  // end of block
      d.mode = d.last ? M_DONE : M_HEADER;
      continue;
    }
    d.err = ST_BAD_CODE;
    break;
  }
  *nsym_out = nsym;
  *nbytes_out = nb;
}

__device__ inline int wave_incl_scan(int v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

__global__ __launch_bounds__(64) void inflate_kernel(const uint8_t* __restrict__ C,
                                                     const int64_t* __restrict__ blk_pos,
                                                     const int32_t* __restrict__ blk_csize,
                                                     const int32_t* __restrict__ blk_usize,
                                                     const int64_t* __restrict__ uoff, int64_t nblk,
                                                     uint8_t* __restrict__ U,
                                                     int32_t* __restrict__ status) {
  __shared__ Lds L;
  const int lane = threadIdx.x;
  const int64_t b = blockIdx.x;
  if (b >= nblk) return;
  const int64_t pos = blk_pos[b];
  const int32_t csize = blk_csize[b];
  const int32_t isize = blk_usize[b];
  uint8_t* out = U + uoff[b];
  if (isize > 65536 || isize < 0) {
    if (lane == 0) status[b] = ST_ISIZE;
    return;
  }
  const int64_t dstart = pos + 18;              // XLEN == 6 (checked by the chain)
  const int32_t dbytes = csize - 26;            // deflate data bytes
  const int32_t dwords = (dbytes + 3) >> 2;
  const int sh = (int)(dstart & 3) * 8;
  const uint32_t* C32 = reinterpret_cast<const uint32_t*>(C) + (dstart >> 2);

  Dec d;
  d.bb = 0;
  d.bc = 0;
  d.inw = 0;
  d.mode = isize == 0 ? M_HEADER : M_HEADER;
  d.last = 0;
  d.stored_left = 0;
  d.err = 0;
  d.lmask = 0;
  d.dmask = 0;
  int32_t loaded = 0;      // words loaded into the ring (uniform)
  int32_t produced = 0;    // bytes of output stored (uniform)
  int32_t st = ST_OK;

  int32_t guard = 0;
  for (;;) {
    if (++guard > 140000) {  // every batch makes progress; a block needs < 70000 batches
      st = ST_HANG;
      if (lane == 0)
        printf("[dq inflate] block %lld stuck: mode %d inw %u bc %u produced %d isize %d\n",
               (long long)b, d.mode, d.inw, d.bc, produced, isize);
      break;
    }
    // 1. top up the ring up to RING_WORDS words ahead of lane 0's read position
    uint32_t inw = __builtin_amdgcn_readfirstlane(d.inw);
    int32_t target = min((int32_t)inw + RING_WORDS, dwords + 2);
    while (loaded < target) {
      int32_t w = loaded + lane;
      if (w < target) {
        uint32_t v = 0;
        if (w < dwords) {
          uint64_t pair = (uint64_t)C32[w] | ((uint64_t)C32[w + 1] << 32);
          v = (uint32_t)(pair >> sh);
          int32_t valid = dbytes - 4 * w;  // bytes of this word inside the data
          if (valid < 4) v &= (1u << (8 * valid)) - 1;
        }
        L.ring[w & (RING_WORDS - 1)] = v;
      }
      loaded += 64;
      if (loaded > target) loaded = target;
    }
    __syncthreads();
    // 2. lane 0 decodes a batch
    if (lane == 0) {
      int32_t ns, nb;
      decode_batch(d, L, produced, isize, &ns, &nb);
      if (d.err == 0 && d.inw > (uint32_t)dwords + 2) d.err = ST_OVERREAD;
      L.misc[0] = ns;
      L.misc[1] = nb;
      L.misc[2] = d.err;
      L.misc[3] = d.mode == M_DONE ? 1 : 0;
    }
    __syncthreads();
    const int32_t nsym = L.misc[0];
    const int32_t nbytes = L.misc[1];
    const int32_t err = L.misc[2];
    const int32_t done = L.misc[3];
    if (err) {
      st = err;
      break;
    }
    // 3. place the batch
    uint32_t sy = lane < nsym ? L.sym[lane] : 0;
    bool is_match = lane < nsym && (sy & 0x80000000u);
    int len = lane < nsym ? (is_match ? (int)((sy >> 16) & 0x1ff) : 1) : 0;
    int dist = is_match ? (int)(sy & 0xffff) : 0;
    int incl = wave_incl_scan(len, lane);
    int dst = incl - len;  // offset inside the batch
    if (lane < nsym && !is_match) L.obuf[dst] = (uint8_t)sy;
    // far matches: source entirely before the batch (already in HBM)
    bool far = is_match && (dst - dist + len <= 0);
    bool near = is_match && !far;
    int flen = far ? len : 0;
    int fincl = wave_incl_scan(flen, lane);
    L.fpre[lane + 1] = fincl;
    L.dsts[lane] = dst;
    if (lane == 0) L.fpre[0] = 0;
    __syncthreads();
    const int32_t ftotal = L.fpre[64];
    for (int32_t base = 0; base < ftotal; base += 64) {
      int32_t fb = base + lane;
      if (fb < ftotal) {
        // owner symbol: largest k with fpre[k] <= fb (binary search over 64 entries)
        int lo = 0, hi = 63;
        while (lo < hi) {
          int mid = (lo + hi + 1) >> 1;
          if ((int32_t)L.fpre[mid] <= fb) lo = mid;
          else hi = mid - 1;
        }
        int d2 = (int)(L.sym[lo] & 0xffff);
        int j = fb - (int32_t)L.fpre[lo];
        int dd = L.dsts[lo];
        int src = dd - d2 + j;  // < 0: before the batch, already in HBM
        L.obuf[dd + j] = out[produced + src];
      }
    }
    // near matches in order, each copied by the whole wave from LDS / HBM
    uint64_t nearmask = __ballot(near);
    while (nearmask) {
      int k = __builtin_ctzll(nearmask);
      nearmask &= nearmask - 1;
      int kd = __shfl(dst, k, 64), kl = __shfl(len, k, 64), kdist = __shfl(dist, k, 64);
      for (int j0 = 0; j0 < kl; j0 += 64) {
        int j = j0 + lane;
        if (j < kl) {
          int src = kd - kdist + (j % kdist);
          uint8_t v = src >= 0 ? L.obuf[src] : out[produced + src];
          L.obuf[kd + j] = v;
        }
        __syncthreads();
      }
    }
    __syncthreads();
    // 4. store the batch to HBM
    for (int32_t o = lane; o < nbytes; o += 64) out[produced + o] = L.obuf[o];
    produced += nbytes;
    // later batches gather their far-match sources from these stores
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (done) break;
  }
  if (lane == 0) {
    if (st == ST_OK && produced != isize) st = ST_SHORT;
    status[b] = st;
  }
}

}  // namespace

void launch_inflate(const uint8_t* C, const int64_t* blk_pos, const int32_t* blk_csize,
                    const int32_t* blk_usize, const int64_t* uoff, int64_t nblk, uint8_t* U,
                    int32_t* status, hipStream_t s) {
  if (nblk <= 0) return;
  hipLaunchKernelGGL(inflate_kernel, dim3((unsigned)nblk), dim3(64), 0, s, C, blk_pos, blk_csize,
                     blk_usize, uoff, nblk, U, status);
}

}  // namespace dq
