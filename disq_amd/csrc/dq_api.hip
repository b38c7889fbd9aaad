// dq_api.hip -- C ABI (include/disq_gpu.h) and host orchestration of the device pipeline.
//
// Host side of the drop-in boundary: the split arithmetic of PathSplitSource.getPathSplits
// (D/impl/file/PathSplitSource.java:26-64), header parsing (H/BAMFileReader2.java:747-821), the
// .bai facts read by AbstractBinarySamSource (AbstractBinarySamSource.java:92-94), interval
// preparation (BoundedTraversalUtil.java:10-27) and the per-chunk record selection of
// BamSource.getIterator / createIndexIterator.  All byte/bit work runs in the HIP kernels of
// dq_kernels.hip and dq_inflate3.hip; there is no CPU fallback.
#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <sys/mman.h>
#include <mutex>
#include <vector>

#include "../../include/disq_gpu.h"
#include "dq_internal.h"

using namespace dq;

namespace {

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  template <typename T>
  T* as() const {
    return reinterpret_cast<T*>(p);
  }
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap && p) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = bytes + bytes / 8 + 256;
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
};

struct Interval {
  int32_t ref, start, end;
};

// The export arena's ownership, shared by the context and the batch exported into it (a JNI
// caller frees batches from its own threads, AutocloseIteratorWrapper.java:26-36 style): while a
// batch lives, the context may not export another batch there (DQ_EINVAL), resize it, or free it
// -- dq_ctx_destroy leaves the arena to the batch, whose dq_batch_free releases it.
struct ArenaHold {
  std::mutex mu;
  uint8_t* arena = nullptr;
  bool live = false;    // a batch's arrays are in the arena
  bool orphan = false;  // the context was destroyed first: the batch frees the arena
};

// A .bai (SAMv1 section 5.2) as htsjdk's index reads it: per reference its bins' chunks (the
// 37450 pseudo-bin left out) and its 16 kbp linear index.
struct VChunk {
  uint64_t b, e;
};
struct BaiRef {
  std::vector<uint32_t> bin;
  std::vector<std::vector<VChunk>> chunks;  // per bin, in file order
  std::vector<uint64_t> linear;
};
struct Bai {
  std::vector<BaiRef> refs;
  int64_t solb = -1, ncc = -1;
};

}  // namespace

struct dq_ctx {
  dq_opts o{};
  hipStream_t s = nullptr;
  hipEvent_t ev[8] = {};
  // DQ_EXPORT_STREAMS=2: the export's device-to-pinned copies alternate between s and this second
  // stream (a second DMA engine); created on first use
  hipStream_t sx = nullptr;
  hipEvent_t ev_x[2] = {};
  std::string err;
  // resident file (or byte-range shard of one: DESIGN.md §8)
  int64_t flen = 0;
  DevBuf C;
  bool have_file = false;
  bool shard = false;        // C holds file bytes [base, base + flen) of a file_len-byte file
  int64_t base = 0, file_len = 0;
  int64_t p0 = 0, p1 = 0;    // Disq partitions owned by the shard
  std::vector<uint8_t> hdr;  // shard: the decompressed BAM header, supplied by the caller
  bool header_only = false;  // dq_header_from_prefix: stop after the header
  // BGZF text (VCF) path: the pipeline stops after inflate; lines instead of records
  bool text_mode = false;
  bool have_text = false;
  int32_t text_drop = -1;
  int64_t t_nterm = 0, t_total = 0, t_nkept = 0;
  DevBuf t_tcount, t_toff, t_term, t_crf, t_plans, t_rng, t_idx, t_vs, t_vl, t_hash, t_keep,
      t_keep32, t_koff, t_kept;
  std::vector<TextPlan> tplans_h;
  // VCF interval traversal (VcfSource.getVariants with intervals): tabix model + intervals
  bool have_tbi = false;
  Bai tbi;
  std::vector<std::string> tbi_names;
  bool text_iv = false;
  std::vector<std::string> tiv_contig;           // distinct contigs of the intervals
  std::vector<int32_t> tiv_cid, tiv_start, tiv_end;  // per interval (contig id into tiv_contig)
  DevBuf t_ivnames, t_ivnoff, t_ivbeg, t_ivstart, t_ivend, t_ivmaxend;
  int64_t t_pruned = 0;                          // splits the index filter removed
  // BGZF deflate (write path)
  DevBuf z_in, z_stage, z_link, z_slots, z_size, z_off, z_out;
  int64_t z_len = 0;
  const uint8_t* cext = nullptr;  // dq_open_shard_device: caller-owned device bytes instead of C
  // dq_decode_chunk: the window holds one Chunk [chunk_vs, chunk_ve) (shard coordinates); its
  // records are walked from the exact start pointer, no split planning or guessing
  bool chunk_mode = false;
  uint64_t chunk_vs = 0, chunk_ve = 0;
  std::string chunk_hdr_path;       // path whose header ctx->hdr holds (dq_decode_chunk cache)
  // pinned host staging for file reads (dq_open_path, dq_decode_chunk)
  uint8_t* pin[2] = {nullptr, nullptr};
  size_t pin_cap = 0;
  hipEvent_t pin_ev[2] = {nullptr, nullptr};
  // dq_set_export_arena: batches land in this pinned arena (DMA, no staging copies); it holds one
  // batch at a time, owned by the batch until dq_batch_free (ArenaHold)
  ArenaHold* ah = nullptr;
  uint8_t* arena = nullptr;
  size_t arena_cap = 0;
  DevBuf x_bs4, x_boff, x_voff, x_parts;  // batch export: raw offsets, voffsets, digests
  int64_t h2d_bytes = 0;            // compressed bytes copied host -> device by the last open
  const uint8_t* cbuf() const { return cext ? cext : C.as<uint8_t>(); }
  // kernel 1
  DevBuf slots, counts, offs, cand, flags, voff, scal, tmp;
  DevBuf scan_over, scan_map, scan_big;  // second scan pass (dense BGZF regions)
  int64_t ncand = 0;
  // chain + inflate
  DevBuf blk_pos, blk_cs, blk_us, uoff, status, U;
  DevBuf tails;  // inflate: the tail kernel's descriptors (16 bytes per block)
  int n_cu = 256;
  int64_t nblk = 0, ulen = 0;
  // header
  int32_t n_ref = 0;
  std::vector<int32_t> ref_len;
  std::vector<std::string> ref_name;
  uint64_t first_record = 0;
  int64_t header_bytes = 0;
  DevBuf d_ref_len;
  // planning
  DevBuf plans, plan_best;  // plan_best: the record guesser's per-split minima (planning scratch)
  std::vector<SplitPlan> plans_h;
  // records
  DevBuf segs, segcnt, segbase, segoff, rec_lin, pages;
  DevBuf long_ent, long_cnt;  // long records' pieces (decode_records: hashed by many threads)
  DevBuf f_voff, f_bs, f_ref, f_pos, f_lseq, f_nref, f_npos, f_tlen, f_flag, f_bin, f_ncig, f_mapq,
      f_lrn, f_hash;
  int64_t nrec = 0;
  DevBuf parts;
  std::vector<PartRange> parts_h;
  bool have_pipeline = false;
  // host copy of the record start pointers (chunk lookups; lazily downloaded)
  std::vector<uint64_t> voff_h;
  // record export scratch (make_batch)
  DevBuf x_idx, x_rng, x_soa, x_off, x_raw;
  // .sbi splitting index (dq_set_splitting_index) and the indexer mode of dq_write_sbi
  std::vector<uint64_t> sbi;
  bool sbi_plan = false;   // plan splits from the .sbi (SBIIndex.getChunk) instead of guessing
  bool index_only = false; // dq_write_sbi: chain from the first record, no partition plans
  // index
  bool have_bai = false;
  int64_t solb = -1, ncc = -1;
  Bai bai;
  // partition plans of the open file (file coordinates) from its last full run: a sparse
  // interval run (run_span) reuses them instead of guessing again
  std::vector<SplitPlan> plan_cache;
  bool plan_cached = false;
  // sparse (.bai span) runs
  DevBuf sel, wins, span_c, span_r, span_idx, span_kept, span_keep32, span_off;
  int64_t span_extra_blocks = 4;  // blocks inflated past a window's last chunk (grows x4)
  bool span_parts_valid = false;  // parts_h holds a span run's per-partition kept counts
  // filter scratch
  DevBuf iv_ref, iv_start, iv_end, iv_begin, idx, keep;
  int64_t iota_n = -1;  // idx holds 0..iota_n-1 (dq_run_resident's interval filter)
  dq_stats stats{};

  RecSoA soa() {
    return RecSoA{f_voff.as<uint64_t>(), f_bs.as<int32_t>(),  f_ref.as<int32_t>(),
                  f_pos.as<int32_t>(),   f_lseq.as<int32_t>(), f_nref.as<int32_t>(),
                  f_npos.as<int32_t>(),  f_tlen.as<int32_t>(), f_flag.as<uint16_t>(),
                  f_bin.as<uint16_t>(),  f_ncig.as<uint16_t>(), f_mapq.as<uint8_t>(),
                  f_lrn.as<uint8_t>(),   f_hash.as<uint64_t>()};
  }
};

#define HIPCHK(x)                                                                     \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      ctx->err = std::string(#x) + ": " + hipGetErrorString(e_);                     \
      return DQ_EDEVICE;                                                              \
    }                                                                                 \
  } while (0)
// Every C-ABI entry point runs on the context's device, whatever the calling thread's current
// device is (one dq_ctx per Spark task thread).
#define ON_DEVICE(ctx)                                                               \
  do {                                                                               \
    if (hipSetDevice((ctx)->o.device) != hipSuccess) {                               \
      (ctx)->err = "hipSetDevice failed";                                            \
      return DQ_EDEVICE;                                                             \
    }                                                                                \
  } while (0)
#define RET(code, msg)   \
  do {                   \
    ctx->err = (msg);    \
    return (code);       \
  } while (0)

namespace {

inline int32_t rd32(const uint8_t* p) {
  return (int32_t)((uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
                   ((uint32_t)p[3] << 24));
}
inline uint64_t rd64(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; i--) v = (v << 8) | p[i];
  return v;
}

// PathSplitSource.getPathSplits (D/impl/file/PathSplitSource.java:26-64) for one file:
// NIO ceil(len/splitSize) splits (:32-42) or Hadoop 2.7 FileInputFormat.getSplits (:44-62).
int path_splits(const dq_opts& o, int64_t len, std::vector<std::pair<int64_t, int64_t>>& out) {
  out.clear();
  if (o.use_nio) {
    if (o.split_size <= 0) return DQ_EINVAL;
    int64_t ss = o.split_size;
    int64_t ns = (len + ss - 1) / ss;
    for (int64_t i = 0; i < ns; i++) out.push_back({i * ss, std::min(len, i * ss + ss)});
    return 0;
  }
  int64_t block = o.hadoop_block_size > 0 ? o.hadoop_block_size : 32ll * 1024 * 1024;
  int64_t maxs = o.split_size > 0 ? o.split_size : INT64_MAX;
  int64_t ss = std::max<int64_t>(1, std::min(maxs, block));
  if (len == 0) {
    out.push_back({0, 0});
    return 0;
  }
  int64_t rem = len;
  while ((double)rem / (double)ss > 1.1) {
    out.push_back({len - rem, len - rem + ss});
    rem -= ss;
  }
  if (rem != 0) out.push_back({len - rem, len});
  return 0;
}

int get_i64(dq_ctx* ctx, const void* dptr, int64_t* v) {
  HIPCHK(hipMemcpyAsync(v, dptr, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->s));
  HIPCHK(hipStreamSynchronize(ctx->s));
  return 0;
}

int ensure_all(dq_ctx* ctx, DevBuf& b, size_t bytes) {
  HIPCHK(b.ensure(bytes));
  return 0;
}

// Scratch of launch_exclusive_scan_* over n elements (>= 2 ceil(n / 1024) + 64 entries, plus the
// recursion): every scan sizes it for its own n.
int ensure_scan(dq_ctx* ctx, int64_t n) {
  return ensure_all(ctx, ctx->tmp, sizeof(int64_t) * (size_t)(4 * (n / 1024 + 1) + 4096));
}

// Kernel 3's decode of ctx->rec_lin[0, nrec) into the SoA (+ the page table and the long-record
// piece list it needs as scratch).
int decode_records(dq_ctx* ctx, int64_t nrec, int64_t nblk, int32_t* d_stat, hipStream_t s) {
  int rc;
  const int64_t ulen = ctx->ulen;
  const int64_t lcap = long_list_cap(ulen, nrec);
  if ((rc = ensure_all(ctx, ctx->pages, 4 * (size_t)((ulen >> 16) + 1))) ||
      (rc = ensure_all(ctx, ctx->long_ent, 8 * (size_t)lcap)) ||
      (rc = ensure_all(ctx, ctx->long_cnt, 8)))
    return rc;
  HIPCHK(hipMemsetAsync(d_stat, 0, 4, s));
  launch_decode_records(ctx->U.as<uint8_t>(), ulen, ctx->rec_lin.as<int64_t>(), nrec,
                        ctx->blk_pos.as<int64_t>(), ctx->uoff.as<int64_t>(), nblk,
                        ctx->pages.as<int32_t>(), ctx->soa(), d_stat, ctx->long_ent.as<uint64_t>(),
                        lcap, ctx->long_cnt.as<unsigned long long>(), s);
  return 0;
}

const char* status_name(int32_t st) {
  switch (st) {
    case ST_BAD_HEADER: return "invalid BGZF/GZIP block header";
    case ST_BAD_BLOCKTYPE: return "invalid deflate block type";
    case ST_BAD_STORED: return "invalid stored block lengths";
    case ST_BAD_TABLE: return "invalid Huffman code lengths";
    case ST_BAD_CODE: return "invalid literal/length/distance code";
    case ST_BAD_DIST: return "invalid distance too far back";
    case ST_SHORT: return "Did not inflate expected amount";
    case ST_OVERREAD: return "deflate data overrun";
    case ST_CRC: return "CRC mismatch";
    case ST_ISIZE: return "ISIZE out of range";
    default: { static char b[32]; snprintf(b, sizeof b, "format error %d", st); return b; }
  }
}

// Parse a BAM header (BAMFileReader2.readHeader, H/BAMFileReader2.java:747-801;
// readSequenceRecord :807-821) from the first n bytes of the decompressed stream.  Returns 0,
// 1 when more bytes are needed, or a DQ_ error.
int parse_header_bytes(dq_ctx* ctx, const uint8_t* h, int64_t n) {
  int64_t p = 0;
  auto need = [&](int64_t k) { return p + k <= n; };
  if (!need(8)) return 1;
  if (memcmp(h, "BAM\1", 4) != 0) RET(DQ_EFORMAT, "Invalid BAM file header");
  int32_t l_text = rd32(&h[4]);
  if (l_text < 0) RET(DQ_EFORMAT, "Invalid BAM header text length");
  p = 8 + (int64_t)l_text;
  if (!need(4)) return 1;
  int32_t nr = rd32(&h[(size_t)p]);
  p += 4;
  if (nr < 0) RET(DQ_EFORMAT, "Invalid reference count");
  std::vector<int32_t> lens;
  std::vector<std::string> names;
  for (int32_t i = 0; i < nr; i++) {
    if (!need(4)) return 1;
    int32_t ln = rd32(&h[(size_t)p]);
    if (ln <= 1) RET(DQ_EFORMAT, "Invalid BAM file header: missing sequence name");
    if (!need(4 + (int64_t)ln + 4)) return 1;
    names.emplace_back((const char*)&h[(size_t)p + 4], (size_t)ln - 1);
    lens.push_back(rd32(&h[(size_t)(p + 4 + ln)]));
    p += 8 + ln;
  }
  ctx->n_ref = nr;
  ctx->ref_len = lens;
  ctx->ref_name = names;
  ctx->header_bytes = p;
  return 0;
}

// The header from the front of U (a shard uses the header bytes its caller supplied).
int parse_header(dq_ctx* ctx) {
  if (ctx->shard && !ctx->header_only) {
    const int rc = parse_header_bytes(ctx, ctx->hdr.data(), (int64_t)ctx->hdr.size());
    if (rc == 1) RET(DQ_EINVAL, "truncated BAM header given to dq_open_shard");
    return rc;
  }
  int64_t want = std::min<int64_t>(ctx->ulen, 1 << 20);
  std::vector<uint8_t> h;
  for (;;) {
    h.resize((size_t)want);
    HIPCHK(hipMemcpy(h.data(), ctx->U.p, (size_t)want, hipMemcpyDeviceToHost));
    const int rc = parse_header_bytes(ctx, h.data(), want);
    if (rc != 1) return rc;
    if (want >= ctx->ulen) RET(DQ_EFORMAT, "truncated BAM header");
    want = std::min<int64_t>(ctx->ulen, want * 4);
  }
}

// htsjdk AbstractBAMFileIndex.getStartOfLastLinearBin / getNoCoordinateCount (2.16.0; read at
// D/impl/formats/sam/AbstractBinarySamSource.java:93-94).
// The per-reference bin / chunk / linear-index records shared by .bai and tabix (.tbi) files
// (SAMv1 section 5.2; tabix format), from offset p.
int parse_bai_body(const uint8_t* b, int64_t len, int64_t p, int32_t nr, Bai& out);

int parse_bai(const uint8_t* b, int64_t len, Bai& out) {
  if (len < 8 || memcmp(b, "BAI\1", 4) != 0) return DQ_EFORMAT;
  const int32_t nr = rd32(b + 4);
  if (nr < 0) return DQ_EFORMAT;
  return parse_bai_body(b, len, 8, nr, out);
}

int parse_bai_body(const uint8_t* b, int64_t len, int64_t p, int32_t nr, Bai& out) {
  Bai x;
  x.refs.resize((size_t)nr);
  int64_t last = -1;
  for (int32_t i = 0; i < nr; i++) {
    BaiRef& R = x.refs[(size_t)i];
    if (p + 4 > len) return DQ_EFORMAT;
    const int32_t nbin = rd32(b + p);
    p += 4;
    for (int32_t j = 0; j < nbin; j++) {
      if (p + 8 > len) return DQ_EFORMAT;
      const uint32_t bin = (uint32_t)rd32(b + p);
      const int32_t nch = rd32(b + p + 4);
      p += 8;
      if (nch < 0 || p + 16 * (int64_t)nch > len) return DQ_EFORMAT;
      if (bin != 37450) {  // the pseudo-bin holds metadata, not chunks
        R.bin.push_back(bin);
        std::vector<VChunk> c((size_t)nch);
        for (int32_t k = 0; k < nch; k++) c[(size_t)k] = {rd64(b + p + 16 * k), rd64(b + p + 16 * k + 8)};
        R.chunks.push_back(std::move(c));
      }
      p += 16 * (int64_t)nch;
    }
    if (p + 4 > len) return DQ_EFORMAT;
    const int32_t nint = rd32(b + p);
    p += 4;
    if (nint < 0 || p + 8 * (int64_t)nint > len) return DQ_EFORMAT;
    R.linear.resize((size_t)nint);
    for (int32_t k = 0; k < nint; k++) R.linear[(size_t)k] = rd64(b + p + 8 * k);
    if (nint > 0) last = (int64_t)R.linear.back();
    p += 8 * (int64_t)nint;
  }
  // htsjdk AbstractBAMFileIndex.getStartOfLastLinearBin / getNoCoordinateCount (2.16.0; read at
  // D/impl/formats/sam/AbstractBinarySamSource.java:93-94)
  x.solb = last;
  x.ncc = p + 8 <= len ? (int64_t)rd64(b + p) : -1;
  out = std::move(x);
  return 0;
}

// Tabix index (htsjdk TabixIndex, read by VcfSource through IndexFactory.loadIndex,
// D/impl/formats/vcf/VcfSource.java:155-158): the decompressed bytes -- magic "TBI\1", n_ref,
// format, col_seq, col_beg, col_end, meta, skip, l_nm, the NUL-separated sequence names, then the
// BAI-layout per-reference records.
int parse_tbi(const uint8_t* b, int64_t len, Bai& out, std::vector<std::string>& names) {
  if (len < 36 || memcmp(b, "TBI\1", 4) != 0) return DQ_EFORMAT;
  const int32_t nr = rd32(b + 4), l_nm = rd32(b + 32);
  if (nr < 0 || l_nm < 0 || 36 + (int64_t)l_nm > len) return DQ_EFORMAT;
  names.clear();
  std::string cur;
  for (int32_t i = 0; i < l_nm; i++) {
    const char c = (char)b[36 + i];
    if (c == 0) {
      names.push_back(cur);
      cur.clear();
    } else {
      cur.push_back(c);
    }
  }
  if ((int32_t)names.size() != nr) return DQ_EFORMAT;
  return parse_bai_body(b, len, 36 + l_nm, nr, out);
}

// Chunk.optimizeChunkList (htsjdk 2.16.0): sort; drop chunks ending at or before min_off (linear
// index); coalesce chunks that overlap or share a BGZF block (Chunk.overlaps / isAdjacentTo).
void optimize_chunks(std::vector<VChunk>& c, uint64_t min_off) {
  std::sort(c.begin(), c.end(), [](const VChunk& x, const VChunk& y) {
    return x.b != y.b ? x.b < y.b : x.e < y.e;
  });
  std::vector<VChunk> out;
  for (const VChunk& k : c) {
    if (k.e <= min_off) continue;
    if (!out.empty()) {
      VChunk& l = out.back();
      const bool touch = (l.b == k.b && l.e == k.e) || l.e > k.b || (l.e >> 16) == (k.b >> 16) ||
                         (l.b >> 16) == (k.e >> 16);
      if (touch) {
        if (k.e > l.e) l.e = k.e;
        continue;
      }
    }
    out.push_back(k);
  }
  c.swap(out);
}

// BAMFileReader.getFileSpan (H/BAMFileReader2.java:1004-1019): per optimized interval
// getSpanOverlapping (bins from GenomicIndexUtil.regionToBins, their chunks, optimized against
// LinearIndex.getMinimumOffset(start)), then BAMFileSpan.merge.
std::vector<VChunk> file_span(const Bai& bai, const std::vector<Interval>& q) {
  std::vector<VChunk> all;
  for (const Interval& iv : q) {
    if (iv.ref < 0 || iv.ref >= (int32_t)bai.refs.size()) continue;
    const BaiRef& R = bai.refs[(size_t)iv.ref];
    const int32_t maxp = 0x1FFFFFFF;
    const int32_t s0 = iv.start <= 0 ? 0 : (iv.start - 1) & maxp;
    const int32_t e0 = iv.end <= 0 ? maxp : (iv.end - 1) & maxp;
    if (s0 > e0) continue;
    auto in_bins = [&](uint32_t bin) {
      if (bin == 0) return true;
      const int lvl_first[5] = {1, 9, 73, 585, 4681}, lvl_last[5] = {8, 72, 584, 4680, 37449},
                shift[5] = {26, 23, 20, 17, 14};
      for (int l = 0; l < 5; l++)
        if ((int)bin >= lvl_first[l] && (int)bin <= lvl_last[l])
          return bin >= (uint32_t)(lvl_first[l] + (s0 >> shift[l])) &&
                 bin <= (uint32_t)(lvl_first[l] + (e0 >> shift[l]));
      return false;
    };
    std::vector<VChunk> c;
    for (size_t j = 0; j < R.bin.size(); j++)
      if (in_bins(R.bin[j])) c.insert(c.end(), R.chunks[j].begin(), R.chunks[j].end());
    const size_t lb = (size_t)(s0 >> 14);
    optimize_chunks(c, lb < R.linear.size() ? R.linear[lb] : 0);
    all.insert(all.end(), c.begin(), c.end());
  }
  optimize_chunks(all, 0);
  return all;
}

// BAMFileSpan.removeContentsBefore / removeContentsAfter of one partition chunk
// (D/impl/formats/sam/AbstractBinarySamSource.java:106-107).
std::vector<VChunk> clip_span(const std::vector<VChunk>& span, uint64_t vs, uint64_t ve) {
  std::vector<VChunk> out;
  for (VChunk c : span) {
    if (c.e <= vs) continue;
    if (c.b < vs) c.b = vs;
    if (c.b >= ve) continue;
    if (c.e > ve) c.e = ve;
    out.push_back(c);
  }
  return out;
}

// QueryInterval.optimizeIntervals (htsjdk 2.16.0, BoundedTraversalUtil.java:26): sort, then
// merge overlapping or abutting intervals; end <= 0 means the end of the reference.
std::vector<Interval> optimize(std::vector<Interval> v) {
  auto E = [](int32_t e) -> int64_t { return e <= 0 ? INT32_MAX : e; };
  std::sort(v.begin(), v.end(), [&](const Interval& a, const Interval& b) {
    if (a.ref != b.ref) return a.ref < b.ref;
    if (a.start != b.start) return a.start < b.start;
    return E(a.end) < E(b.end);
  });
  std::vector<Interval> out;
  if (v.empty()) return out;
  Interval prev = v[0];
  for (size_t i = 1; i < v.size(); i++) {
    const Interval nx = v[i];
    bool same = prev.ref == nx.ref;
    int64_t pe = E(prev.end), ne = E(nx.end);
    bool ovl = same && prev.start <= ne && nx.start <= pe;
    bool abut = same && (pe + 1 == nx.start || ne + 1 == prev.start);
    if (ovl || abut) {
      if (ne > pe) prev.end = nx.end;
    } else {
      out.push_back(prev);
      prev = nx;
    }
  }
  out.push_back(prev);
  return out;
}

// DQ_DEBUG=1: synchronise and report after every pipeline stage.
bool dbg_on() {
  static const bool v = getenv("DQ_DEBUG") != nullptr;  // initialised once, thread-safely
  return v;
}
void dbg(hipStream_t s, const char* what, long long a = 0, long long b = 0) {
  if (!dbg_on()) return;
  hipError_t e = hipStreamSynchronize(s);
  fprintf(stderr, "[dq] %s %lld %lld (%s)\n", what, a, b, hipGetErrorString(e));
  fflush(stderr);
}

float ev_ms(hipEvent_t a, hipEvent_t b) {
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms;
}

}  // namespace

// ------------------------------------------------------------------ pipeline
static int run_pipeline(dq_ctx* ctx) {
  if (!ctx->have_file) RET(DQ_EINVAL, "no file open");
  if (ctx->have_pipeline) return 0;
  ctx->span_parts_valid = false;
  hipStream_t s = ctx->s;
  const int64_t L = ctx->flen;
  int rc;
  HIPCHK(hipEventRecord(ctx->ev[0], s));
  // ---- Kernel 1: candidate scan
  const int64_t nch = std::max<int64_t>(1, (L + SCAN_CHUNK - 1) / SCAN_CHUNK);
  if ((rc = ensure_all(ctx, ctx->slots, sizeof(Cand) * (size_t)nch * SCAN_CAP))) return rc;
  if ((rc = ensure_all(ctx, ctx->counts, sizeof(int32_t) * (size_t)nch))) return rc;
  if ((rc = ensure_all(ctx, ctx->offs, sizeof(int64_t) * (size_t)(nch + 1)))) return rc;
  if ((rc = ensure_all(ctx, ctx->tmp, sizeof(int64_t) * (size_t)(4 * (nch / 1024 + 1) + 4096 +
                                                                 4 * (L / 65536 / 1024 + 1)))))
    return rc;
  if ((rc = ensure_all(ctx, ctx->scal, 4096))) return rc;
  int32_t* d_overflow = ctx->scal.as<int32_t>();
  int32_t* d_broken = d_overflow + 1;
  int32_t* d_stat = d_overflow + 2;
  int64_t* d_nblk = reinterpret_cast<int64_t*>(ctx->scal.as<char>() + 64);
  HIPCHK(hipMemsetAsync(ctx->scal.p, 0, 4096, s));
  if ((rc = ensure_all(ctx, ctx->scan_over, sizeof(int32_t) * (size_t)(1 + SCAN_OVER_MAX)))) return rc;
  HIPCHK(hipMemsetAsync(ctx->scan_over.p, 0, sizeof(int32_t), s));
  launch_bgzf_scan(ctx->cbuf(), L, L, ctx->slots.as<Cand>(), 0, ctx->counts.as<int32_t>(),
                   nch, nullptr, ctx->scan_over.as<int32_t>(), s);
  if ((rc = ensure_scan(ctx, nch))) return rc;
  // the candidate count (scan of the chunk counts) and the overflow count come back together;
  // only a file with dense BGZF regions (n_over > 0) takes the second pass and a second trip
  launch_exclusive_scan_i32(ctx->counts.as<int32_t>(), ctx->offs.as<int64_t>(), nch,
                            ctx->tmp.as<int64_t>(), s);
  int64_t ncand = 0;
  int32_t n_over = 0;
  HIPCHK(hipMemcpyAsync(&n_over, ctx->scan_over.p, 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(&ncand, ctx->offs.as<int64_t>() + nch, 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (n_over > SCAN_OVER_MAX) RET(DQ_EFORMAT, "too many dense BGZF regions");
  if (n_over > 0) {  // chunks with more than SCAN_CAP magic positions: second pass
    if ((rc = ensure_all(ctx, ctx->scan_map, sizeof(int32_t) * (size_t)nch))) return rc;
    if ((rc = ensure_all(ctx, ctx->scan_big, sizeof(Cand) * (size_t)n_over * SCAN_CAP_BIG))) return rc;
    HIPCHK(hipMemsetAsync(ctx->scan_map.p, 0xff, sizeof(int32_t) * (size_t)nch, s));
    launch_bgzf_scan_listed(ctx->cbuf(), L, L, ctx->scan_big.as<Cand>(), n_over,
                            ctx->counts.as<int32_t>(), ctx->scan_over.as<int32_t>(),
                            ctx->scan_map.as<int32_t>(), s);
    int32_t bad = 0;
    HIPCHK(hipMemcpyAsync(&bad, ctx->scan_over.p, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (bad < 0) RET(DQ_EFORMAT, "more than 640 BGZF magic positions in a 16 KiB window");
    launch_exclusive_scan_i32(ctx->counts.as<int32_t>(), ctx->offs.as<int64_t>(), nch,
                              ctx->tmp.as<int64_t>(), s);
    if ((rc = get_i64(ctx, ctx->offs.as<int64_t>() + nch, &ncand))) return rc;
  }
  dbg(s, "scan", nch, n_over);
  ctx->ncand = ncand;
  const int64_t capc = std::max<int64_t>(1, ncand);
  if ((rc = ensure_all(ctx, ctx->cand, sizeof(Cand) * (size_t)capc))) return rc;
  if ((rc = ensure_all(ctx, ctx->flags, sizeof(int32_t) * (size_t)capc))) return rc;
  if ((rc = ensure_all(ctx, ctx->voff, sizeof(int64_t) * (size_t)(capc + 1)))) return rc;
  launch_gather_slots(ctx->slots.as<Cand>(), ctx->counts.as<int32_t>(), ctx->offs.as<int64_t>(), nch,
                      ctx->cand.as<Cand>(), capc, n_over > 0 ? ctx->scan_map.as<int32_t>() : nullptr,
                      ctx->scan_big.as<Cand>(), s);
  // ncand on device for the kernels that need it
  int64_t* d_ncand = d_nblk + 1;
  HIPCHK(hipMemcpyAsync(d_ncand, &ncand, sizeof(int64_t), hipMemcpyHostToDevice, s));
  launch_valid_flags(ctx->cand.as<Cand>(), d_ncand, capc, ctx->flags.as<int32_t>(), s);
  if ((rc = ensure_scan(ctx, ncand))) return rc;
  launch_exclusive_scan_i32(ctx->flags.as<int32_t>(), ctx->voff.as<int64_t>(), ncand,
                            ctx->tmp.as<int64_t>(), s);
  const int64_t capb = std::max<int64_t>(1, ncand);
  if ((rc = ensure_all(ctx, ctx->blk_pos, sizeof(int64_t) * (size_t)capb))) return rc;
  if ((rc = ensure_all(ctx, ctx->blk_cs, sizeof(int32_t) * (size_t)capb))) return rc;
  if ((rc = ensure_all(ctx, ctx->blk_us, sizeof(int32_t) * (size_t)capb))) return rc;
  // a shard's bytes end inside the file: the end of the buffer is not EOF
  const int32_t is_eof = (!ctx->shard || ctx->base + L >= ctx->file_len) ? 1 : 0;
  // blk_us zeroed past the chain: the scan below runs over all capb entries before the block count
  // is known on the host, and its total is the decompressed length
  HIPCHK(hipMemsetAsync(ctx->blk_us.p, 0, sizeof(int32_t) * (size_t)capb, s));
  if (ncand > 0)
    launch_chain2(ctx->cbuf(), L, ctx->cand.as<Cand>(), d_ncand, ncand,
                  ctx->voff.as<int64_t>(), ctx->blk_pos.as<int64_t>(), ctx->blk_cs.as<int32_t>(),
                  ctx->blk_us.as<int32_t>(), capb, d_nblk, d_broken, is_eof, s);
  // The chain must start at the file start (htsjdk reads from block 0); a shard's chain starts
  // at the guesser's first block in its first split (the first valid candidate).  The first
  // valid candidate and the chain's first block come from a device reduction: one small copy
  // brings them back with the block count and the broken flag.
  unsigned long long* d_cc = reinterpret_cast<unsigned long long*>(ctx->scal.as<char>() + 128);
  HIPCHK(hipMemsetAsync(d_cc, 0xff, 16, s));
  if (ncand > 0)
    launch_chain_check(ctx->cand.as<Cand>(), d_ncand, capc, ctx->blk_pos.as<int64_t>(), d_nblk, d_cc, s);
  // block offsets in U (exclusive scan of ISIZE) over the capb candidates' slots
  if ((rc = ensure_all(ctx, ctx->uoff, sizeof(int64_t) * (size_t)(capb + 1)))) return rc;
  if ((rc = ensure_scan(ctx, capb))) return rc;
  launch_exclusive_scan_i32(ctx->blk_us.as<int32_t>(), ctx->uoff.as<int64_t>(), capb,
                            ctx->tmp.as<int64_t>(), s);
  alignas(8) unsigned char sc[144];
  int64_t ulen = 0;
  HIPCHK(hipMemcpyAsync(sc, ctx->scal.p, sizeof sc, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(&ulen, ctx->uoff.as<int64_t>() + capb, 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  int64_t nblk = 0;
  int32_t broken = 0;
  unsigned long long minvalid = 0, p0 = 0;
  memcpy(&broken, sc + 4, 4);
  memcpy(&nblk, sc + 64, 8);
  memcpy(&minvalid, sc + 128, 8);
  memcpy(&p0, sc + 136, 8);
  int64_t chain_start = 0;
  if (ctx->shard && !ctx->chunk_mode && ncand > 0) chain_start = minvalid == ~0ull ? L : (int64_t)minvalid;
  if (!broken && ncand > 0 && (int64_t)p0 != chain_start) broken = 1;
  if (broken) {  // walk htsjdk headers from the start (false-positive or non-BC headers present)
    int64_t capw = L / 26 + 2;
    if ((rc = ensure_all(ctx, ctx->blk_pos, sizeof(int64_t) * (size_t)capw))) return rc;
    if ((rc = ensure_all(ctx, ctx->blk_cs, sizeof(int32_t) * (size_t)capw))) return rc;
    if ((rc = ensure_all(ctx, ctx->blk_us, sizeof(int32_t) * (size_t)capw))) return rc;
    launch_chain_serial(ctx->cbuf(), L, chain_start, ctx->blk_pos.as<int64_t>(),
                        ctx->blk_cs.as<int32_t>(), ctx->blk_us.as<int32_t>(), capw, d_nblk, d_stat, s);
    if ((rc = get_i64(ctx, d_nblk, &nblk))) return rc;
    if ((rc = ensure_all(ctx, ctx->uoff, sizeof(int64_t) * (size_t)(nblk + 1)))) return rc;
    if ((rc = ensure_scan(ctx, nblk))) return rc;
    launch_exclusive_scan_i32(ctx->blk_us.as<int32_t>(), ctx->uoff.as<int64_t>(), nblk,
                              ctx->tmp.as<int64_t>(), s);
    if ((rc = get_i64(ctx, ctx->uoff.as<int64_t>() + nblk, &ulen))) return rc;
  }
  dbg(s, "chain", nblk, broken);
  ctx->nblk = nblk;
  if (nblk == 0 && L > 0) RET(DQ_EFORMAT, "no BGZF blocks found");
  ctx->ulen = ulen;
  HIPCHK(hipEventRecord(ctx->ev[1], s));
  // ---- Kernel 2: inflate
  if ((rc = ensure_all(ctx, ctx->U, (size_t)ulen + 256))) return rc;
  if ((rc = ensure_all(ctx, ctx->status, sizeof(int32_t) * (size_t)(nblk + 1)))) return rc;
  HIPCHK(hipMemsetAsync(ctx->status.p, 0, sizeof(int32_t) * (size_t)(nblk + 1), s));
  HIPCHK(hipMemsetAsync(ctx->U.as<uint8_t>() + ulen, 0, 256, s));
  {
    const uint32_t* crc_init = inflate3_tables(ctx->o.device);
    if (!crc_init) RET(DQ_EDEVICE, "CRC32 table initialisation failed on this device");
    static const bool timing = getenv("DQ_TIMING") != nullptr;
    uint64_t* tim = nullptr;
    if (timing) {
      HIPCHK(hipMalloc(&tim, sizeof(uint64_t) * 48 * (size_t)std::max<int64_t>(1, nblk)));
      HIPCHK(hipMemsetAsync(tim, 0, sizeof(uint64_t) * 48 * (size_t)std::max<int64_t>(1, nblk), s));
    }
    HIPCHK(hipEventRecord(ctx->ev[5], s));
    if ((rc = ensure_all(ctx, ctx->tails, INFLATE_TAIL_BYTES * (size_t)std::max<int64_t>(1, nblk)))) return rc;
    launch_inflate3(ctx->cbuf(), ctx->blk_pos.as<int64_t>(), ctx->blk_cs.as<int32_t>(),
                    ctx->blk_us.as<int32_t>(), ctx->uoff.as<int64_t>(), nblk, ctx->U.as<uint8_t>(),
                    ctx->status.as<int32_t>(), ctx->o.verify_crc, crc_init, tim, s, nullptr, 0,
                    ctx->tails.p);
    HIPCHK(hipEventRecord(ctx->ev[6], s));
    if (timing) {
      std::vector<uint64_t> h(48 * (size_t)nblk);  // 32 words per block (TIM_W), 16 per tail
      HIPCHK(hipMemcpyAsync(h.data(), tim, 8 * h.size(), hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      (void)hipFree(tim);
      double acc[24] = {0};
      for (int64_t i = 0; i < nblk; i++)
        for (int k = 0; k < 24; k++) acc[k] += (double)h[32 * (size_t)i + k];
      static const char* nm[16] = {"header", "tables", "spec", "rounds", "scan", "emit",
                                   "resolve+store", "crc", "hdr_read_lengths", "resolve_hop_next", "redo_rounds", "tables_build",
                                   "resolve_steps_jumps", "resolve_store", "resolve_jump_tail", "res_batches"};
      fprintf(stderr, "[dq] inflate3 phase cycles per BGZF block (thread 0, s_memtime):");
      for (int k = 0; k < 16; k++)
        if (nm[k][0] != '-') fprintf(stderr, " %s=%.0f", nm[k], acc[k] / (double)std::max<int64_t>(1, nblk));
      fprintf(stderr, "\n");
      const double nb = (double)std::max<int64_t>(1, nblk);
      fprintf(stderr, "[dq] first deflate block: header=%.0f tables=%.0f spec=%.0f rounds=%.0f emit=%.0f; "
              "later ones: header=%.0f tables=%.0f spec=%.0f rounds=%.0f emit=%.0f; deflate blocks per "
              "BGZF block %.3f\n", acc[16] / nb, acc[17] / nb, acc[18] / nb, acc[19] / nb, acc[21] / nb,
              (acc[0] - acc[16]) / nb, (acc[1] - acc[17]) / nb, (acc[2] - acc[18]) / nb,
              (acc[3] - acc[19]) / nb, (acc[5] - acc[21]) / nb, acc[22] / nb);
      double rr[7] = {0};
      for (int64_t i = 0; i < nblk; i++)
        for (int k = 0; k < 7; k++) rr[k] += (double)h[32 * (size_t)i + 24 + k];
      fprintf(stderr, "[dq] rounds' re-decodes per BGZF block: lanes=%.2f merged=%.2f (mean checkpoint %.2f) "
              "unmerged: spec err/eob=%.2f spec exit=%.2f other=%.2f\n", rr[0] / nb, rr[2] / nb,
              rr[3] / std::max(1.0, rr[2]), rr[4] / nb, rr[5] / nb, rr[6] / nb);
      double ta[16] = {0};
      for (int64_t i = 0; i < nblk; i++)
        for (int k = 0; k < 16; k++) ta[k] += (double)h[32 * (size_t)nblk + 16 * (size_t)i + k];
      if (ta[3] > 0)
        fprintf(stderr, "[dq] tail kernel: %.0f tails (%.1f %% of blocks), cycles per tail (lane 0): "
                "decode=%.0f (header=%.0f tables=%.0f spec=%.0f rounds=%.0f emit=%.0f) "
                "rows=%.0f store_crc=%.0f\n", ta[3], 100.0 * ta[3] / nb, ta[0] / ta[3],
                ta[4] / ta[3], ta[5] / ta[3], ta[6] / ta[3], ta[7] / ta[3], ta[8] / ta[3],
                ta[1] / ta[3], ta[2] / ta[3]);
      if (ta[3] > 0)
        fprintf(stderr, "[dq] tail rows per tail %.1f, jump rounds per row %.2f, rows with in-row chains %.1f %%, "
                "round cycles per tail %.0f\n", ta[9] / ta[3], ta[10] / std::max(1.0, ta[9]),
                100.0 * ta[11] / std::max(1.0, ta[9]), ta[12] / ta[3]);
    }
  }
  dbg(s, "inflate", nblk, ulen);
  HIPCHK(hipEventRecord(ctx->ev[2], s));
  // the first failed block, by a device reduction: one word back instead of the status array.  A
  // shard (header supplied by the caller, U not read on the host before planning) takes the word
  // back with the planning's results; a whole file checks it before its header is read from U.
  unsigned long long* d_bad = reinterpret_cast<unsigned long long*>(ctx->scal.as<char>() + 144);
  const bool defer_bad = ctx->shard && !ctx->header_only && !ctx->text_mode;
  unsigned long long bad = ~0ull;
  HIPCHK(hipMemsetAsync(d_bad, 0xff, 8, s));
  launch_first_bad(ctx->status.as<int32_t>(), nullptr, nblk, d_bad, s);
  auto bad_block = [&]() -> int {
    int32_t st = 0;
    int64_t pos = 0;
    HIPCHK(hipMemcpy(&st, ctx->status.as<int32_t>() + bad, 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&pos, ctx->blk_pos.as<int64_t>() + bad, 8, hipMemcpyDeviceToHost));
    char msg[256];
    snprintf(msg, sizeof msg, "%s in BGZF block at %lld", status_name(st), (long long)pos);
    RET(DQ_EFORMAT, msg);
  };
  if (!defer_bad) {
    HIPCHK(hipMemcpyAsync(&bad, d_bad, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (bad != ~0ull) return bad_block();
  }
  if (ctx->text_mode) {  // BGZF text: lines are planned by text_run
    ctx->stats = dq_stats{};
    ctx->stats.ms_scan = ev_ms(ctx->ev[0], ctx->ev[1]);
    ctx->stats.ms_inflate = ev_ms(ctx->ev[5], ctx->ev[6]);
    ctx->have_pipeline = true;
    return 0;
  }
  // ---- header (n_ref, reference lengths for the guesser)
  if ((rc = parse_header(ctx))) return rc;
  if (ctx->header_only) return 0;
  if ((rc = ensure_all(ctx, ctx->d_ref_len, sizeof(int32_t) * (size_t)(ctx->n_ref + 1)))) return rc;
  if (ctx->n_ref)
    HIPCHK(hipMemcpyAsync(ctx->d_ref_len.p, ctx->ref_len.data(), sizeof(int32_t) * ctx->n_ref,
                          hipMemcpyHostToDevice, s));
  // ---- planning (a1-a5)
  std::vector<std::pair<int64_t, int64_t>> splits;
  if (ctx->chunk_mode) {
    // record starts wanted: blocks up to the chunk end's block (chain_end below)
    splits.push_back({0, (int64_t)(ctx->chunk_ve >> 16)});
  } else if (path_splits(ctx->o, ctx->shard ? ctx->file_len : L, splits)) {
    RET(DQ_EINVAL, "splitSize must be > 0 with useNio");
  }
  if (ctx->shard && !ctx->chunk_mode) {  // the shard's partitions, in shard coordinates
    if (ctx->p0 < 0 || ctx->p1 > (int64_t)splits.size() || ctx->p0 >= ctx->p1)
      RET(DQ_EINVAL, "shard partition range out of bounds");
    std::vector<std::pair<int64_t, int64_t>> mine;
    for (int64_t i = ctx->p0; i < ctx->p1; i++)
      mine.push_back({splits[(size_t)i].first - ctx->base, splits[(size_t)i].second - ctx->base});
    if (mine.front().first < 0) RET(DQ_EINVAL, "shard bytes start after its first split");
    splits.swap(mine);
  }
  const int64_t nsplit = (int64_t)splits.size();
  ctx->plans_h.assign((size_t)nsplit, SplitPlan{});
  for (int64_t i = 0; i < nsplit; i++) {
    ctx->plans_h[(size_t)i].split_start = splits[(size_t)i].first;
    ctx->plans_h[(size_t)i].split_end = splits[(size_t)i].second;
  }
  if ((rc = ensure_all(ctx, ctx->plans, sizeof(SplitPlan) * (size_t)(nsplit + 1)))) return rc;
  HIPCHK(hipMemcpyAsync(ctx->plans.p, ctx->plans_h.data(), sizeof(SplitPlan) * (size_t)nsplit,
                        hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(d_nblk, &ctx->nblk, sizeof(int64_t), hipMemcpyHostToDevice, s));
  const bool no_guess = ctx->index_only || ctx->sbi_plan || ctx->chunk_mode;
  if ((ctx->index_only || ctx->sbi_plan) && ctx->shard && !ctx->chunk_mode)
    RET(DQ_EINVAL, "splitting-index planning and indexing need the whole file");
  if (ctx->chunk_mode) {
    // one partition: the caller's Chunk; both ends are pointers (BAMFileIndexIterator limits,
    // H/BAMFileReader2.java:1082-1095), the start must be a record start
    SplitPlan& P = ctx->plans_h[0];
    P.first_blk = SPLIT_FROM_SBI;
    P.rec_lin = (int64_t)(ctx->chunk_vs & 0xffff);  // window block 0 starts at the chunk's block
    P.vstart = ctx->chunk_vs;
    P.vend = ctx->chunk_ve;
    if ((ctx->chunk_vs >> 16) != 0) RET(DQ_EINVAL, "chunk window must start at the chunk's block");
    HIPCHK(hipMemcpyAsync(ctx->plans.p, ctx->plans_h.data(), sizeof(SplitPlan), hipMemcpyHostToDevice, s));
  } else if (no_guess) {
    // No record guessing: the chain starts at the first record (BAMFileReader2
    // .findVirtualOffsetOfFirstRecord); .sbi plans are SBIIndex.getChunk (SBIIndex.java:244-277)
    for (auto& P : ctx->plans_h) {
      P.first_blk = SPLIT_FROM_SBI;
      P.rec_lin = -1;
      if (!ctx->sbi_plan || ctx->index_only || ctx->sbi.empty()) continue;
      const uint64_t last = ctx->sbi.back();
      const int64_t max_end = (int64_t)(last >> 16);
      const uint64_t vs = (uint64_t)std::min(P.split_start, max_end) << 16;
      const uint64_t ve = (uint64_t)std::min(P.split_end, max_end) << 16;
      const uint64_t a = *std::lower_bound(ctx->sbi.begin(), ctx->sbi.end(), vs);
      const uint64_t e = *std::lower_bound(ctx->sbi.begin(), ctx->sbi.end(), ve);
      P.vstart = a;
      P.vend = e;
      if (a != e) P.rec_lin = ctx->header_bytes;  // non-empty (the range is found by pointer)
    }
    HIPCHK(hipMemcpyAsync(ctx->plans.p, ctx->plans_h.data(), sizeof(SplitPlan) * (size_t)nsplit,
                          hipMemcpyHostToDevice, s));
  } else {
  launch_plan_blocks(ctx->cand.as<Cand>(), d_ncand, ctx->blk_pos.as<int64_t>(),
                     ctx->blk_us.as<int32_t>(), ctx->uoff.as<int64_t>(), d_nblk,
                     ctx->plans.as<SplitPlan>(), nsplit, s);
  if ((rc = ensure_all(ctx, ctx->plan_best, 16 * (size_t)nsplit))) return rc;
  launch_first_record(ctx->U.as<uint8_t>(), ulen, is_eof, ctx->d_ref_len.as<int32_t>(), ctx->n_ref,
                      ctx->blk_pos.as<int64_t>(), ctx->uoff.as<int64_t>(), d_nblk,
                      ctx->plans.as<SplitPlan>(), nsplit, ctx->plan_best.as<unsigned long long>(), s);
  HIPCHK(hipMemcpyAsync(ctx->plans_h.data(), ctx->plans.p, sizeof(SplitPlan) * (size_t)nsplit,
                        hipMemcpyDeviceToHost, s));
  }
  // block statistics (DEFLATE payload bytes, the shard's chain end and owned bytes) by a device
  // reduction, back with the same synchronisation (the block table itself stays in HBM)
  uint64_t bstat[4] = {0, 0, 0, 0};
  {
    uint64_t* d_bs = reinterpret_cast<uint64_t*>(ctx->scal.as<char>() + 160);
    launch_block_stats(ctx->blk_pos.as<int64_t>(), ctx->blk_cs.as<int32_t>(), ctx->uoff.as<int64_t>(),
                       nblk, ulen, splits.empty() ? 0 : splits.back().second, d_bs, s);
    HIPCHK(hipMemcpyAsync(bstat, d_bs, sizeof bstat, hipMemcpyDeviceToHost, s));
  }
  if (defer_bad) HIPCHK(hipMemcpyAsync(&bad, d_bad, 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (bad != ~0ull) return bad_block();  // before any planning status: the inflate failed first
  HIPCHK(hipEventRecord(ctx->ev[3], s));
  dbg(s, "plan", nsplit);
  int64_t start_lin = ctx->chunk_mode ? ctx->plans_h[0].rec_lin : no_guess ? ctx->header_bytes : -1;
  for (auto& P : ctx->plans_h) {
    if (P.status == 100 && ctx->shard && !is_eof)
      RET(DQ_EFORMAT, "shard halo too small: the record guesser needs bytes past the shard");
    if (P.status != 0) {
      char msg[224];
      snprintf(msg, sizeof msg, "split planning failed for split [%lld, %lld): %s (code %d)",
               (long long)P.split_start, (long long)P.split_end,
               P.status == ST_BAD_HEADER ? "the guessed BGZF block is a member header inside block "
                                           "payload that carries data"
                                         : status_name(P.status),
               P.status);
      RET(DQ_EFORMAT, msg);
    }
    if (P.rec_lin >= 0 && start_lin < 0) start_lin = P.rec_lin;
  }
  if (ctx->o.compat == DQ_COMPAT_DEDUPE && !ctx->chunk_mode) {
    // chunk ends at splitEnd << 16: the records of a block starting at the split end belong to
    // the next partition only
    for (auto& P : ctx->plans_h)
      if (P.rec_lin >= 0 && P.first_blk != SPLIT_FROM_SBI) P.vend = (uint64_t)P.split_end << 16;
    HIPCHK(hipMemcpyAsync(ctx->plans.p, ctx->plans_h.data(), sizeof(SplitPlan) * (size_t)nsplit,
                          hipMemcpyHostToDevice, s));
  }
  // ---- Kernel 3: record chain, SoA decode, hashes
  int64_t nrec = 0;
  // record-chain segment: one wave finds its first record start by the guesser, one lane walks it.
  // 64 KiB for short reads (~180 records to walk); for long records, ~16 typical records (the
  // median 10-record span the planning's guesser chained), so the speculation does not run the
  // guesser over every byte of segments that no record starts in (long reads, configs[4])
  int64_t SEG = 64 * 1024;
  {
    std::vector<int32_t> sp;
    for (auto& P : ctx->plans_h)
      if (P.rec_lin >= 0 && P.rec_span > 0) sp.push_back(P.rec_span);
    if (!sp.empty()) {
      std::nth_element(sp.begin(), sp.begin() + sp.size() / 2, sp.end());
      const int64_t want = 16 * (int64_t)sp[sp.size() / 2] / 10;
      while (SEG < want && SEG < (4 << 20)) SEG <<= 1;
    }
  }
  // record starts wanted: all of U, or (shard) those in blocks at or before the last split end
  int64_t chain_end = ulen;
  if (ctx->shard && !is_eof && nblk > 0) {
    if ((int64_t)bstat[3] >= nblk) RET(DQ_EFORMAT, "shard halo too small: no BGZF block after the last split");
    chain_end = (int64_t)bstat[1];
  }
  if (start_lin >= 0 && start_lin < chain_end) {
    const int64_t nseg = (chain_end - start_lin + SEG - 1) / SEG;
    if ((rc = ensure_all(ctx, ctx->segs, sizeof(Seg) * (size_t)(nseg + 1)))) return rc;
    if ((rc = ensure_all(ctx, ctx->segcnt, sizeof(int64_t) * (size_t)(nseg + 1)))) return rc;
    if ((rc = ensure_all(ctx, ctx->segbase, sizeof(int64_t) * (size_t)(nseg + 1)))) return rc;
    // the walk's recorded record starts (64 KiB segments): 1 KiB per segment, 1.6 % of U
    uint16_t* offs = nullptr;
    if (SEG <= 65536) {
      if ((rc = ensure_all(ctx, ctx->segoff, 2 * (size_t)SEG_OFF_CAP * (size_t)nseg))) return rc;
      offs = ctx->segoff.as<uint16_t>();
    }
    HIPCHK(hipMemsetAsync(d_broken, 0, 8, s));
    launch_seg_spec(ctx->U.as<uint8_t>(), ulen, is_eof, chain_end, ctx->d_ref_len.as<int32_t>(), ctx->n_ref,
                    ctx->segs.as<Seg>(), nseg, SEG, start_lin, offs, s);
    launch_seg_link(ctx->segs.as<Seg>(), nseg, SEG, start_lin, chain_end, d_broken, s);
    // the link check and the record count come back together; a broken link (a guesser false
    // positive) is repaired serially and the count taken again
    if ((rc = ensure_scan(ctx, nseg))) return rc;
    launch_seg_counts(ctx->segs.as<Seg>(), nseg, ctx->segcnt.as<int64_t>(), s);
    launch_exclusive_scan_i64(ctx->segcnt.as<int64_t>(), ctx->segbase.as<int64_t>(), nseg,
                              ctx->tmp.as<int64_t>(), s);
    int32_t br = 0;
    HIPCHK(hipMemcpyAsync(&br, d_broken, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(&nrec, ctx->segbase.as<int64_t>() + nseg, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (br) {
      launch_seg_fix2(ctx->U.as<uint8_t>(), ulen, is_eof, chain_end, ctx->segs.as<Seg>(), nseg, SEG, start_lin,
                      d_stat, s);
      int32_t st = 0;
      HIPCHK(hipMemcpyAsync(&st, d_stat, 4, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      if (st == 4) RET(DQ_EFORMAT, "shard halo too small: the record chain runs past the shard bytes");
      if (st) RET(DQ_EFORMAT, st == ST_BAD_CODE ? "Invalid record length" : "truncated record chain");
      launch_seg_counts(ctx->segs.as<Seg>(), nseg, ctx->segcnt.as<int64_t>(), s);
      launch_exclusive_scan_i64(ctx->segcnt.as<int64_t>(), ctx->segbase.as<int64_t>(), nseg,
                                ctx->tmp.as<int64_t>(), s);
      if ((rc = get_i64(ctx, ctx->segbase.as<int64_t>() + nseg, &nrec))) return rc;
    }
    dbg(s, "segs", nseg, br);
    const size_t nr = (size_t)std::max<int64_t>(1, nrec);
    if ((rc = ensure_all(ctx, ctx->rec_lin, 8 * nr))) return rc;
    launch_seg_emit2(ctx->U.as<uint8_t>(), ulen, ctx->segs.as<Seg>(), ctx->segbase.as<int64_t>(),
                     nseg, ctx->rec_lin.as<int64_t>(), s, offs, SEG, start_lin);
    DevBuf* b8[] = {&ctx->f_voff, &ctx->f_hash};
    DevBuf* b4[] = {&ctx->f_bs, &ctx->f_ref, &ctx->f_pos, &ctx->f_lseq, &ctx->f_nref, &ctx->f_npos,
                    &ctx->f_tlen};
    DevBuf* b2[] = {&ctx->f_flag, &ctx->f_bin, &ctx->f_ncig};
    DevBuf* b1[] = {&ctx->f_mapq, &ctx->f_lrn};
    for (auto* b : b8) if ((rc = ensure_all(ctx, *b, 8 * nr))) return rc;
    for (auto* b : b4) if ((rc = ensure_all(ctx, *b, 4 * nr))) return rc;
    for (auto* b : b2) if ((rc = ensure_all(ctx, *b, 2 * nr))) return rc;
    for (auto* b : b1) if ((rc = ensure_all(ctx, *b, nr))) return rc;
    if ((rc = decode_records(ctx, nrec, nblk, d_stat, s))) return rc;
  }
  dbg(s, "decode", nrec);
  ctx->nrec = nrec;
  // ---- partitions
  if ((rc = ensure_all(ctx, ctx->parts, sizeof(PartRange) * (size_t)(nsplit + 1)))) return rc;
  launch_partition_ranges(ctx->plans.as<SplitPlan>(), nsplit, ctx->rec_lin.as<int64_t>(),
                          ctx->f_voff.as<uint64_t>(), nrec, ctx->parts.as<PartRange>(), d_stat, s);
  launch_partition_digest2(ctx->f_hash.as<uint64_t>(), ctx->parts.as<PartRange>(), nsplit, s);
  HIPCHK(hipEventRecord(ctx->ev[4], s));
  ctx->parts_h.assign((size_t)nsplit, PartRange{});
  HIPCHK(hipMemcpyAsync(ctx->parts_h.data(), ctx->parts.p, sizeof(PartRange) * (size_t)nsplit,
                        hipMemcpyDeviceToHost, s));
  int32_t st = 0;
  HIPCHK(hipMemcpyAsync(&st, d_stat, 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (st == 101) RET(DQ_EFORMAT, "record guesser start is not on the record chain");
  if (st == 102 && ctx->chunk_mode) RET(DQ_EFORMAT, "chunk start is not a record start");
  if (st == 102) RET(DQ_EFORMAT, "splitting index offset is not a record start");
  if (st && ctx->shard && !is_eof) RET(DQ_EFORMAT, "shard halo too small: a record ends past the shard bytes");
  if (st) RET(DQ_EFORMAT, "truncated BAM record");
  // stats
  dq_stats& S = ctx->stats;
  S = dq_stats{};
  S.compressed_bytes = L;
  S.decompressed_bytes = ulen;
  S.n_blocks = nblk;
  S.n_partitions = nsplit;
  int64_t emitted = 0;
  uint64_t dg = 0;
  for (int64_t i = 0; i < nsplit; i++) {
    const PartRange& r = ctx->parts_h[(size_t)i];
    emitted += r.end - r.begin;
    dg += dq_mix64(r.digest ^ ((uint64_t)(i + 1) * DQ_K_WORD));
  }
  S.n_records = emitted;
  S.digest = dg;
  S.ms_scan = ev_ms(ctx->ev[0], ctx->ev[1]);
  S.ms_inflate = ev_ms(ctx->ev[5], ctx->ev[6]);  // the inflate kernel (CRC32 fused)
  S.ms_crc = 0;                                   // fused into the inflate kernel
  // DEFLATE payload bytes = sum over blocks of (BSIZE + 1 - 26): csize - 18 header - 8 trailer;
  // owned bytes = the decompressed bytes of the blocks that start inside the splits (the whole
  // stream for a whole file; over the shards of a file they add up to its size)
  S.deflate_bytes = (int64_t)bstat[0];
  S.owned_bytes = ctx->shard && nblk ? (int64_t)bstat[2] : ulen;
  S.ms_plan = ev_ms(ctx->ev[2], ctx->ev[3]);
  S.ms_records = ev_ms(ctx->ev[3], ctx->ev[4]);
  S.ms_total = ev_ms(ctx->ev[0], ctx->ev[4]);
  S.h2d_bytes = ctx->h2d_bytes;
  S.blocks_inflated = nblk;
  ctx->have_pipeline = true;
  if (!ctx->chunk_mode && !ctx->index_only) {
    ctx->plan_cache = ctx->plans_h;
    ctx->plan_cached = true;
  }
  ctx->voff_h.clear();
  return 0;
}

// ------------------------------------------------------------------ BGZF text (VCF) path
// TextInputFormat + LineRecordReader over Disq's splittable BGZF codec, per split (dq_text.hip
// holds the characterisation, oracle/disq_oracle.c the literal restatement): terminators of the
// resident stream, each split's line range, the values (drop '#' lines as VcfSource does), their
// hashes and per-partition digests; everything stays in HBM.
static int text_run(dq_ctx* ctx, int32_t drop_hash) {
  if (!ctx->text_mode) RET(DQ_EINVAL, "not a text context (dq_text_open_*)");
  int rc = run_pipeline(ctx);
  if (rc) return rc;
  if (ctx->have_text && ctx->text_drop == drop_hash) return 0;
  hipStream_t s = ctx->s;
  const int64_t nblk = ctx->nblk, ulen = ctx->ulen, L = ctx->flen;
  int32_t* d_stat = ctx->scal.as<int32_t>() + 2;
  int64_t* d_ncand = reinterpret_cast<int64_t*>(ctx->scal.as<char>() + 64) + 1;
  HIPCHK(hipEventRecord(ctx->ev[2], s));
  {  // an empty block inside the stream would end a split's stream there: not reproduced
    std::vector<int32_t> us((size_t)nblk);
    if (nblk) HIPCHK(hipMemcpyAsync(us.data(), ctx->blk_us.p, 4 * (size_t)nblk, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    for (int64_t b = 0; b + 1 < nblk; b++)
      if (us[(size_t)b] == 0) RET(DQ_EFORMAT, "empty BGZF block inside a text stream is not supported");
  }
  // terminators
  const int64_t nt = text_tiles(ulen);
  if ((rc = ensure_all(ctx, ctx->t_tcount, 4 * (size_t)std::max<int64_t>(1, nt)))) return rc;
  if ((rc = ensure_all(ctx, ctx->t_toff, 8 * (size_t)(nt + 1)))) return rc;
  if ((rc = ensure_all(ctx, ctx->tmp, sizeof(int64_t) * (size_t)(4 * (nt / 1024 + 1) + 4096)))) return rc;
  launch_text_terms(ctx->U.as<uint8_t>(), ulen, ctx->t_tcount.as<int32_t>(), nullptr, nullptr, false, s);
  if (nt > 0)
    launch_exclusive_scan_i32(ctx->t_tcount.as<int32_t>(), ctx->t_toff.as<int64_t>(), nt,
                              ctx->tmp.as<int64_t>(), s);
  int64_t nterm = 0;
  if (nt > 0 && (rc = get_i64(ctx, ctx->t_toff.as<int64_t>() + nt, &nterm))) return rc;
  if ((rc = ensure_all(ctx, ctx->t_term, 8 * (size_t)(nterm + 1)))) return rc;
  launch_text_terms(ctx->U.as<uint8_t>(), ulen, nullptr, ctx->t_toff.as<int64_t>(),
                    ctx->t_term.as<int64_t>(), true, s);
  ctx->t_nterm = nterm;
  if ((rc = ensure_all(ctx, ctx->t_crf, 8 * (size_t)std::max<int64_t>(1, nblk)))) return rc;
  launch_text_cr_fills(ctx->U.as<uint8_t>(), ctx->uoff.as<int64_t>(), ctx->blk_us.as<int32_t>(), nblk,
                       ctx->t_crf.as<int64_t>(), s);
  // split plans (FileInputFormat splits: the same arithmetic as the BAM path, a1)
  std::vector<std::pair<int64_t, int64_t>> splits;
  if (path_splits(ctx->o, L, splits)) RET(DQ_EINVAL, "splitSize must be > 0 with useNio");
  ctx->t_pruned = 0;
  if (ctx->text_iv) {
    // TribbleIndexIntervalFilteringTextInputFormat.getSplits (D/impl/formats/tribble/
    // TribbleIndexIntervalFilteringTextInputFormat.java:32-62): the index blocks of every interval
    // (TabixIndex.getBlocks -> the bins' chunks, optimized against the linear index), and only the
    // splits whose [start << 16, end << 16] overlaps one of them (its `overlaps`, :64-68).
    if (!ctx->have_tbi) RET(DQ_EINVAL, "Intervals set but no index file found");
    std::vector<VChunk> blocks;
    for (size_t i = 0; i < ctx->tiv_start.size(); i++) {
      const std::string& cn = ctx->tiv_contig[(size_t)ctx->tiv_cid[i]];
      const auto it = std::find(ctx->tbi_names.begin(), ctx->tbi_names.end(), cn);
      if (it == ctx->tbi_names.end()) continue;
      const int32_t tid = (int32_t)(it - ctx->tbi_names.begin());
      const std::vector<VChunk> c = file_span(ctx->tbi, {Interval{tid, ctx->tiv_start[i], ctx->tiv_end[i]}});
      blocks.insert(blocks.end(), c.begin(), c.end());
    }
    auto ov = [](uint64_t a, uint64_t b, uint64_t a2, uint64_t b2) {
      return (a2 >= a && a2 <= b) || (b2 >= a && b2 <= b) || (a >= a2 && b <= b2);
    };
    std::vector<std::pair<int64_t, int64_t>> kept;
    for (const auto& sp : splits) {
      const uint64_t vs = (uint64_t)sp.first << 16, ve = (uint64_t)sp.second << 16;
      bool any = false;
      for (const VChunk& c : blocks)
        if (ov(vs, ve, c.b, c.e)) {
          any = true;
          break;
        }
      if (any) kept.push_back(sp);
    }
    ctx->t_pruned = (int64_t)(splits.size() - kept.size());
    splits.swap(kept);
    drop_hash = 1;  // the VCF codec never sees header lines (VcfSource.java:108)
  }
  const int64_t nsplit = (int64_t)splits.size();
  ctx->tplans_h.assign((size_t)nsplit, TextPlan{});
  for (int64_t i = 0; i < nsplit; i++) {
    ctx->tplans_h[(size_t)i].split_start = splits[(size_t)i].first;
    ctx->tplans_h[(size_t)i].split_end = splits[(size_t)i].second;
  }
  if ((rc = ensure_all(ctx, ctx->t_plans, sizeof(TextPlan) * (size_t)(nsplit + 1)))) return rc;
  HIPCHK(hipMemcpyAsync(ctx->t_plans.p, ctx->tplans_h.data(), sizeof(TextPlan) * (size_t)nsplit,
                        hipMemcpyHostToDevice, s));
  launch_text_plan(ctx->cand.as<Cand>(), d_ncand, ctx->blk_pos.as<int64_t>(), ctx->blk_us.as<int32_t>(),
                   ctx->uoff.as<int64_t>(), nblk, L, ctx->U.as<uint8_t>(), ulen,
                   ctx->t_term.as<int64_t>(), nterm, ctx->t_crf.as<int64_t>(),
                   ctx->t_plans.as<TextPlan>(), nsplit, s);
  HIPCHK(hipMemcpyAsync(ctx->tplans_h.data(), ctx->t_plans.p, sizeof(TextPlan) * (size_t)nsplit,
                        hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  HIPCHK(hipEventRecord(ctx->ev[3], s));
  int32_t bom = 0;
  std::vector<int64_t> rng(2 * (size_t)nsplit + 1);  // begin[nsplit] | out_off[nsplit + 1]
  int64_t total = 0;
  for (int64_t i = 0; i < nsplit; i++) {
    const TextPlan& P = ctx->tplans_h[(size_t)i];
    if (P.status) {
      char msg[224];
      snprintf(msg, sizeof msg, "text split [%lld, %lld): %s", (long long)P.split_start,
               (long long)P.split_end,
               P.status == ST_TEXT_START
                   ? "no BGZF block starts in the split or at its end (the reference fails reading it)"
                   : "the guessed BGZF block is not on the block chain");
      RET(DQ_EFORMAT, msg);
    }
    if (P.k0 == 0 && P.bom) bom = 1;
    rng[(size_t)i] = P.k0;
    rng[(size_t)nsplit + (size_t)i] = total;
    total += P.k1 - P.k0;
  }
  rng[2 * (size_t)nsplit] = total;
  ctx->t_total = total;
  const size_t nt1 = (size_t)std::max<int64_t>(1, total);
  if ((rc = ensure_all(ctx, ctx->t_rng, 8 * rng.size()))) return rc;
  if ((rc = ensure_all(ctx, ctx->t_idx, 8 * nt1))) return rc;
  if ((rc = ensure_all(ctx, ctx->t_vs, 8 * nt1))) return rc;
  if ((rc = ensure_all(ctx, ctx->t_vl, 4 * nt1))) return rc;
  if ((rc = ensure_all(ctx, ctx->t_hash, 8 * nt1))) return rc;
  if ((rc = ensure_all(ctx, ctx->t_keep, nt1))) return rc;
  if ((rc = ensure_all(ctx, ctx->t_keep32, 4 * nt1))) return rc;
  if ((rc = ensure_all(ctx, ctx->t_koff, 8 * (nt1 + 1)))) return rc;
  if ((rc = ensure_all(ctx, ctx->t_kept, 8 * nt1))) return rc;
  if ((rc = ensure_all(ctx, ctx->tmp, sizeof(int64_t) * (size_t)(4 * ((int64_t)nt1 / 1024 + 1) + 4096))))
    return rc;
  HIPCHK(hipMemcpyAsync(ctx->t_rng.p, rng.data(), 8 * rng.size(), hipMemcpyHostToDevice, s));
  const int64_t* d_begin = ctx->t_rng.as<int64_t>();
  const int64_t* d_outoff = d_begin + nsplit;
  launch_ranges_to_idx(d_begin, d_outoff, nsplit, ctx->t_idx.as<int64_t>(), s);
  launch_text_values(ctx->U.as<uint8_t>(), ulen, ctx->t_term.as<int64_t>(), nterm,
                     ctx->t_idx.as<int64_t>(), total, bom, drop_hash, ctx->t_vs.as<int64_t>(),
                     ctx->t_vl.as<int32_t>(), ctx->t_hash.as<uint64_t>(), ctx->t_keep.as<uint8_t>(), s);
  if (ctx->text_iv)
    launch_vcf_overlap(ctx->U.as<uint8_t>(), ctx->t_vs.as<int64_t>(), ctx->t_vl.as<int32_t>(), total,
                       ctx->t_ivnames.as<uint8_t>(), ctx->t_ivnoff.as<int32_t>(),
                       (int32_t)ctx->tiv_contig.size(), ctx->t_ivbeg.as<int32_t>(),
                       ctx->t_ivstart.as<int32_t>(), ctx->t_ivmaxend.as<int32_t>(),
                       ctx->t_keep.as<uint8_t>(), s);
  launch_keep_to_i32(ctx->t_keep.as<uint8_t>(), total, ctx->t_keep32.as<int32_t>(), s);
  if ((rc = ensure_scan(ctx, total))) return rc;
  if (total > 0)
    launch_exclusive_scan_i32(ctx->t_keep32.as<int32_t>(), ctx->t_koff.as<int64_t>(), total,
                              ctx->tmp.as<int64_t>(), s);
  int64_t nkept = 0;
  if (total > 0 && (rc = get_i64(ctx, ctx->t_koff.as<int64_t>() + total, &nkept))) return rc;
  launch_compact_kept(nullptr, ctx->t_keep.as<uint8_t>(), ctx->t_koff.as<int64_t>(), total,
                      ctx->t_kept.as<int64_t>(), s);
  ctx->t_nkept = nkept;
  if ((rc = ensure_all(ctx, ctx->parts, sizeof(PartRange) * (size_t)(nsplit + 1)))) return rc;
  if (total > 0) {
    launch_text_parts(d_outoff, ctx->t_koff.as<int64_t>(), nsplit, ctx->parts.as<PartRange>(), s);
  } else {
    HIPCHK(hipMemsetAsync(ctx->parts.p, 0, sizeof(PartRange) * (size_t)nsplit, s));
  }
  launch_partition_digest_idx(ctx->t_hash.as<uint64_t>(), ctx->t_kept.as<int64_t>(),
                              ctx->parts.as<PartRange>(), nsplit, s);
  HIPCHK(hipEventRecord(ctx->ev[4], s));
  ctx->parts_h.assign((size_t)nsplit, PartRange{});
  HIPCHK(hipMemcpyAsync(ctx->parts_h.data(), ctx->parts.p, sizeof(PartRange) * (size_t)nsplit,
                        hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  (void)d_stat;
  dq_stats& S = ctx->stats;
  S.compressed_bytes = L;
  S.decompressed_bytes = ulen;
  S.n_blocks = nblk;
  S.n_partitions = nsplit;
  S.n_records = nkept;
  S.n_filtered = total - nkept;  // '#' lines dropped
  uint64_t dg = 0;
  for (int64_t i = 0; i < nsplit; i++)
    dg += dq_mix64(ctx->parts_h[(size_t)i].digest ^ ((uint64_t)(i + 1) * DQ_K_WORD));
  S.digest = dg;
  S.ms_plan = ev_ms(ctx->ev[2], ctx->ev[3]);
  S.ms_records = ev_ms(ctx->ev[3], ctx->ev[4]);
  S.ms_total = ev_ms(ctx->ev[0], ctx->ev[4]);
  S.h2d_bytes = ctx->h2d_bytes;
  S.blocks_inflated = nblk;
  {
    std::vector<int32_t> cs((size_t)nblk);
    if (nblk) HIPCHK(hipMemcpy(cs.data(), ctx->blk_cs.p, 4 * (size_t)nblk, hipMemcpyDeviceToHost));
    int64_t db = 0;
    for (int32_t c : cs) db += c - 26;
    S.deflate_bytes = db;
    S.owned_bytes = ulen;
  }
  ctx->have_text = true;
  ctx->text_drop = drop_hash;
  return 0;
}

// ------------------------------------------------------------------ BGZF deflate (write path)
// htsjdk BlockCompressedOutputStream over a byte stream in HBM: blocks of 65280 bytes compressed
// in batches of DQ_DEFLATE_BATCH blocks (default 16384, about 1 GB of input: per block 384 KB of
// staged-match space -- a dense area and an overflow pool per chunk, of which the parse fills about
// 10 KB -- and 35 KB of segment / chunk records), packed into ctx->z_out at offsets scanned on the
// device: no host round trip between batches.
static int bgzf_compress_dev(dq_ctx* ctx, const uint8_t* d_src, int64_t len, double* ms) {
  if (!deflate_tables(ctx->o.device)) RET(DQ_EDEVICE, "deflate table initialisation failed");
  hipStream_t s = ctx->s;
  const int64_t nblk = bgzf_block_count(len);
#ifdef DQ_TUNING
  static const int64_t max_batch = [] {
    const char* e = getenv("DQ_DEFLATE_BATCH");
    return e && atoll(e) > 0 ? (int64_t)atoll(e) : (int64_t)16384;
  }();
#else
  constexpr int64_t max_batch = 16384;  // blocks per launch (profiles/r4au_deflate_dense_stage.txt)
#endif
  // (the batches evenly sized: the last one no shorter than the others)
  const int64_t nbat = std::max<int64_t>(1, (nblk + max_batch - 1) / max_batch);
  const int64_t batch = std::max<int64_t>(1, (nblk + nbat - 1) / nbat);
  int rc;
  if ((rc = ensure_all(ctx, ctx->z_stage, bgzf_stage_bytes(batch)))) return rc;
  if ((rc = ensure_all(ctx, ctx->z_link, bgzf_meta_bytes(batch)))) return rc;
  if ((rc = ensure_all(ctx, ctx->z_slots, bgzf_slot_bytes(batch)))) return rc;
  if ((rc = ensure_all(ctx, ctx->z_size, 4 * (size_t)batch))) return rc;
  if ((rc = ensure_all(ctx, ctx->z_off, 8 * (size_t)batch + 8))) return rc;  // + the running total
  if ((rc = ensure_all(ctx, ctx->z_out, (size_t)std::max<int64_t>(nblk, 1) * 65536))) return rc;
  int64_t* d_total = ctx->z_off.as<int64_t>() + batch;
  HIPCHK(hipEventRecord(ctx->ev[0], s));
  HIPCHK(hipMemsetAsync(d_total, 0, 8, s));
  for (int64_t b0 = 0; b0 < nblk; b0 += batch) {
    const int64_t nb = std::min(batch, nblk - b0);
    static const bool timing = getenv("DQ_DEFLATE_TIMING") != nullptr;
    uint64_t* tim = nullptr;
    const size_t ntim = 8 * (size_t)nb * 4;  // 2 parse workgroups + 1 Huffman + 1 code per block
    if (timing) HIPCHK(hipMalloc(&tim, 8 * ntim));
    launch_bgzf_deflate(d_src, len, b0, nb, ctx->z_stage.as<uint32_t>(), ctx->z_link.as<uint32_t>(),
                        ctx->z_slots.as<uint8_t>(), ctx->z_size.as<int32_t>(), tim, s);
    HIPCHK(hipGetLastError());
    if (timing) {
      std::vector<uint64_t> h(ntim);
      HIPCHK(hipMemcpyAsync(h.data(), tim, 8 * h.size(), hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      (void)hipFree(tim);
      // parse workgroups (per chunk), then the code workgroups (per block)
      static const char* nm[3][8] = {{"", "load", "counts", "scan", "scatter", "parse", "continue", "merge+hist"},
                                     {"", "sum", "lengths", "codes+rle", "cl_code", "", "", ""},
                                     {"", "load", "count+scan", "write", "store", "", "", ""}};
      static const char* kn[3] = {"parse", "huffman", "code"};
      const int64_t cnt[3] = {2 * nb, nb, nb};
      size_t at = 0;
      for (int kk = 0; kk < 3; kk++) {
        double acc[8] = {0};
        for (int64_t i = 0; i < cnt[kk]; i++)
          for (int k = 1; k < 8; k++) {
            const uint64_t a = h[at + 8 * (size_t)i + k], z = h[at + 8 * (size_t)i + k - 1];
            if (a) acc[k] += (double)(a - z);
          }
        at += 8 * (size_t)cnt[kk];
        fprintf(stderr, "[dq] deflate %s cycles per workgroup:", kn[kk]);
        for (int k = 1; k < 8; k++)
          if (nm[kk][k][0]) fprintf(stderr, " %s=%.0f", nm[kk][k], acc[k] / (double)cnt[kk]);
        fprintf(stderr, "\n");
      }
    }
    launch_bgzf_pack(ctx->z_slots.as<uint8_t>(), ctx->z_size.as<int32_t>(), ctx->z_off.as<int64_t>(),
                     d_total, nb, ctx->z_out.as<uint8_t>(), s);
    HIPCHK(hipGetLastError());
  }
  HIPCHK(hipEventRecord(ctx->ev[1], s));
  int64_t total = 0;
  HIPCHK(hipMemcpyAsync(&total, d_total, 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  ctx->z_len = total;
  if (ms) *ms = ev_ms(ctx->ev[0], ctx->ev[1]);
  return 0;
}

// ------------------------------------------------------------------ record export
static int fetch_index(dq_ctx* ctx) {
  if ((int64_t)ctx->voff_h.size() == ctx->nrec) return 0;
  ctx->voff_h.resize((size_t)ctx->nrec);
  if (ctx->nrec)
    HIPCHK(hipMemcpy(ctx->voff_h.data(), ctx->f_voff.p, 8 * (size_t)ctx->nrec, hipMemcpyDeviceToHost));
  return 0;
}

// Two pinned staging buffers (file reads in, record batches out).
constexpr size_t PIN_PIECE = 64u << 20;
static int ensure_pinned(dq_ctx* ctx) {
  if (ctx->pin_cap >= PIN_PIECE) return 0;
  for (int k = 0; k < 2; k++) {
    if (ctx->pin[k]) (void)hipHostFree(ctx->pin[k]);
    ctx->pin[k] = nullptr;
    HIPCHK(hipHostMalloc((void**)&ctx->pin[k], PIN_PIECE, hipHostMallocDefault));
    if (!ctx->pin_ev[k]) HIPCHK(hipEventCreateWithFlags(&ctx->pin_ev[k], hipEventDisableTiming));
  }
  ctx->pin_cap = PIN_PIECE;
  return 0;
}

// Device -> pageable host copy of n bytes: pieces land in the two pinned buffers in turn while
// host threads move the previous piece out (a plain hipMemcpy into pageable memory stages through
// one runtime buffer on one thread).
// Host arrays of a batch: large ones 2 MiB-aligned with transparent huge pages requested, so the
// first touch by the staging copies faults 2 MiB pages instead of 4 KiB ones (the D2H of SoA + raw
// bytes is bound by that first touch, not by PCIe).  Freed with free() like the small ones.
static void* host_alloc(size_t n) {
  if (n < (64u << 20)) return malloc(n);
  constexpr size_t H = 2u << 20;
  const size_t r = (n + H - 1) & ~(H - 1);
  void* p = aligned_alloc(H, r);
  if (p) madvise(p, r, MADV_HUGEPAGE);
  return p;
}

static int d2h_large(dq_ctx* ctx, void* dst, const void* src, size_t n) {
  if (n < (8u << 20)) {
    HIPCHK(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, ctx->s));
    HIPCHK(hipStreamSynchronize(ctx->s));
    return 0;
  }
  int rc;
  if ((rc = ensure_pinned(ctx))) return rc;
  const size_t np = (n + PIN_PIECE - 1) / PIN_PIECE;
  auto issue = [&](size_t i) -> hipError_t {
    const size_t off = i * PIN_PIECE, len = std::min(PIN_PIECE, n - off);
    hipError_t e = hipMemcpyAsync(ctx->pin[i & 1], (const uint8_t*)src + off, len,
                                  hipMemcpyDeviceToHost, ctx->s);
    if (e == hipSuccess) e = hipEventRecord(ctx->pin_ev[i & 1], ctx->s);
    return e;
  };
  HIPCHK(issue(0));
  for (size_t i = 0; i < np; i++) {
    HIPCHK(hipEventSynchronize(ctx->pin_ev[i & 1]));
    if (i + 1 < np) HIPCHK(issue(i + 1));  // the other buffer is free: its piece was moved out
    const size_t off = i * PIN_PIECE, len = std::min(PIN_PIECE, n - off);
    constexpr int T = 8;
    std::thread th[T];
    const size_t part = (len + T - 1) / T;
    for (int t = 0; t < T; t++)
      th[t] = std::thread([&, t] {
        const size_t a = std::min(len, (size_t)t * part), b = std::min(len, a + part);
        if (b > a) memcpy((uint8_t*)dst + off + a, ctx->pin[i & 1] + a, b - a);
      });
    for (auto& x : th) x.join();
  }
  return 0;
}

// Build a batch from record-index ranges (in order; ranges may repeat records) or an explicit
// index list.  Only the selected records cross PCIe: one contiguous range is copied straight from
// the resident arrays, anything else is first gathered into compact device buffers.
static int make_batch(dq_ctx* ctx, const std::vector<std::pair<int64_t, int64_t>>& ranges_in,
                      const std::vector<int64_t>* explicit_idx, int32_t with_raw,
                      const std::vector<int64_t>& part_bounds, dq_batch** out) {
  hipStream_t s = ctx->s;
  if (with_raw < DQ_EXPORT_FIELDS || with_raw > DQ_EXPORT_LEAN) RET(DQ_EINVAL, "unknown export mode");
  // adjacent ranges (consecutive partitions) form one run of the resident arrays
  std::vector<std::pair<int64_t, int64_t>> ranges;
  for (auto& r : ranges_in) {
    if (r.second <= r.first) continue;
    if (!ranges.empty() && ranges.back().second == r.first) ranges.back().second = r.second;
    else ranges.push_back(r);
  }
  int64_t n = 0;
  if (explicit_idx) n = (int64_t)explicit_idx->size();
  else
    for (auto& r : ranges) n += r.second - r.first;
  dq_batch* b = (dq_batch*)calloc(1, sizeof(dq_batch));
  if (!b) RET(DQ_ENOMEM, "out of host memory");
  b->n_records = n;
  int rc = 0;
  auto fail = [&](int code) {
    // copies queued on the second export stream may still write into the batch's arrays (the
    // arena): let them land before the arrays are given up
    if (ctx->sx) (void)hipStreamSynchronize(ctx->sx);
    (void)hipStreamSynchronize(s);
    dq_batch_free(b);
    return code;
  };
#define XCHK(x)                                                \
  do {                                                         \
    hipError_t e_ = (x);                                       \
    if (e_ != hipSuccess) {                                    \
      ctx->err = std::string(#x) + ": " + hipGetErrorString(e_); \
      return fail(DQ_EDEVICE);                                 \
    }                                                          \
  } while (0)
  const bool direct = !explicit_idx && ranges.size() <= 1;
  int64_t first = direct && !ranges.empty() ? ranges[0].first : 0;
  RecSoA rows = ctx->soa();
  const int64_t* d_idx = nullptr;
  if (n > 0 && !direct) {
    if ((rc = ensure_all(ctx, ctx->x_idx, 8 * (size_t)n))) return fail(rc);
    if (explicit_idx) {
      XCHK(hipMemcpyAsync(ctx->x_idx.p, explicit_idx->data(), 8 * (size_t)n, hipMemcpyHostToDevice, s));
    } else {
      const int64_t nr = (int64_t)ranges.size();
      std::vector<int64_t> rg((size_t)(2 * nr + 1));
      int64_t o = 0;
      for (int64_t r = 0; r < nr; r++) {
        rg[(size_t)r] = ranges[(size_t)r].first;
        rg[(size_t)(nr + r)] = o;
        o += std::max<int64_t>(0, ranges[(size_t)r].second - ranges[(size_t)r].first);
      }
      rg[(size_t)(2 * nr)] = o;
      if ((rc = ensure_all(ctx, ctx->x_rng, 8 * rg.size()))) return fail(rc);
      XCHK(hipMemcpyAsync(ctx->x_rng.p, rg.data(), 8 * rg.size(), hipMemcpyHostToDevice, s));
      launch_ranges_to_idx(ctx->x_rng.as<int64_t>(), ctx->x_rng.as<int64_t>() + nr, nr,
                           ctx->x_idx.as<int64_t>(), s);
    }
    d_idx = ctx->x_idx.as<int64_t>();
    // compact rows: 8-byte fields, then 4-, 2- and 1-byte ones (each array 8-byte aligned)
    const size_t a8 = ((size_t)n * 8 + 7) & ~(size_t)7, a4 = ((size_t)n * 4 + 7) & ~(size_t)7,
                 a2 = ((size_t)n * 2 + 7) & ~(size_t)7, a1 = ((size_t)n + 7) & ~(size_t)7;
    if ((rc = ensure_all(ctx, ctx->x_soa, 2 * a8 + 7 * a4 + 3 * a2 + 2 * a1))) return fail(rc);
    char* q = ctx->x_soa.as<char>();
    auto take = [&](size_t bytes) {
      char* r = q;
      q += bytes;
      return r;
    };
    RecSoA dst;
    dst.voffset = (uint64_t*)take(a8);
    dst.hash = (uint64_t*)take(a8);
    dst.block_size = (int32_t*)take(a4);
    dst.ref_id = (int32_t*)take(a4);
    dst.pos = (int32_t*)take(a4);
    dst.l_seq = (int32_t*)take(a4);
    dst.next_ref_id = (int32_t*)take(a4);
    dst.next_pos = (int32_t*)take(a4);
    dst.tlen = (int32_t*)take(a4);
    dst.flag = (uint16_t*)take(a2);
    dst.bin = (uint16_t*)take(a2);
    dst.n_cigar = (uint16_t*)take(a2);
    dst.mapq = (uint8_t*)take(a1);
    dst.l_read_name = (uint8_t*)take(a1);
    launch_gather_soa(d_idx, n, ctx->soa(), dst, s);
    rows = dst;
    first = 0;
  }
  // per-record work on the device: raw offsets (an exclusive scan of 4 + block_size), voffsets in
  // file coordinates, the partitions' ordered digests; the host only receives arrays
  const int64_t np = std::max<int64_t>(0, (int64_t)part_bounds.size() - 1);
  const size_t m = (size_t)std::max<int64_t>(1, n);
  int64_t raw_len = 0;
  const uint64_t* d_voff = rows.voffset + first;
  if (n > 0) {
    if ((rc = ensure_all(ctx, ctx->x_bs4, 4 * m)) || (rc = ensure_all(ctx, ctx->x_boff, 8 * (m + 1))) ||
        (rc = ensure_scan(ctx, n)))
      return fail(rc);
    launch_bs_plus4(rows.block_size + first, n, ctx->x_bs4.as<int32_t>(), s);
    launch_exclusive_scan_i32(ctx->x_bs4.as<int32_t>(), ctx->x_boff.as<int64_t>(), n,
                              ctx->tmp.as<int64_t>(), s);
    if (ctx->base) {
      if ((rc = ensure_all(ctx, ctx->x_voff, 8 * m))) return fail(rc);
      launch_add_u64(d_voff, n, (uint64_t)ctx->base << 16, ctx->x_voff.as<uint64_t>(), s);
      d_voff = ctx->x_voff.as<uint64_t>();
    }
    XCHK(hipMemcpyAsync(&raw_len, ctx->x_boff.as<int64_t>() + n, 8, hipMemcpyDeviceToHost, s));
  }
  std::vector<PartRange> pr((size_t)np + 1);
  for (int64_t p = 0; p < np; p++) pr[(size_t)p] = {part_bounds[(size_t)p], part_bounds[(size_t)p + 1], 0};
  if (np > 0 && n > 0) {
    if ((rc = ensure_all(ctx, ctx->x_parts, sizeof(PartRange) * (size_t)(np + 1)))) return fail(rc);
    XCHK(hipMemcpyAsync(ctx->x_parts.p, pr.data(), sizeof(PartRange) * (size_t)np, hipMemcpyHostToDevice, s));
    launch_partition_digest2(rows.hash + first, ctx->x_parts.as<PartRange>(), np, s);
  }
  XCHK(hipStreamSynchronize(s));  // raw_len
  b->raw_len = raw_len;
  // host arrays: the pinned arena when it is set and large enough, else heap memory
  const size_t soa_bytes = 8 * ((8 * m + 7) / 8) * 3 + 8 * ((4 * m + 7) / 8) * 7 +
                           8 * ((2 * m + 7) / 8) * 3 + 8 * ((m + 7) / 8) * 2;
  // DQ_EXPORT_LEAN: voffsets + raw bytes only -- every other field is in each record's first 36
  // raw bytes, where htsjdk's BAMRecordCodec.decode parses it (H/BAMFileReader2.java:929-931)
  const bool lean = with_raw == DQ_EXPORT_LEAN;
  const size_t want = (lean ? 8 * ((8 * m + 7) / 8) : soa_bytes) +
                      (with_raw ? (size_t)std::max<int64_t>(1, raw_len) : 0) + 64 * 20;
  const bool in_arena = ctx->arena && want <= ctx->arena_cap;
  if (in_arena) {
    std::lock_guard<std::mutex> lk(ctx->ah->mu);
    if (ctx->ah->live) {
      ctx->err = "the export arena still holds a batch: dq_batch_free it before the next batch";
      free(b);
      return DQ_EINVAL;
    }
    ctx->ah->live = true;  // released by dq_batch_free (also on the failure paths below)
    b->arena_hold = ctx->ah;
  }
  size_t used = 0;
  auto halloc = [&](size_t bytes) -> void* {
    if (!in_arena) return host_alloc(bytes);
    void* p = ctx->arena + used;
    used += (bytes + 63) & ~(size_t)63;
    return p;
  };
  b->in_arena = in_arena ? 1 : 0;
  b->voffset = (uint64_t*)halloc(8 * m);
  if (!lean) {
    b->block_size = (int32_t*)halloc(4 * m);
    b->ref_id = (int32_t*)halloc(4 * m);
    b->pos = (int32_t*)halloc(4 * m);
    b->l_seq = (int32_t*)halloc(4 * m);
    b->next_ref_id = (int32_t*)halloc(4 * m);
    b->next_pos = (int32_t*)halloc(4 * m);
    b->tlen = (int32_t*)halloc(4 * m);
    b->flag = (uint16_t*)halloc(2 * m);
    b->bin = (uint16_t*)halloc(2 * m);
    b->n_cigar = (uint16_t*)halloc(2 * m);
    b->mapq = (uint8_t*)halloc(m);
    b->l_read_name = (uint8_t*)halloc(m);
    b->hash = (uint64_t*)halloc(8 * m);
    b->raw_offset = (int64_t*)halloc(8 * m);
    if (!b->block_size || !b->ref_id || !b->pos || !b->l_seq || !b->next_ref_id ||
        !b->next_pos || !b->tlen || !b->flag || !b->bin || !b->n_cigar || !b->mapq ||
        !b->l_read_name || !b->hash || !b->raw_offset)
      return fail(DQ_ENOMEM);
  }
  if (!b->voffset) return fail(DQ_ENOMEM);
  // pinned destination: one DMA per array (with DQ_EXPORT_STREAMS=2 the arrays, and the halves of
  // the raw bytes, alternate between two streams so two DMA engines run); heap: through the staging
  // buffers
#ifdef DQ_TUNING
  static const bool two = [] {
    const char* e = getenv("DQ_EXPORT_STREAMS");
    return e && atoi(e) == 2;
  }();
#else
  constexpr bool two = false;  // two export streams gained nothing (profiles/r4x_*): tuning only
#endif
  const bool split = in_arena && two && n > 0;
  if (split) {
    if (!ctx->sx) {
      XCHK(hipStreamCreateWithFlags(&ctx->sx, hipStreamNonBlocking));
      for (auto& e : ctx->ev_x) XCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    // everything the copies read was produced on s
    XCHK(hipEventRecord(ctx->ev_x[0], s));
    XCHK(hipStreamWaitEvent(ctx->sx, ctx->ev_x[0], 0));
  }
  int turn = 0;
  auto dma = [&](void* dst, const void* src, size_t bytes) -> int {
    hipStream_t q = split && (turn++ & 1) ? ctx->sx : s;
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, q));
    return 0;
  };
  if (n > 0) {
    auto d2h = [&](const void* src, size_t bytes, void* dst) -> int {
      if (in_arena) return dma(dst, src, bytes);
      return d2h_large(ctx, dst, src, bytes);
    };
    auto fld = [&](const void* dbase, size_t esz, void* dst) {
      return d2h((const char*)dbase + (size_t)first * esz, (size_t)n * esz, dst);
    };
    if ((rc = d2h(d_voff, 8 * (size_t)n, b->voffset))) return fail(rc);
    if (!lean &&
        ((rc = fld(rows.block_size, 4, b->block_size)) ||
         (rc = fld(rows.ref_id, 4, b->ref_id)) || (rc = fld(rows.pos, 4, b->pos)) ||
         (rc = fld(rows.l_seq, 4, b->l_seq)) || (rc = fld(rows.next_ref_id, 4, b->next_ref_id)) ||
         (rc = fld(rows.next_pos, 4, b->next_pos)) || (rc = fld(rows.tlen, 4, b->tlen)) ||
         (rc = fld(rows.flag, 2, b->flag)) || (rc = fld(rows.bin, 2, b->bin)) ||
         (rc = fld(rows.n_cigar, 2, b->n_cigar)) || (rc = fld(rows.mapq, 1, b->mapq)) ||
         (rc = fld(rows.l_read_name, 1, b->l_read_name)) || (rc = fld(rows.hash, 8, b->hash)) ||
         (rc = d2h(ctx->x_boff.p, 8 * (size_t)n, b->raw_offset))))
      return fail(rc);
  }
  if (with_raw && n > 0) {
    b->raw = (uint8_t*)halloc((size_t)std::max<int64_t>(1, raw_len));
    if (!b->raw) return fail(DQ_ENOMEM);
    // the raw bytes: in halves over the two streams when split
    auto raw_d2h = [&](const uint8_t* src) -> int {
      const size_t len = (size_t)raw_len;
      if (!in_arena) return d2h_large(ctx, b->raw, src, len);
      if (!split || len < (8u << 20)) return dma(b->raw, src, len);
      const size_t h = (len / 2 + 63) & ~(size_t)63;
      int r = dma(b->raw, src, h);
      return r ? r : dma(b->raw + h, src + h, len - h);
    };
    if (direct) {  // consecutive chain records are contiguous in U
      int64_t lo = 0;
      XCHK(hipMemcpy(&lo, ctx->rec_lin.as<int64_t>() + first, 8, hipMemcpyDeviceToHost));
      if ((rc = raw_d2h(ctx->U.as<uint8_t>() + lo))) return fail(rc);
    } else {
      if ((rc = ensure_all(ctx, ctx->x_raw, (size_t)raw_len))) return fail(rc);
      launch_gather_raw(ctx->U.as<uint8_t>(), ctx->rec_lin.as<int64_t>(), ctx->f_bs.as<int32_t>(),
                        d_idx, 0, n, ctx->x_boff.as<int64_t>(), ctx->x_raw.as<uint8_t>(), s);
      if (split) {  // the second stream waits for the gather too
        XCHK(hipEventRecord(ctx->ev_x[0], s));
        XCHK(hipStreamWaitEvent(ctx->sx, ctx->ev_x[0], 0));
      }
      if ((rc = raw_d2h(ctx->x_raw.as<uint8_t>()))) return fail(rc);
    }
  }
  if (split) {  // s completes after the second stream's copies
    XCHK(hipEventRecord(ctx->ev_x[1], ctx->sx));
    XCHK(hipStreamWaitEvent(s, ctx->ev_x[1], 0));
  }
  b->n_partitions = np;
  b->part_offset = (int64_t*)malloc(sizeof(int64_t) * (size_t)(np + 1));
  b->part_digest = (uint64_t*)calloc((size_t)np + 1, sizeof(uint64_t));
  if (!b->part_offset || !b->part_digest) return fail(DQ_ENOMEM);
  for (int64_t p = 0; p <= np; p++) b->part_offset[p] = part_bounds[(size_t)p];
  if (np > 0 && n > 0) {
    XCHK(hipMemcpyAsync(pr.data(), ctx->x_parts.p, sizeof(PartRange) * (size_t)np, hipMemcpyDeviceToHost, s));
  }
  XCHK(hipStreamSynchronize(s));
  for (int64_t p = 0; p < np; p++) b->part_digest[p] = n > 0 ? pr[(size_t)p].digest : 0;
#undef XCHK
  *out = b;
  return 0;
}

// Records of one chunk: from the record at vstart while the start pointer < vend.
static int chunk_range(dq_ctx* ctx, uint64_t vstart, uint64_t vend, int64_t* b, int64_t* e) {
  int rc;
  if ((rc = fetch_index(ctx))) return rc;
  const uint64_t vb = (uint64_t)ctx->base << 16;  // file coordinates -> shard coordinates
  vstart = vstart >= vb ? vstart - vb : 0;
  vend = vend >= vb ? vend - vb : 0;
  auto& v = ctx->voff_h;
  auto it = std::lower_bound(v.begin(), v.end(), vstart);
  if (it == v.end() || *it != vstart) {
    // a start pointer past the last record reads nothing (EOF)
    if (it == v.end()) {
      *b = *e = ctx->nrec;
      return 0;
    }
    RET(DQ_EFORMAT, "chunk start is not a record start");
  }
  *b = it - v.begin();
  *e = std::lower_bound(v.begin(), v.end(), vend) - v.begin();
  if (*e < *b) *e = *b;
  return 0;
}

// QueryInterval.optimizeIntervals of the traversal, uploaded per contig (interval_filter_kernel's
// layout: sorted intervals + a per-contig begin table).
static int upload_intervals(dq_ctx* ctx, const dq_traversal* tr) {
  int rc;
  std::vector<Interval> iv;
  for (int64_t i = 0; i < tr->n; i++) {
    if (tr->ref[i] < 0 || tr->ref[i] >= ctx->n_ref) RET(DQ_EINVAL, "Invalid reference index");
    iv.push_back({tr->ref[i], tr->start[i], tr->end[i]});
  }
  iv = optimize(iv);
  std::vector<int32_t> r, st, en, beg((size_t)ctx->n_ref + 1, 0);
  for (auto& x : iv) {
    r.push_back(x.ref);
    st.push_back(x.start);
    en.push_back(x.end);
  }
  for (auto& x : iv) beg[(size_t)x.ref + 1]++;
  for (int32_t k = 0; k < ctx->n_ref; k++) beg[(size_t)k + 1] += beg[(size_t)k];
  const size_t ni = iv.size();
  if ((rc = ensure_all(ctx, ctx->iv_ref, 4 * ni + 4)) || (rc = ensure_all(ctx, ctx->iv_start, 4 * ni + 4)) ||
      (rc = ensure_all(ctx, ctx->iv_end, 4 * ni + 4)) ||
      (rc = ensure_all(ctx, ctx->iv_begin, 4 * beg.size() + 4)))
    return rc;
  HIPCHK(hipMemcpy(ctx->iv_ref.p, r.data(), 4 * ni, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(ctx->iv_start.p, st.data(), 4 * ni, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(ctx->iv_end.p, en.data(), 4 * ni, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(ctx->iv_begin.p, beg.data(), 4 * beg.size(), hipMemcpyHostToDevice));
  return 0;
}

// createIndexIterator (contained=false) over [b, e) + the unplaced-unmapped tail
// (AbstractBinarySamSource.java:86-134).
static int filtered_indices(dq_ctx* ctx, uint64_t vstart, uint64_t vend, int64_t b, int64_t e,
                            const dq_traversal* tr, std::vector<int64_t>& out) {
  int rc;
  out.clear();
  if (!ctx->have_bai) RET(DQ_EINVAL, "Intervals set but no index file found");
  if (tr->has_intervals && tr->n > 0 && e > b) {
    if ((rc = upload_intervals(ctx, tr))) return rc;
    const int64_t n = e - b;
    std::vector<int64_t> idx((size_t)n);
    for (int64_t k = 0; k < n; k++) idx[(size_t)k] = b + k;
    if ((rc = ensure_all(ctx, ctx->idx, 8 * (size_t)n)) || (rc = ensure_all(ctx, ctx->keep, (size_t)n)))
      return rc;
    HIPCHK(hipMemcpy(ctx->idx.p, idx.data(), 8 * (size_t)n, hipMemcpyHostToDevice));
    ctx->iota_n = -1;
    launch_interval_filter(ctx->U.as<uint8_t>(), ctx->rec_lin.as<int64_t>(), ctx->soa(),
                           ctx->idx.as<int64_t>(), n, ctx->iv_ref.as<int32_t>(),
                           ctx->iv_start.as<int32_t>(), ctx->iv_end.as<int32_t>(),
                           ctx->iv_begin.as<int32_t>(), ctx->n_ref, ctx->keep.as<uint8_t>(), ctx->s);
    std::vector<uint8_t> keep((size_t)n);
    HIPCHK(hipMemcpyAsync(keep.data(), ctx->keep.p, (size_t)n, hipMemcpyDeviceToHost, ctx->s));
    HIPCHK(hipStreamSynchronize(ctx->s));
    for (int64_t k = 0; k < n; k++)
      if (keep[(size_t)k]) out.push_back(b + k);
  }
  const uint64_t vb = (uint64_t)ctx->base << 16;
  const uint64_t solb = ctx->solb >= 0 && (uint64_t)ctx->solb >= vb ? (uint64_t)ctx->solb - vb : 0;
  if (tr->traverse_unplaced_unmapped && ctx->solb != -1 && ctx->ncc >= 1 &&
      (uint64_t)ctx->solb >= vb && vstart <= solb && solb < vend) {
    if ((rc = fetch_index(ctx))) return rc;
    auto& v = ctx->voff_h;
    auto it = std::lower_bound(v.begin(), v.end(), solb);
    int64_t k = it - v.begin();
    if (k < ctx->nrec) {
      std::vector<int32_t> refs((size_t)(ctx->nrec - k));
      HIPCHK(hipMemcpy(refs.data(), ctx->f_ref.as<int32_t>() + k, 4 * refs.size(), hipMemcpyDeviceToHost));
      size_t j = 0;
      while (j < refs.size() && refs[j] != -1) j++;
      for (; j < refs.size(); j++) out.push_back(k + (int64_t)j);
    }
  }
  return 0;
}

// ------------------------------------------------------------------ .bai span runs
// The interval traversal of every partition as Disq runs it (AbstractBinarySamSource.java:86-112):
// the .bai span of the optimized intervals (getFileSpan), clipped to each partition chunk, is all
// that is read.  Only the BGZF blocks of those spans are inflated (plus a few after each span to
// finish its last record), in the whole-file U layout; records are walked from every span start
// (windowed chains), selected per span chunk (BAMFileIndexIterator over the chunk list) and
// filtered by kernel 4.  The partition plans come from the last full run of the open file.
// Results: per-partition kept counts and digests (dq_partition_digests), stats.
static int run_span(dq_ctx* ctx, const dq_traversal* tr, dq_stats* out) {
  hipStream_t s = ctx->s;
  int rc;
  if (!ctx->plan_cached || !ctx->have_bai) RET(DQ_EINVAL, "span run needs a planned file and a .bai");
  const int64_t nblk = ctx->nblk;
  const uint64_t vb = (uint64_t)ctx->base << 16;  // shard coordinates <-> file coordinates
  // 1. the span of the optimized intervals, clipped to every partition chunk (shard coordinates)
  std::vector<Interval> iv;
  for (int64_t i = 0; i < tr->n; i++) {
    if (tr->ref[i] < 0 || tr->ref[i] >= ctx->n_ref) RET(DQ_EINVAL, "Invalid reference index");
    iv.push_back({tr->ref[i], tr->start[i], tr->end[i]});
  }
  const std::vector<Interval> q = optimize(iv);
  const std::vector<VChunk> span = file_span(ctx->bai, q);
  const std::vector<SplitPlan>& plans = ctx->plan_cache;
  const int64_t nsplit = (int64_t)plans.size();
  std::vector<uint64_t> cb, ce;            // span chunks, partition order
  std::vector<int64_t> part_first((size_t)nsplit + 1, 0);
  // traverseUnplacedUnmapped: the partition whose chunk holds the start of the last linear bin
  // also reads the unplaced-unmapped tail from there to the end of the file, after its interval
  // records (AbstractBinarySamSource.java:116-129) -- one more chunk, kept by tail_keep
  const bool want_tail = tr->traverse_unplaced_unmapped && ctx->solb != -1 && ctx->ncc >= 1;
  int64_t tail_chunk = -1;
  for (int64_t i = 0; i < nsplit; i++) {
    part_first[(size_t)i] = (int64_t)cb.size();
    const SplitPlan& P = plans[(size_t)i];
    if (P.rec_lin < 0) continue;
    for (const VChunk& c : clip_span(span, P.vstart + vb, P.vend + vb)) {
      if (c.b < vb) continue;
      cb.push_back(c.b - vb);
      ce.push_back(c.e - vb);
    }
    if (want_tail && P.vstart + vb <= (uint64_t)ctx->solb && (uint64_t)ctx->solb < P.vend + vb &&
        (uint64_t)ctx->solb >= vb) {
      tail_chunk = (int64_t)cb.size();
      cb.push_back((uint64_t)ctx->solb - vb);
      ce.push_back(((uint64_t)ctx->flen << 16) | 0xffff);
    }
  }
  part_first[(size_t)nsplit] = (int64_t)cb.size();
  const int64_t nchunk = (int64_t)cb.size();
  // block table of the open file (from its full run)
  std::vector<int64_t> bp((size_t)nblk), uo((size_t)nblk + 1);
  if (nblk) {
    HIPCHK(hipMemcpyAsync(bp.data(), ctx->blk_pos.p, 8 * (size_t)nblk, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(uo.data(), ctx->uoff.p, 8 * (size_t)(nblk + 1), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
  }
  const bool is_eof = !ctx->shard || ctx->base + ctx->flen >= ctx->file_len;
  // 2. windows over the union of the chunks: [block of the start, block after the end's block +
  //    extra), neighbours closer than GAP blocks merged
  struct W { int64_t j0, jc, j1; uint64_t v0; };
  constexpr int64_t GAP = 16;
  int64_t extra = ctx->span_extra_blocks;
  std::vector<uint64_t> ub(cb), ue(ce);
  {
    std::vector<size_t> ord(cb.size());
    for (size_t k = 0; k < ord.size(); k++) ord[k] = k;
    std::sort(ord.begin(), ord.end(), [&](size_t x, size_t y) { return cb[x] < cb[y]; });
    for (size_t k = 0; k < ord.size(); k++) {
      ub[k] = cb[ord[k]];
      ue[k] = ce[ord[k]];
    }
  }
  for (;;) {
    std::vector<W> win;
    for (size_t k = 0; k < ub.size(); k++) {
      const int64_t a = (int64_t)(ub[k] >> 16), e = (int64_t)(ue[k] >> 16);
      const int64_t j0 = std::lower_bound(bp.begin(), bp.end(), a) - bp.begin();
      if (j0 >= nblk || bp[(size_t)j0] != a) RET(DQ_EFORMAT, ".bai chunk does not start at a BGZF block");
      const int64_t jc = std::upper_bound(bp.begin(), bp.end(), e) - bp.begin();
      const int64_t j1 = std::min(nblk, jc + extra);
      if (!win.empty() && j0 <= win.back().j1 + GAP) {
        W& w = win.back();
        w.jc = std::max(w.jc, jc);
        w.j1 = std::max(w.j1, j1);
      } else {
        win.push_back({j0, jc, j1, ub[k]});
      }
    }
    // 3. sparse inflate of the windows' blocks
    std::vector<int32_t> sel;
    for (const W& w : win)
      for (int64_t j = std::max<int64_t>(w.j0, sel.empty() ? 0 : sel.back() + 1); j < w.j1; j++)
        sel.push_back((int32_t)j);
    const int64_t nsel = (int64_t)sel.size();
    HIPCHK(hipEventRecord(ctx->ev[5], s));
    if (nsel) {
      if ((rc = ensure_all(ctx, ctx->sel, 4 * (size_t)nsel))) return rc;
      HIPCHK(hipMemcpyAsync(ctx->sel.p, sel.data(), 4 * (size_t)nsel, hipMemcpyHostToDevice, s));
      HIPCHK(hipMemsetAsync(ctx->status.p, 0, sizeof(int32_t) * (size_t)(nblk + 1), s));
      const uint32_t* crc_init = inflate3_tables(ctx->o.device);
      if (!crc_init) RET(DQ_EDEVICE, "CRC32 table initialisation failed on this device");
      if ((rc = ensure_all(ctx, ctx->tails, INFLATE_TAIL_BYTES * (size_t)nsel))) return rc;
      launch_inflate3(ctx->cbuf(), ctx->blk_pos.as<int64_t>(), ctx->blk_cs.as<int32_t>(),
                      ctx->blk_us.as<int32_t>(), ctx->uoff.as<int64_t>(), nblk, ctx->U.as<uint8_t>(),
                      ctx->status.as<int32_t>(), ctx->o.verify_crc, crc_init, nullptr, s,
                      ctx->sel.as<int32_t>(), nsel, ctx->tails.p);
    }
    HIPCHK(hipEventRecord(ctx->ev[6], s));
    {
      // the first failed selected block, by a device reduction (one word back)
      unsigned long long* d_bad = reinterpret_cast<unsigned long long*>(ctx->scal.as<char>() + 144);
      HIPCHK(hipMemsetAsync(d_bad, 0xff, 8, s));
      if (nsel) launch_first_bad(ctx->status.as<int32_t>(), ctx->sel.as<int32_t>(), nsel, d_bad, s);
      unsigned long long bad = 0;
      HIPCHK(hipMemcpyAsync(&bad, d_bad, 8, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      if (bad != ~0ull) {
        int32_t st = 0;
        HIPCHK(hipMemcpy(&st, ctx->status.as<int32_t>() + bad, 4, hipMemcpyDeviceToHost));
        char msg[256];
        snprintf(msg, sizeof msg, "%s in BGZF block at %lld", status_name(st),
                 (long long)(bp[(size_t)bad] + ctx->base));
        RET(DQ_EFORMAT, msg);
      }
    }
    // 4. windowed record chains
    const int64_t SEG = 64 * 1024;
    std::vector<Win> wv;
    int64_t nseg = 0;
    for (const W& w : win) {
      Win x;
      x.u_start = uo[(size_t)w.j0] + (int64_t)(w.v0 & 0xffff);
      x.u_chain_end = uo[(size_t)w.jc];
      x.u_limit = uo[(size_t)w.j1];
      x.at_eof = (w.j1 == nblk && is_eof) ? 1 : 0;
      x.pad = 0;
      x.seg0 = nseg;
      if (x.u_chain_end <= x.u_start) x.u_chain_end = x.u_start + 1;
      nseg += (x.u_chain_end - x.u_start + SEG - 1) / SEG;
      wv.push_back(x);
    }
    const int64_t nwin = (int64_t)wv.size();
    int64_t nrec = 0;
    int32_t* d_broken = ctx->scal.as<int32_t>() + 1;
    int32_t* d_stat = ctx->scal.as<int32_t>() + 2;
    if (nseg > 0) {
      if ((rc = ensure_all(ctx, ctx->wins, sizeof(Win) * (size_t)nwin)) ||
          (rc = ensure_all(ctx, ctx->segs, sizeof(Seg) * (size_t)(nseg + 1))) ||
          (rc = ensure_all(ctx, ctx->segcnt, sizeof(int64_t) * (size_t)(nseg + 1))) ||
          (rc = ensure_all(ctx, ctx->segbase, sizeof(int64_t) * (size_t)(nseg + 1))))
        return rc;
      HIPCHK(hipMemcpyAsync(ctx->wins.p, wv.data(), sizeof(Win) * (size_t)nwin, hipMemcpyHostToDevice, s));
      HIPCHK(hipMemsetAsync(ctx->scal.p, 0, 64, s));
      launch_wseg(ctx->U.as<uint8_t>(), ctx->d_ref_len.as<int32_t>(), ctx->n_ref, ctx->wins.as<Win>(),
                  nwin, ctx->segs.as<Seg>(), nseg, SEG, d_broken, s);
      int32_t br = 0;
      HIPCHK(hipMemcpyAsync(&br, d_broken, 4, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      int32_t st = 0;
      if (br) {
        launch_wseg_fix(ctx->U.as<uint8_t>(), ctx->segs.as<Seg>(), ctx->wins.as<Win>(), nwin, nseg,
                        SEG, d_stat, s);
        HIPCHK(hipMemcpyAsync(&st, d_stat, 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
      }
      if (st == 4) {  // a window's last record runs past its blocks: more blocks, again
        if (extra >= nblk) RET(DQ_EFORMAT, "truncated record chain");
        extra *= 4;
        ctx->span_extra_blocks = extra;
        continue;
      }
      if (st) RET(DQ_EFORMAT, st == ST_BAD_CODE ? "Invalid record length" : "truncated record chain");
      launch_seg_counts(ctx->segs.as<Seg>(), nseg, ctx->segcnt.as<int64_t>(), s);
      if ((rc = ensure_scan(ctx, nseg))) return rc;
      launch_exclusive_scan_i64(ctx->segcnt.as<int64_t>(), ctx->segbase.as<int64_t>(), nseg,
                                ctx->tmp.as<int64_t>(), s);
      if ((rc = get_i64(ctx, ctx->segbase.as<int64_t>() + nseg, &nrec))) return rc;
    }
    const size_t nr = (size_t)std::max<int64_t>(1, nrec);
    if ((rc = ensure_all(ctx, ctx->rec_lin, 8 * nr))) return rc;
    DevBuf* b8[] = {&ctx->f_voff, &ctx->f_hash};
    DevBuf* b4[] = {&ctx->f_bs, &ctx->f_ref, &ctx->f_pos, &ctx->f_lseq, &ctx->f_nref, &ctx->f_npos,
                    &ctx->f_tlen};
    DevBuf* b2[] = {&ctx->f_flag, &ctx->f_bin, &ctx->f_ncig};
    DevBuf* b1[] = {&ctx->f_mapq, &ctx->f_lrn};
    for (auto* b : b8) if ((rc = ensure_all(ctx, *b, 8 * nr))) return rc;
    for (auto* b : b4) if ((rc = ensure_all(ctx, *b, 4 * nr))) return rc;
    for (auto* b : b2) if ((rc = ensure_all(ctx, *b, 2 * nr))) return rc;
    for (auto* b : b1) if ((rc = ensure_all(ctx, *b, nr))) return rc;
    ctx->have_pipeline = false;  // the record arrays now hold the span records
    ctx->voff_h.clear();
    if (nrec > 0) {
      launch_seg_emit2(ctx->U.as<uint8_t>(), ctx->ulen, ctx->segs.as<Seg>(),
                       ctx->segbase.as<int64_t>(), nseg, ctx->rec_lin.as<int64_t>(), s);
      if ((rc = decode_records(ctx, nrec, nblk, d_stat, s))) return rc;
    }
    // 5. records of every span chunk, kernel 4, per-partition digests of the kept records
    int64_t nidx = 0;
    const size_t ncs = (size_t)std::max<int64_t>(1, nchunk);
    if ((rc = ensure_all(ctx, ctx->span_c, 16 * ncs)) ||
        (rc = ensure_all(ctx, ctx->span_r, 8 * (3 * ncs + 2))))
      return rc;
    uint64_t* d_cb = ctx->span_c.as<uint64_t>();
    uint64_t* d_ce = d_cb + ncs;
    int64_t* d_first = ctx->span_r.as<int64_t>();
    int64_t* d_cnt = d_first + ncs;
    int64_t* d_off = d_cnt + ncs;  // nchunk + 1
    if (nchunk) {
      HIPCHK(hipMemcpyAsync(d_cb, cb.data(), 8 * (size_t)nchunk, hipMemcpyHostToDevice, s));
      HIPCHK(hipMemcpyAsync(d_ce, ce.data(), 8 * (size_t)nchunk, hipMemcpyHostToDevice, s));
      launch_span_ranges(ctx->f_voff.as<uint64_t>(), nrec, d_cb, d_ce, nchunk, d_first, d_cnt, s);
      if ((rc = ensure_scan(ctx, nchunk))) return rc;
      launch_exclusive_scan_i64(d_cnt, d_off, nchunk, ctx->tmp.as<int64_t>(), s);
      if ((rc = get_i64(ctx, d_off + nchunk, &nidx))) return rc;
    }
    const size_t ni = (size_t)std::max<int64_t>(1, nidx);
    if ((rc = ensure_all(ctx, ctx->span_idx, 8 * ni)) || (rc = ensure_all(ctx, ctx->keep, ni)) ||
        (rc = ensure_all(ctx, ctx->span_keep32, 4 * ni)) ||
        (rc = ensure_all(ctx, ctx->span_off, 8 * (ni + 1))) ||
        (rc = ensure_all(ctx, ctx->span_kept, 8 * ni)))
      return rc;
    int64_t nkept = 0;
    if (nidx > 0) {
      launch_ranges_to_idx(d_first, d_off, nchunk, ctx->span_idx.as<int64_t>(), s);
      if ((rc = upload_intervals(ctx, tr))) return rc;
      launch_interval_filter(ctx->U.as<uint8_t>(), ctx->rec_lin.as<int64_t>(), ctx->soa(),
                             ctx->span_idx.as<int64_t>(), nidx, ctx->iv_ref.as<int32_t>(),
                             ctx->iv_start.as<int32_t>(), ctx->iv_end.as<int32_t>(),
                             ctx->iv_begin.as<int32_t>(), ctx->n_ref, ctx->keep.as<uint8_t>(), s);
      if (tail_chunk >= 0) {
        unsigned long long* d_first = reinterpret_cast<unsigned long long*>(ctx->scal.as<char>() + 152);
        HIPCHK(hipMemsetAsync(d_first, 0xff, 8, s));
        launch_tail_keep(ctx->span_idx.as<int64_t>(), d_off, (int)tail_chunk, ctx->f_ref.as<int32_t>(),
                         d_first, ctx->keep.as<uint8_t>(), nidx, s);
      }
      launch_keep_to_i32(ctx->keep.as<uint8_t>(), nidx, ctx->span_keep32.as<int32_t>(), s);
      if ((rc = ensure_scan(ctx, nidx))) return rc;
      launch_exclusive_scan_i32(ctx->span_keep32.as<int32_t>(), ctx->span_off.as<int64_t>(), nidx,
                                ctx->tmp.as<int64_t>(), s);
      launch_compact_kept(ctx->span_idx.as<int64_t>(), ctx->keep.as<uint8_t>(),
                          ctx->span_off.as<int64_t>(), nidx, ctx->span_kept.as<int64_t>(), s);
      if ((rc = get_i64(ctx, ctx->span_off.as<int64_t>() + nidx, &nkept))) return rc;
    }
    // partition p: span chunks [part_first[p], part_first[p+1]) -> idx [off[.], off[.]) -> kept
    std::vector<int64_t> cpos((size_t)nsplit + 1), ipos((size_t)nsplit + 1, 0), kpos((size_t)nsplit + 1, 0);
    if (nchunk) {
      std::vector<int64_t> offh((size_t)nchunk + 1);
      HIPCHK(hipMemcpy(offh.data(), d_off, 8 * (size_t)(nchunk + 1), hipMemcpyDeviceToHost));
      for (int64_t p = 0; p <= nsplit; p++) ipos[(size_t)p] = offh[(size_t)part_first[(size_t)p]];
    }
    if (nidx > 0) {
      DevBuf pos;
      HIPCHK(pos.ensure(16 * (size_t)(nsplit + 1)));
      HIPCHK(hipMemcpyAsync(pos.p, ipos.data(), 8 * (size_t)(nsplit + 1), hipMemcpyHostToDevice, s));
      launch_gather_i64(ctx->span_off.as<int64_t>(), pos.as<int64_t>(), nsplit + 1,
                        pos.as<int64_t>() + nsplit + 1, s);
      HIPCHK(hipMemcpyAsync(kpos.data(), pos.as<int64_t>() + nsplit + 1, 8 * (size_t)(nsplit + 1),
                            hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
    }
    std::vector<PartRange> parts((size_t)nsplit);
    for (int64_t p = 0; p < nsplit; p++) parts[(size_t)p] = {kpos[(size_t)p], kpos[(size_t)p + 1], 0};
    if ((rc = ensure_all(ctx, ctx->parts, sizeof(PartRange) * (size_t)(nsplit + 1)))) return rc;
    if (nsplit) {
      HIPCHK(hipMemcpyAsync(ctx->parts.p, parts.data(), sizeof(PartRange) * (size_t)nsplit,
                            hipMemcpyHostToDevice, s));
      if (nkept > 0)
        launch_partition_digest_idx(ctx->f_hash.as<uint64_t>(), ctx->span_kept.as<int64_t>(),
                                    ctx->parts.as<PartRange>(), nsplit, s);
      HIPCHK(hipEventRecord(ctx->ev[7], s));
      HIPCHK(hipMemcpyAsync(parts.data(), ctx->parts.p, sizeof(PartRange) * (size_t)nsplit,
                            hipMemcpyDeviceToHost, s));
    } else {
      HIPCHK(hipEventRecord(ctx->ev[7], s));
    }
    int32_t st2 = 0;
    HIPCHK(hipMemcpyAsync(&st2, d_stat, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (st2 && nrec > 0) {
      // diagnostics: the first record start that is out of order or whose block_size runs past U
      std::vector<int64_t> rl((size_t)nrec);
      HIPCHK(hipMemcpy(rl.data(), ctx->rec_lin.p, 8 * (size_t)nrec, hipMemcpyDeviceToHost));
      int64_t bad = -1, wmax = 0;
      for (const Win& x : wv) wmax = std::max(wmax, x.u_limit - x.u_start);
      for (int64_t i = 0; i < nrec && bad < 0; i++) {
        int32_t bs = 0;
        if (rl[(size_t)i] < 0 || rl[(size_t)i] + 4 > ctx->ulen) { bad = i; break; }
        if (i % 4096 == 0 || (i > 0 && rl[(size_t)i] <= rl[(size_t)i - 1])) {
          HIPCHK(hipMemcpy(&bs, ctx->U.as<uint8_t>() + rl[(size_t)i], 4, hipMemcpyDeviceToHost));
          if (bs < 32 || rl[(size_t)i] + 4 + bs > ctx->ulen || (i > 0 && rl[(size_t)i] <= rl[(size_t)i - 1])) bad = i;
        }
      }
      char msg[320];
      snprintf(msg, sizeof msg,
               "truncated BAM record (span run: %lld records, %lld windows, %lld segments, largest "
               "window %lld bytes, ulen %lld, first bad record %lld at %lld)",
               (long long)nrec, (long long)nwin, (long long)nseg, (long long)wmax,
               (long long)ctx->ulen, (long long)bad, bad >= 0 ? (long long)rl[(size_t)bad] : -1LL);
      RET(DQ_EFORMAT, msg);
    }
    ctx->parts_h = parts;
    dq_stats S = ctx->stats;
    S.n_records = nidx;
    S.n_filtered = nkept;
    S.blocks_inflated = nsel;
    S.ms_inflate = ev_ms(ctx->ev[5], ctx->ev[6]);
    S.ms_span = ev_ms(ctx->ev[5], ctx->ev[7]);
    uint64_t dg = 0;
    for (int64_t i = 0; i < nsplit; i++)
      dg += dq_mix64(parts[(size_t)i].digest ^ ((uint64_t)(i + 1) * DQ_K_WORD));
    S.digest = dg;
    ctx->span_parts_valid = true;
    *out = S;
    return 0;
  }
}

// ------------------------------------------------------------------ opening inputs
static void reset_open(dq_ctx* ctx, int64_t len) {
  ctx->plan_cached = false;
  ctx->flen = len;
  ctx->have_file = true;
  ctx->have_pipeline = false;
  ctx->shard = false;
  ctx->base = 0;
  ctx->file_len = len;
  ctx->p0 = 0;
  ctx->p1 = 0;
  ctx->cext = nullptr;
  ctx->chunk_mode = false;
  ctx->text_mode = false;
  ctx->have_text = false;
}

// Bytes [off, off + len) of an open file into C (plus the 4 KiB zero pad): read() into two pinned
// staging buffers in turn, each copied asynchronously while the next piece is read from the page
// cache (the role of Disq's 2 x 4 MB NIO prefetcher, SeekableByteChannelPrefetcher.java:45).
// DQ_MMAP=1 (tuning builds, -DDQ_TUNING): the same by DMA straight from the file's page-cache pages (the range mapped read-only
// and registered with the device, one copy into C).  Measured slower than the staging path (page
// registration of 2 GB windows: end-to-end 14.9-19.9 GB/s against 27.5-35.3 GB/s,
// profiles/r3s_e2e_ab.txt), so it is off by default.  Returns 1 when it is off or unavailable.
static int upload_file_range_mapped(dq_ctx* ctx, int fd, int64_t off, int64_t len) {
#ifdef DQ_TUNING
  static const bool enabled = getenv("DQ_MMAP") && atoi(getenv("DQ_MMAP")) == 1;
#else
  constexpr bool enabled = false;  // measured slower than pinned staging (profiles/r3s_e2e_ab.txt)
#endif
  if (!enabled || len < (64 << 20)) return 1;
  const int64_t pg = (int64_t)sysconf(_SC_PAGESIZE);
  const int64_t a = off & ~(pg - 1), d = off - a, mlen = len + d;
  void* p = mmap(nullptr, (size_t)mlen, PROT_READ, MAP_SHARED, fd, (off_t)a);
  if (p == MAP_FAILED) return 1;
  if (hipHostRegister(p, (size_t)mlen, hipHostRegisterReadOnly) != hipSuccess) {
    (void)hipGetLastError();
    munmap(p, (size_t)mlen);
    return 1;
  }
  int rc = ensure_all(ctx, ctx->C, (size_t)len + 4096);
  hipError_t e = hipSuccess;
  if (!rc) {
    e = hipMemcpyAsync(ctx->C.as<uint8_t>(), (const uint8_t*)p + d, (size_t)len, hipMemcpyHostToDevice, ctx->s);
    if (e == hipSuccess) e = hipMemsetAsync(ctx->C.as<uint8_t>() + len, 0, 4096, ctx->s);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->s);
  }
  (void)hipHostUnregister(p);
  munmap(p, (size_t)mlen);
  if (rc) return rc;
  if (e != hipSuccess) RET(DQ_EDEVICE, std::string("file range H2D: ") + hipGetErrorString(e));
  reset_open(ctx, len);
  ctx->h2d_bytes = len;
  return 0;
}

static int upload_file_range(dq_ctx* ctx, int fd, int64_t off, int64_t len) {
  constexpr size_t PIECE = PIN_PIECE;
  int rc;
  if ((rc = upload_file_range_mapped(ctx, fd, off, len)) != 1) return rc;
  if ((rc = ensure_all(ctx, ctx->C, (size_t)len + 4096))) return rc;
  if ((rc = ensure_pinned(ctx))) return rc;
  bool used[2] = {false, false};
  int k = 0;
  for (int64_t done = 0; done < len; k ^= 1) {
    const size_t n = (size_t)std::min<int64_t>((int64_t)PIECE, len - done);
    if (used[k]) HIPCHK(hipEventSynchronize(ctx->pin_ev[k]));  // its previous copy is done
    // sixteen readers per piece (one thread copies out of the page cache at a fraction of PCIe)
    constexpr int T = 16;
    bool ok[T];
    std::thread th[T];
    const size_t part = (n + T - 1) / T;
    for (int t = 0; t < T; t++)
      th[t] = std::thread([&, t] {
        const size_t a = std::min(n, (size_t)t * part), b = std::min(n, a + part);
        size_t got = a;
        ok[t] = true;
        while (got < b) {
          const ssize_t r = pread(fd, ctx->pin[k] + got, b - got, (off_t)(off + done + (int64_t)got));
          if (r <= 0) {
            ok[t] = false;
            return;
          }
          got += (size_t)r;
        }
      });
    for (auto& x : th) x.join();
    for (int t = 0; t < T; t++)
      if (!ok[t]) RET(DQ_EIO, "short read");
    HIPCHK(hipMemcpyAsync(ctx->C.as<uint8_t>() + done, ctx->pin[k], n, hipMemcpyHostToDevice, ctx->s));
    HIPCHK(hipEventRecord(ctx->pin_ev[k], ctx->s));
    used[k] = true;
    done += (int64_t)n;
  }
  HIPCHK(hipMemsetAsync(ctx->C.as<uint8_t>() + len, 0, 4096, ctx->s));
  HIPCHK(hipStreamSynchronize(ctx->s));
  reset_open(ctx, len);
  ctx->h2d_bytes = len;
  return 0;
}

struct Fd {
  int fd = -1;
  ~Fd() {
    if (fd >= 0) close(fd);
  }
};

static int open_fd(dq_ctx* ctx, const char* path, Fd& f, int64_t* flen) {
  f.fd = open(path, O_RDONLY);
  if (f.fd < 0) RET(DQ_EIO, std::string("cannot open ") + path);
  struct stat st;
  if (fstat(f.fd, &st) != 0) RET(DQ_EIO, std::string("cannot stat ") + path);
  *flen = (int64_t)st.st_size;
  return 0;
}

// The file's decompressed BAM header into ctx->hdr (AbstractSamSource.getFileHeader): the first
// bytes of the file, growing the prefix until the header is whole.
static int load_header(dq_ctx* ctx, int fd, int64_t flen) {
  int64_t n = std::min<int64_t>(flen, 1 << 20);
  for (;;) {
    int rc = upload_file_range(ctx, fd, 0, n);
    if (rc) return rc;
    ctx->shard = true;  // a prefix: its end is not EOF unless it is the whole file
    ctx->file_len = n < flen ? INT64_MAX / 4 : flen;
    ctx->header_only = true;
    rc = run_pipeline(ctx);
    ctx->header_only = false;
    ctx->have_pipeline = false;
    ctx->have_file = false;
    if (rc == 0) {
      ctx->hdr.resize((size_t)ctx->header_bytes);
      HIPCHK(hipMemcpy(ctx->hdr.data(), ctx->U.p, (size_t)ctx->header_bytes, hipMemcpyDeviceToHost));
      return 0;
    }
    if (n >= flen) return rc;
    n = std::min<int64_t>(flen, n * 8);
  }
}

// The header of `path` into ctx->hdr, read once per context and path.
static int chunk_header(dq_ctx* ctx, const char* path, int fd, int64_t flen) {
  if (ctx->chunk_hdr_path == path) return 0;
  ctx->chunk_hdr_path.clear();
  int rc = load_header(ctx, fd, flen);
  if (rc) return rc;
  ctx->chunk_hdr_path = path;
  return 0;
}

// One Chunk [vstart, vend) of an open file decoded from its own bytes (dq_decode_chunk): the
// chunk's blocks, then enough to finish its last record (grown x4 while it runs past).  On
// success *any says whether records were read; ctx->parts_h[0] is their range.
static int chunk_run(dq_ctx* ctx, int fd, int64_t flen, uint64_t vstart, uint64_t vend, bool* any) {
  *any = false;
  const int64_t c0 = (int64_t)(vstart >> 16);
  if (vend <= vstart || c0 >= flen) return 0;
  int64_t extra = 256 << 10, h2d = ctx->h2d_bytes;
  int rc;
  for (;;) {
    const int64_t c1 = std::min<int64_t>(flen, std::min<int64_t>(flen, (int64_t)(vend >> 16)) + extra);
    if ((rc = upload_file_range(ctx, fd, c0, c1 - c0))) return rc;
    h2d += c1 - c0;
    ctx->shard = true;
    ctx->base = c0;
    ctx->file_len = flen;
    ctx->p0 = 0;
    ctx->p1 = 1;
    ctx->chunk_mode = true;
    ctx->chunk_vs = vstart - ((uint64_t)c0 << 16);
    ctx->chunk_ve = vend - ((uint64_t)c0 << 16);
    ctx->h2d_bytes = h2d;
    rc = run_pipeline(ctx);
    if (rc == DQ_EFORMAT && ctx->err.find("halo too small") != std::string::npos && c1 < flen) {
      extra *= 4;
      continue;
    }
    break;
  }
  ctx->chunk_mode = false;
  ctx->stats.h2d_bytes = h2d;
  if (rc) {
    ctx->have_file = false;
    return rc;
  }
  *any = true;
  return 0;
}

// One batch holding the records of `parts` in order (a single partition).  The parts carry every
// field (the digest needs the hashes); lean: the result keeps only voffset and raw.
static int concat_batches(dq_ctx* ctx, const std::vector<dq_batch*>& parts, bool lean, dq_batch** out) {
  int64_t n = 0, raw = 0;
  bool with_raw = true;
  for (const dq_batch* b : parts) {
    n += b->n_records;
    raw += b->raw_len;
    with_raw = with_raw && (b->raw != nullptr || b->n_records == 0);
  }
  dq_batch* o = (dq_batch*)calloc(1, sizeof(dq_batch));
  if (!o) RET(DQ_ENOMEM, "out of host memory");
  const size_t m = (size_t)std::max<int64_t>(1, n);
  o->n_records = n;
  o->voffset = (uint64_t*)malloc(8 * m);
  if (!lean) {
    o->block_size = (int32_t*)malloc(4 * m);
    o->ref_id = (int32_t*)malloc(4 * m);
    o->pos = (int32_t*)malloc(4 * m);
    o->l_seq = (int32_t*)malloc(4 * m);
    o->next_ref_id = (int32_t*)malloc(4 * m);
    o->next_pos = (int32_t*)malloc(4 * m);
    o->tlen = (int32_t*)malloc(4 * m);
    o->flag = (uint16_t*)malloc(2 * m);
    o->bin = (uint16_t*)malloc(2 * m);
    o->n_cigar = (uint16_t*)malloc(2 * m);
    o->mapq = (uint8_t*)malloc(m);
    o->l_read_name = (uint8_t*)malloc(m);
    o->hash = (uint64_t*)malloc(8 * m);
    o->raw_offset = (int64_t*)malloc(8 * m);
  }
  o->raw = with_raw ? (uint8_t*)malloc((size_t)std::max<int64_t>(1, raw)) : nullptr;
  o->raw_len = raw;
  o->n_partitions = 1;
  o->part_offset = (int64_t*)malloc(16);
  o->part_digest = (uint64_t*)calloc(2, sizeof(uint64_t));
  if (!o->voffset || (with_raw && !o->raw) || !o->part_offset || !o->part_digest ||
      (!lean && (!o->block_size || !o->ref_id || !o->pos || !o->l_seq || !o->next_ref_id ||
                 !o->next_pos || !o->tlen || !o->flag || !o->bin || !o->n_cigar || !o->mapq ||
                 !o->l_read_name || !o->hash || !o->raw_offset))) {
    dq_batch_free(o);
    RET(DQ_ENOMEM, "out of host memory");
  }
  int64_t k = 0, r = 0;
  uint64_t d = 0;
  for (const dq_batch* b : parts) {
    const size_t c = (size_t)b->n_records;
#define CP(f, sz) memcpy(o->f + k, b->f, (sz) * c)
    CP(voffset, 8);
    if (!lean) {
      CP(block_size, 4); CP(ref_id, 4); CP(pos, 4); CP(l_seq, 4); CP(next_ref_id, 4);
      CP(next_pos, 4); CP(tlen, 4); CP(flag, 2); CP(bin, 2); CP(n_cigar, 2); CP(mapq, 1);
      CP(l_read_name, 1); CP(hash, 8);
      for (size_t i = 0; i < c; i++) o->raw_offset[k + (int64_t)i] = b->raw_offset[i] + r;
    }
#undef CP
    for (size_t i = 0; i < c; i++) d += dq_mix64(b->hash[i] + (uint64_t)(k + (int64_t)i + 1) * DQ_K_LEN);
    if (with_raw && b->raw_len) memcpy(o->raw + r, b->raw, (size_t)b->raw_len);
    k += (int64_t)c;
    r += b->raw_len;
  }
  o->part_offset[0] = 0;
  o->part_offset[1] = n;
  o->part_digest[0] = d;
  *out = o;
  return 0;
}

// ------------------------------------------------------------------ C ABI
// queryUnmapped reads the unplaced-unmapped tail to the end of the FILE (H/BAMFileReader2.java:
// 715-738): a shard whose bytes stop before it cannot produce that tail.
static int check_tail_reachable(dq_ctx* ctx, const dq_traversal* tr) {
  if (tr && tr->traverse_unplaced_unmapped && ctx->shard && !ctx->chunk_mode &&
      ctx->base + ctx->flen < ctx->file_len)
    RET(DQ_EINVAL, "traverseUnplacedUnmapped on a shard that does not reach the end of the file");
  return 0;
}

extern "C" {

const char* dq_version(void) { return "disq_amd 0.2 (gfx950)"; }
int32_t dq_abi_version(void) { return DQ_ABI_VERSION; }

int dq_ctx_create(dq_ctx** out, const dq_opts* opts) {
  if (!out) return DQ_EINVAL;
  dq_ctx* ctx = new dq_ctx();
  if (opts) ctx->o = *opts;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    ctx->err = "no HIP device";
    *out = ctx;
    return DQ_EDEVICE;
  }
  if (ctx->o.device < 0 || ctx->o.device >= ndev) {
    ctx->err = "bad device ordinal";
    *out = ctx;
    return DQ_EINVAL;
  }
  HIPCHK(hipSetDevice(ctx->o.device));
  HIPCHK(hipStreamCreateWithFlags(&ctx->s, hipStreamNonBlocking));
  {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, ctx->o.device) == hipSuccess && prop.multiProcessorCount > 0)
      ctx->n_cu = prop.multiProcessorCount;
  }
  for (auto& e : ctx->ev) HIPCHK(hipEventCreate(&e));
  *out = ctx;
  return 0;
}

void dq_ctx_destroy(dq_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->o.device);
  // both streams drained before any pinned buffer they copy into is released
  if (ctx->s) (void)hipStreamSynchronize(ctx->s);
  if (ctx->sx) (void)hipStreamSynchronize(ctx->sx);
  for (auto& e : ctx->ev)
    if (e) (void)hipEventDestroy(e);
  for (int k = 0; k < 2; k++) {
    if (ctx->pin_ev[k]) (void)hipEventDestroy(ctx->pin_ev[k]);
    if (ctx->pin[k]) (void)hipHostFree(ctx->pin[k]);
  }
  if (ctx->ah) {  // a live arena batch keeps the arena: its dq_batch_free releases it
    bool keep;
    {
      std::lock_guard<std::mutex> lk(ctx->ah->mu);
      keep = ctx->ah->live;
      ctx->ah->orphan = true;
    }
    if (!keep) {
      if (ctx->ah->arena) (void)hipHostFree(ctx->ah->arena);
      delete ctx->ah;
    }
    ctx->ah = nullptr;
    ctx->arena = nullptr;
  }
  for (auto& e : ctx->ev_x)
    if (e) (void)hipEventDestroy(e);
  if (ctx->sx) (void)hipStreamDestroy(ctx->sx);
  if (ctx->s) (void)hipStreamDestroy(ctx->s);
  delete ctx;
}

const char* dq_last_error(const dq_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int dq_open_memory(dq_ctx* ctx, const uint8_t* bam, int64_t len) {
  if (!ctx || (!bam && len > 0) || len < 0) return DQ_EINVAL;
  ON_DEVICE(ctx);
  int rc;
  if ((rc = ensure_all(ctx, ctx->C, (size_t)len + 4096))) return rc;
  if (len) HIPCHK(hipMemcpy(ctx->C.p, bam, (size_t)len, hipMemcpyHostToDevice));
  HIPCHK(hipMemset(ctx->C.as<uint8_t>() + len, 0, 4096));
  reset_open(ctx, len);
  ctx->h2d_bytes = len;
  return 0;
}

int dq_open_shard_device(dq_ctx* ctx, const void* dev_bytes, int64_t len, int64_t base,
                         int64_t file_len, int64_t p0, int64_t p1, const uint8_t* header,
                         int64_t header_len) {
  if (!ctx || !dev_bytes || len <= 0 || base < 0 || base + len > file_len || p0 < 0 || p1 <= p0 ||
      !header || header_len <= 0)
    return DQ_EINVAL;
  ON_DEVICE(ctx);
  reset_open(ctx, len);
  ctx->cext = static_cast<const uint8_t*>(dev_bytes);
  ctx->h2d_bytes = 0;
  ctx->shard = true;
  ctx->base = base;
  ctx->file_len = file_len;
  ctx->p0 = p0;
  ctx->p1 = p1;
  ctx->hdr.assign(header, header + header_len);
  return 0;
}

int dq_open_shard(dq_ctx* ctx, const uint8_t* bytes, int64_t len, int64_t base, int64_t file_len,
                  int64_t p0, int64_t p1, const uint8_t* header, int64_t header_len) {
  if (!ctx || (!bytes && len > 0) || len < 0 || base < 0 || base + len > file_len || p0 < 0 ||
      p1 <= p0 || !header || header_len <= 0)
    return DQ_EINVAL;
  const int rc = dq_open_memory(ctx, bytes, len);
  if (rc) return rc;
  ctx->shard = true;
  ctx->base = base;
  ctx->file_len = file_len;
  ctx->p0 = p0;
  ctx->p1 = p1;
  ctx->hdr.assign(header, header + header_len);
  return 0;
}

int dq_open_path(dq_ctx* ctx, const char* path) {
  if (!ctx || !path) return DQ_EINVAL;
  ON_DEVICE(ctx);
  Fd f;
  int64_t len = 0;
  int rc = open_fd(ctx, path, f, &len);
  if (rc) return rc;
  return upload_file_range(ctx, f.fd, 0, len);
}

int dq_open_shard_path(dq_ctx* ctx, const char* path, int64_t base, int64_t len, int64_t p0,
                       int64_t p1, const uint8_t* header, int64_t header_len) {
  if (!ctx || !path || base < 0 || len <= 0 || p0 < 0 || p1 <= p0 || !header || header_len <= 0)
    return DQ_EINVAL;
  ON_DEVICE(ctx);
  Fd f;
  int64_t flen = 0;
  int rc = open_fd(ctx, path, f, &flen);
  if (rc) return rc;
  if (base + len > flen) RET(DQ_EINVAL, "shard range past the end of the file");
  if ((rc = upload_file_range(ctx, f.fd, base, len))) return rc;
  ctx->shard = true;
  ctx->base = base;
  ctx->file_len = flen;
  ctx->p0 = p0;
  ctx->p1 = p1;
  ctx->hdr.assign(header, header + header_len);
  return 0;
}

int dq_decode_chunk(dq_ctx* ctx, const char* path, uint64_t vstart, uint64_t vend, int32_t with_raw,
                    dq_batch** out) {
  if (!ctx || !path || !out) return DQ_EINVAL;
  ON_DEVICE(ctx);
  Fd f;
  int64_t flen = 0;
  int rc = open_fd(ctx, path, f, &flen);
  if (rc) return rc;
  if ((rc = chunk_header(ctx, path, f.fd, flen))) return rc;
  ctx->h2d_bytes = 0;
  bool any = false;
  if ((rc = chunk_run(ctx, f.fd, flen, vstart, vend, &any))) return rc;
  if (!any) return make_batch(ctx, {}, nullptr, with_raw, {0, 0}, out);
  const PartRange r = ctx->parts_h[0];
  rc = make_batch(ctx, {{r.begin, r.end}}, nullptr, with_raw, {0, r.end - r.begin}, out);
  ctx->have_file = false;  // the window is not a file the other calls can use
  ctx->have_pipeline = false;
  return rc;
}

int dq_decode_chunk_filtered(dq_ctx* ctx, const char* path, uint64_t vstart, uint64_t vend,
                             const dq_traversal* tr, int32_t with_raw, dq_batch** out) {
  if (!ctx || !path || !out || !tr) return DQ_EINVAL;
  ON_DEVICE(ctx);
  if (!tr->has_intervals && !tr->traverse_unplaced_unmapped)
    RET(DQ_EINVAL, "Traversing mapped reads only is not supported.");
  if (!ctx->have_bai) RET(DQ_EINVAL, "Intervals set but no index file found");
  if (with_raw < DQ_EXPORT_FIELDS || with_raw > DQ_EXPORT_LEAN) RET(DQ_EINVAL, "unknown export mode");
  // the windows' batches carry every field (their hashes make the chunk's digest); a lean result
  // keeps voffset + raw of them (concat_batches)
  const int32_t part_mode = with_raw == DQ_EXPORT_LEAN ? DQ_EXPORT_RAW : with_raw;
  Fd f;
  int64_t flen = 0;
  int rc = open_fd(ctx, path, f, &flen);
  if (rc) return rc;
  if ((rc = chunk_header(ctx, path, f.fd, flen))) return rc;
  ctx->h2d_bytes = 0;
  std::vector<dq_batch*> parts;
  auto cleanup = [&](int code) {
    for (dq_batch* b : parts) dq_batch_free(b);
    ctx->have_file = false;
    ctx->have_pipeline = false;
    return code;
  };
  if (tr->has_intervals && tr->n > 0) {
    // the .bai span of the optimized intervals clipped to this chunk (AbstractBinarySamSource
    // .java:102-107); nearby span chunks are read as one window
    std::vector<Interval> iv;
    for (int64_t i = 0; i < tr->n; i++) {
      if (tr->ref[i] < 0 || tr->ref[i] >= ctx->n_ref) return cleanup(DQ_EINVAL);
      iv.push_back({tr->ref[i], tr->start[i], tr->end[i]});
    }
    const std::vector<VChunk> span = clip_span(file_span(ctx->bai, optimize(iv)), vstart, vend);
    constexpr int64_t GAP = 1 << 20;  // compressed bytes between chunks read through
    for (size_t i = 0; i < span.size();) {
      size_t j = i + 1;
      while (j < span.size() && (int64_t)(span[j].b >> 16) <= (int64_t)(span[j - 1].e >> 16) + GAP) j++;
      bool any = false;
      if ((rc = chunk_run(ctx, f.fd, flen, span[i].b, span[j - 1].e, &any))) return cleanup(rc);
      if (any) {
        // records of the window inside one of its span chunks (BAMFileIndexIterator over the
        // chunk list), then kernel 4 (BAMQueryMultipleIntervalsIteratorFilter, contained=false)
        const PartRange r = ctx->parts_h[0];
        std::vector<uint64_t> v((size_t)(r.end - r.begin));
        if (!v.empty())
          HIPCHK(hipMemcpy(v.data(), ctx->f_voff.as<uint64_t>() + r.begin, 8 * v.size(),
                           hipMemcpyDeviceToHost));
        const uint64_t vb = (uint64_t)ctx->base << 16;
        std::vector<int64_t> idx;
        size_t c = i;
        for (size_t k = 0; k < v.size(); k++) {
          const uint64_t x = v[k] + vb;
          while (c < j && span[c].e <= x) c++;
          if (c < j && span[c].b <= x) idx.push_back(r.begin + (int64_t)k);
        }
        std::vector<int64_t> kept;
        if (!idx.empty()) {
          const int64_t n = (int64_t)idx.size();
          if ((rc = upload_intervals(ctx, tr)) || (rc = ensure_all(ctx, ctx->idx, 8 * (size_t)n)) ||
              (rc = ensure_all(ctx, ctx->keep, (size_t)n)))
            return cleanup(rc);
          HIPCHK(hipMemcpy(ctx->idx.p, idx.data(), 8 * (size_t)n, hipMemcpyHostToDevice));
          ctx->iota_n = -1;
          launch_interval_filter(ctx->U.as<uint8_t>(), ctx->rec_lin.as<int64_t>(), ctx->soa(),
                                 ctx->idx.as<int64_t>(), n, ctx->iv_ref.as<int32_t>(),
                                 ctx->iv_start.as<int32_t>(), ctx->iv_end.as<int32_t>(),
                                 ctx->iv_begin.as<int32_t>(), ctx->n_ref, ctx->keep.as<uint8_t>(),
                                 ctx->s);
          std::vector<uint8_t> keep((size_t)n);
          HIPCHK(hipMemcpyAsync(keep.data(), ctx->keep.p, (size_t)n, hipMemcpyDeviceToHost, ctx->s));
          HIPCHK(hipStreamSynchronize(ctx->s));
          for (int64_t k = 0; k < n; k++)
            if (keep[(size_t)k]) kept.push_back(idx[(size_t)k]);
        }
        dq_batch* b = nullptr;
        if ((rc = make_batch(ctx, {}, &kept, part_mode, {0, (int64_t)kept.size()}, &b))) return cleanup(rc);
        parts.push_back(b);
      }
      i = j;
    }
  }
  // the unplaced-unmapped tail (AbstractBinarySamSource.java:116-129; queryUnmapped,
  // H/BAMFileReader2.java:715-738): from the .bai's start of the last linear bin to EOF, the
  // records from the first one with refID -1 on
  if (tr->traverse_unplaced_unmapped && ctx->solb != -1 && ctx->ncc >= 1 &&
      vstart <= (uint64_t)ctx->solb && (uint64_t)ctx->solb < vend) {
    bool any = false;
    if ((rc = chunk_run(ctx, f.fd, flen, (uint64_t)ctx->solb, ((uint64_t)flen << 16) | 0xffff, &any)))
      return cleanup(rc);
    if (any) {
      const PartRange r = ctx->parts_h[0];
      std::vector<int32_t> refs((size_t)(r.end - r.begin));
      if (!refs.empty())
        HIPCHK(hipMemcpy(refs.data(), ctx->f_ref.as<int32_t>() + r.begin, 4 * refs.size(),
                         hipMemcpyDeviceToHost));
      size_t k = 0;
      while (k < refs.size() && refs[k] != -1) k++;
      dq_batch* b = nullptr;
      if ((rc = make_batch(ctx, {{r.begin + (int64_t)k, r.end}}, nullptr, part_mode,
                           {0, r.end - r.begin - (int64_t)k}, &b)))
        return cleanup(rc);
      parts.push_back(b);
    }
  }
  dq_batch* all = nullptr;
  if ((rc = concat_batches(ctx, parts, with_raw == DQ_EXPORT_LEAN, &all))) return cleanup(rc);
  cleanup(0);
  *out = all;
  return 0;
}

int dq_get_stats(dq_ctx* ctx, dq_stats* stats) {
  if (!ctx || !stats) return DQ_EINVAL;
  *stats = ctx->stats;
  return 0;
}

int dq_partition_digests(dq_ctx* ctx, int64_t* counts, uint64_t* digests, int64_t cap,
                         int64_t* n) {
  if (!ctx || !n) return DQ_EINVAL;
  if (!ctx->have_pipeline && !ctx->span_parts_valid)
    RET(DQ_EINVAL, "no pipeline run (call dq_run_resident first)");
  *n = (int64_t)ctx->parts_h.size();
  for (int64_t i = 0; i < std::min(cap, *n); i++) {
    const PartRange& r = ctx->parts_h[(size_t)i];
    if (counts) counts[i] = r.end - r.begin;
    if (digests) digests[i] = r.digest;
  }
  return 0;
}

// Whole-node mode in one process (SURVEY.md section 8(b) dq_decode_file_multi): the file's Disq
// partitions are cut into contiguous groups, one per device, by the byte range holding each split's
// first byte (even ranges: parallel.shard_plan); every device decodes its group from the file
// alone -- its split range plus a halo for the straddling record, grown x4 while too short -- on
// its own context and host thread.  No data crosses between devices: each reads its halo from the
// (page-cached) file.  The per-partition digests fold, in partition order, to the digest of a
// single-device run of the whole file.
int dq_decode_file_multi(dq_ctx* ctx, const char* path, const int32_t* devices, int32_t n_devices,
                         dq_multi_result* out) {
  if (!ctx || !path || !out || n_devices <= 0 || n_devices > 64) return DQ_EINVAL;
  ON_DEVICE(ctx);
  memset(out, 0, sizeof(*out));
  const auto t0 = std::chrono::steady_clock::now();
  int64_t flen = 0;
  int rc;
  {
    Fd f;
    if ((rc = open_fd(ctx, path, f, &flen))) return rc;
    if ((rc = chunk_header(ctx, path, f.fd, flen))) return rc;
  }
  std::vector<std::pair<int64_t, int64_t>> splits;
  if (path_splits(ctx->o, flen, splits)) RET(DQ_EINVAL, "splitSize must be > 0 with useNio");
  const int64_t P = (int64_t)splits.size();
  const int W = n_devices;
  std::vector<int64_t> O((size_t)W + 1);
  for (int r = 0; r < W; r++) O[(size_t)r] = (int64_t)(((__int128)r * flen + W - 1) / W);
  O[(size_t)W] = flen;
  struct Shard {
    int64_t p0 = 0, p1 = 0, lo = 0, hi = 0;
    int rc = 0;
    std::string err;
    std::vector<int64_t> counts;
    std::vector<uint64_t> digests;
    double ms_device = 0, ms_wall = 0;
    int64_t owned = 0;
  };
  std::vector<Shard> sh((size_t)W);
  for (int64_t p = 0; p < P; p++) {
    const int64_t st = splits[(size_t)p].first;
    int r = (int)(std::upper_bound(O.begin(), O.end(), st) - O.begin()) - 1;
    r = std::min(W - 1, std::max(0, r));
    Shard& s = sh[(size_t)r];
    if (s.p1 == s.p0) {
      s.p0 = p;
      s.lo = st;
    }
    s.p1 = p + 1;
    s.hi = splits[(size_t)p].second;
  }
  const std::vector<uint8_t> hdr = ctx->hdr;
  const std::string pth = path;
  auto work = [&](int r) {
    Shard& s = sh[(size_t)r];
    const auto w0 = std::chrono::steady_clock::now();
    dq_opts o = ctx->o;
    o.device = devices[r];
    dq_ctx* c = nullptr;
    if ((s.rc = dq_ctx_create(&c, &o))) {
      // dq_ctx_create hands back an allocated context on its error paths too: keep its message,
      // then free it
      s.err = "dq_ctx_create failed on device " + std::to_string(devices[r]) +
              (c ? std::string(": ") + dq_last_error(c) : std::string());
      if (c) dq_ctx_destroy(c);
      return;
    }
    int64_t halo = 4 << 20;
    for (;;) {
      const int64_t end = std::min(flen, s.hi + halo);
      dq_stats st;
      s.rc = dq_open_shard_path(c, pth.c_str(), s.lo, end - s.lo, s.p0, s.p1, hdr.data(),
                                (int64_t)hdr.size());
      if (!s.rc) s.rc = dq_run_resident(c, nullptr, &st);
      if (s.rc == DQ_EFORMAT && end < flen &&
          std::string(dq_last_error(c)).find("halo too small") != std::string::npos) {
        halo *= 4;
        continue;
      }
      if (!s.rc) {
        s.ms_device = st.ms_total;
        s.owned = st.owned_bytes;
      }
      break;
    }
    if (!s.rc) {
      const int64_t np = s.p1 - s.p0;
      s.counts.resize((size_t)np);
      s.digests.resize((size_t)np);
      int64_t n = 0;
      s.rc = dq_partition_digests(c, s.counts.data(), s.digests.data(), np, &n);
      if (!s.rc && n != np) {
        s.rc = DQ_EFORMAT;
        s.err = "shard partition count mismatch";
      }
    }
    if (s.rc && s.err.empty()) s.err = dq_last_error(c);
    dq_ctx_destroy(c);
    s.ms_wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
  };
  std::vector<std::thread> th;
  for (int r = 0; r < W; r++)
    if (sh[(size_t)r].p1 > sh[(size_t)r].p0) th.emplace_back(work, r);
  for (auto& x : th) x.join();
  uint64_t dg = 0;
  for (int r = 0; r < W; r++) {
    const Shard& s = sh[(size_t)r];
    if (s.p1 == s.p0) continue;
    if (s.rc) {
      ctx->err = "device " + std::to_string(devices[r]) + ": " + s.err;
      return s.rc;
    }
    for (int64_t k = 0; k < s.p1 - s.p0; k++) {
      const int64_t i = s.p0 + k;
      out->n_records += s.counts[(size_t)k];
      dg += dq_mix64(s.digests[(size_t)k] ^ ((uint64_t)(i + 1) * DQ_K_WORD));
    }
    out->ms_device_max = std::max(out->ms_device_max, s.ms_device);
    out->ms_shard_wall_max = std::max(out->ms_shard_wall_max, s.ms_wall);
    out->decompressed_bytes += s.owned;
  }
  // partitions owned by no shard (none: every split has an owner) would fold as empty
  out->n_devices = W;
  out->n_partitions = P;
  out->digest = dg;
  out->compressed_bytes = flen;
  out->ms_wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return 0;
}

int dq_header_from_prefix(dq_ctx* ctx, const uint8_t* bytes, int64_t len, uint8_t* out,
                          int64_t cap, int64_t* out_len) {
  if (!ctx || !bytes || len <= 0) return DQ_EINVAL;
  ON_DEVICE(ctx);
  int rc = dq_open_memory(ctx, bytes, len);
  if (rc) return rc;
  ctx->shard = true;  // the prefix is not the whole file: its end is not EOF
  ctx->file_len = INT64_MAX / 4;
  ctx->header_only = true;
  rc = run_pipeline(ctx);
  ctx->header_only = false;
  ctx->have_pipeline = false;
  ctx->have_file = false;  // the prefix is not a usable file
  if (rc) return rc;
  if (out_len) *out_len = ctx->header_bytes;
  if (out && cap > 0)
    HIPCHK(hipMemcpy(out, ctx->U.p, (size_t)std::min(cap, ctx->header_bytes), hipMemcpyDeviceToHost));
  return 0;
}

int dq_set_index(dq_ctx* ctx, const uint8_t* bai, int64_t len) {
  if (!ctx) return DQ_EINVAL;
  if (!bai) {
    ctx->have_bai = false;
    return 0;
  }
  Bai x;
  if (parse_bai(bai, len, x)) RET(DQ_EFORMAT, "invalid .bai");
  ctx->solb = x.solb;
  ctx->ncc = x.ncc;
  ctx->bai = std::move(x);
  ctx->have_bai = true;
  return 0;
}

int dq_set_splitting_index(dq_ctx* ctx, const uint8_t* sbi, int64_t len, int32_t use_for_planning) {
  if (!ctx) return DQ_EINVAL;
  ctx->have_pipeline = false;
  if (!sbi) {
    ctx->sbi.clear();
    ctx->sbi_plan = false;
    return 0;
  }
  // SBIIndex.readIndex / readHeader (M/htsjdk/samtools/SBIIndex.java:123-165)
  if (len < 68 || memcmp(sbi, "SBI\1", 4) != 0) RET(DQ_EFORMAT, "Invalid file header in SBI");
  const int64_t n = (int64_t)rd64(sbi + 60);
  if (n > INT32_MAX) RET(DQ_EFORMAT, "Cannot read SBI with more than 2147483647 offsets.");
  if (n < 1 || 68 + 8 * n > len) RET(DQ_EFORMAT, "truncated SBI");
  std::vector<uint64_t> v((size_t)n);
  for (int64_t i = 0; i < n; i++) {
    v[(size_t)i] = rd64(sbi + 68 + 8 * i);
    if (i && (int64_t)v[(size_t)i - 1] > (int64_t)v[(size_t)i]) RET(DQ_EFORMAT, "Invalid SBI; offsets not in order");
  }
  ctx->sbi.swap(v);
  ctx->sbi_plan = use_for_planning != 0;
  return 0;
}

int dq_write_sbi(dq_ctx* ctx, int64_t granularity, uint8_t** out, int64_t* out_len) {
  if (!ctx || !out || !out_len) return DQ_EINVAL;
  ON_DEVICE(ctx);
  if (granularity <= 0) granularity = 4096;  // SBIIndexWriter.DEFAULT_GRANULARITY
  if (ctx->shard) RET(DQ_EINVAL, "dq_write_sbi indexes a whole file, not a shard");
  ctx->have_pipeline = false;
  ctx->index_only = true;
  int rc = run_pipeline(ctx);
  ctx->index_only = false;
  ctx->have_pipeline = false;  // the next call re-plans with the caller's settings
  if (rc) return rc;
  const int64_t nrec = ctx->nrec, nent = (nrec + granularity - 1) / granularity;
  std::vector<uint64_t> ent((size_t)nent + 1);
  if (nent) {
    DevBuf d;
    HIPCHK(d.ensure(8 * (size_t)nent));
    launch_sbi_sample(ctx->f_voff.as<uint64_t>(), nrec, granularity, d.as<uint64_t>(), ctx->s);
    HIPCHK(hipMemcpyAsync(ent.data(), d.p, 8 * (size_t)nent, hipMemcpyDeviceToHost, ctx->s));
    HIPCHK(hipStreamSynchronize(ctx->s));
  }
  // finish(finalVirtualOffset): the file pointer after the last record (or after the header),
  // normalised as BlockCompressedInputStream.getFilePointer does: a consumed block points to the
  // next block's start (the EOF block, or the file end)
  int64_t E = ctx->header_bytes;
  if (nrec) {
    int64_t lin = 0;
    int32_t bs = 0;
    HIPCHK(hipMemcpy(&lin, ctx->rec_lin.as<int64_t>() + nrec - 1, 8, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&bs, ctx->f_bs.as<int32_t>() + nrec - 1, 4, hipMemcpyDeviceToHost));
    E = lin + 4 + (int64_t)bs;
  }
  std::vector<int64_t> uo((size_t)ctx->nblk + 1), bp((size_t)ctx->nblk);
  HIPCHK(hipMemcpy(uo.data(), ctx->uoff.p, 8 * uo.size(), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(bp.data(), ctx->blk_pos.p, 8 * bp.size(), hipMemcpyDeviceToHost));
  uint64_t fin = (uint64_t)ctx->flen << 16;
  if (E > 0) {
    const int64_t j = (int64_t)(std::upper_bound(uo.begin(), uo.end() - 1, E - 1) - uo.begin()) - 1;
    if (j >= 0 && E < uo[(size_t)j + 1]) fin = ((uint64_t)bp[(size_t)j] << 16) | (uint64_t)(E - uo[(size_t)j]);
    else if (j + 1 < ctx->nblk) fin = (uint64_t)bp[(size_t)j + 1] << 16;
  }
  ent[(size_t)nent] = fin;
  // SBIIndexWriter.finish (SBIIndexWriter.java:120-151): magic, file length, MD5, UUID, record
  // count, granularity, offset count, offsets (all little-endian)
  const int64_t n = 68 + 8 * (int64_t)ent.size();
  uint8_t* b = (uint8_t*)calloc((size_t)n, 1);
  if (!b) return DQ_ENOMEM;
  auto w64 = [&](int64_t at, uint64_t v) { memcpy(b + at, &v, 8); };
  memcpy(b, "SBI\1", 4);
  w64(4, (uint64_t)ctx->flen);
  w64(44, (uint64_t)nrec);
  w64(52, (uint64_t)granularity);
  w64(60, (uint64_t)ent.size());
  for (size_t i = 0; i < ent.size(); i++) w64(68 + 8 * (int64_t)i, ent[i]);
  *out = b;
  *out_len = n;
  return 0;
}

int dq_read_header(dq_ctx* ctx, dq_header_info* info, uint8_t* header_bytes, int64_t cap) {
  if (!ctx) return DQ_EINVAL;
  ON_DEVICE(ctx);
  int rc = run_pipeline(ctx);
  if (rc) return rc;
  if (info) {
    info->n_ref = ctx->n_ref;
    info->header_bytes = ctx->header_bytes;
    info->first_record_voffset = 0;
    if (ctx->nrec) {
      uint64_t v;
      HIPCHK(hipMemcpy(&v, ctx->f_voff.p, 8, hipMemcpyDeviceToHost));
      info->first_record_voffset = v + ((uint64_t)ctx->base << 16);
    }
  }
  if (header_bytes && cap > 0) {
    int64_t n = std::min(cap, ctx->header_bytes);
    if (ctx->shard) memcpy(header_bytes, ctx->hdr.data(), (size_t)n);
    else HIPCHK(hipMemcpy(header_bytes, ctx->U.p, (size_t)n, hipMemcpyDeviceToHost));
  }
  return 0;
}

int dq_plan(dq_ctx* ctx, dq_chunk** chunks, int64_t* n) {
  if (!ctx || !chunks || !n) return DQ_EINVAL;
  ON_DEVICE(ctx);
  int rc = run_pipeline(ctx);
  if (rc) return rc;
  *n = (int64_t)ctx->plans_h.size();
  dq_chunk* c = (dq_chunk*)calloc((size_t)std::max<int64_t>(1, *n), sizeof(dq_chunk));
  for (int64_t i = 0; i < *n; i++) {
    const SplitPlan& P = ctx->plans_h[(size_t)i];
    const uint64_t vb = (uint64_t)ctx->base << 16;  // shard coordinates -> file coordinates
    c[i].split_start = P.split_start + ctx->base;
    c[i].split_end = P.split_end + ctx->base;
    c[i].has_chunk = P.rec_lin >= 0;
    c[i].vstart = P.rec_lin >= 0 ? P.vstart + vb : 0;
    c[i].vend = P.vend + vb;
  }
  *chunks = c;
  return 0;
}

int dq_decode(dq_ctx* ctx, uint64_t vstart, uint64_t vend, int32_t with_raw, dq_batch** out) {
  if (!ctx || !out) return DQ_EINVAL;
  ON_DEVICE(ctx);
  int rc = run_pipeline(ctx);
  if (rc) return rc;
  int64_t b, e;
  if ((rc = chunk_range(ctx, vstart, vend, &b, &e))) return rc;
  return make_batch(ctx, {{b, e}}, nullptr, with_raw, {0, e - b}, out);
}

int dq_decode_filtered(dq_ctx* ctx, uint64_t vstart, uint64_t vend, const dq_traversal* tr,
                       int32_t with_raw, dq_batch** out) {
  if (!ctx || !out || !tr) return DQ_EINVAL;
  ON_DEVICE(ctx);
  if (!tr->has_intervals && !tr->traverse_unplaced_unmapped)
    RET(DQ_EINVAL, "Traversing mapped reads only is not supported.");
  if (int rc0 = check_tail_reachable(ctx, tr)) return rc0;
  int rc = run_pipeline(ctx);
  if (rc) return rc;
  int64_t b, e;
  if ((rc = chunk_range(ctx, vstart, vend, &b, &e))) return rc;
  const uint64_t vb = (uint64_t)ctx->base << 16;
  std::vector<int64_t> idx;
  if ((rc = filtered_indices(ctx, vstart >= vb ? vstart - vb : 0, vend >= vb ? vend - vb : 0, b, e,
                             tr, idx)))
    return rc;
  return make_batch(ctx, {}, &idx, with_raw, {0, (int64_t)idx.size()}, out);
}

int dq_read(dq_ctx* ctx, const dq_traversal* tr, int32_t with_raw, dq_batch** out) {
  if (!ctx || !out) return DQ_EINVAL;
  ON_DEVICE(ctx);
  if (tr && !tr->has_intervals && !tr->traverse_unplaced_unmapped)
    RET(DQ_EINVAL, "Traversing mapped reads only is not supported.");
  if (int rc0 = check_tail_reachable(ctx, tr)) return rc0;
  int rc = run_pipeline(ctx);
  if (rc) return rc;
  std::vector<int64_t> idx, bounds{0};
  std::vector<std::pair<int64_t, int64_t>> ranges;
  int64_t total = 0;
  for (size_t i = 0; i < ctx->plans_h.size(); i++) {
    const SplitPlan& P = ctx->plans_h[i];
    if (P.rec_lin < 0) continue;  // empty partition (no PathChunk)
    const PartRange& r = ctx->parts_h[i];
    if (!tr) {
      ranges.push_back({r.begin, r.end});
      total += r.end - r.begin;
    } else {
      std::vector<int64_t> f;
      if ((rc = filtered_indices(ctx, P.vstart, P.vend, r.begin, r.end, tr, f))) return rc;
      idx.insert(idx.end(), f.begin(), f.end());
      total = (int64_t)idx.size();
    }
    bounds.push_back(total);
  }
  if (!tr) {
    // a single range is copied straight from the resident arrays (ranges.size() <= 1)
    return make_batch(ctx, ranges, nullptr, with_raw, bounds, out);
  }
  return make_batch(ctx, {}, &idx, with_raw, bounds, out);
}

int dq_run_resident(dq_ctx* ctx, const dq_traversal* tr, dq_stats* stats) {
  if (!ctx) return DQ_EINVAL;
  ON_DEVICE(ctx);
  if (tr && !tr->has_intervals && !tr->traverse_unplaced_unmapped)
    RET(DQ_EINVAL, "Traversing mapped reads only is not supported.");
  if (int rc0 = check_tail_reachable(ctx, tr)) return rc0;
  int rc;
  if (tr && tr->has_intervals && tr->n > 0 && ctx->have_bai && !ctx->o.full_traversal &&
      !ctx->chunk_mode) {
    // .bai span run: only the spans' blocks are inflated; the partition plans come from a full
    // run of the open file (made once here if there is none yet)
    if (!ctx->plan_cached) {
      ctx->have_pipeline = false;
      if ((rc = run_pipeline(ctx))) return rc;
    }
    dq_stats S{};
    if ((rc = run_span(ctx, tr, &S))) return rc;
    if (stats) *stats = S;
    return 0;
  }
  ctx->have_pipeline = false;
  rc = run_pipeline(ctx);
  if (rc) return rc;
  dq_stats S = ctx->stats;
  S.n_filtered = -1;
  if (tr && tr->has_intervals && tr->n > 0 && ctx->nrec > 0) {
    // Kernel 4 over every record of the resident stream (the interval filter of all partitions
    // at once; the unplaced-unmapped tail is a host-side pointer range and is not timed here)
    if (!ctx->have_bai) RET(DQ_EINVAL, "Intervals set but no index file found");
    if ((rc = upload_intervals(ctx, tr))) return rc;
    const int64_t n = ctx->nrec;
    if (ctx->iota_n != n) {
      std::vector<int64_t> idx((size_t)n);
      for (int64_t k = 0; k < n; k++) idx[(size_t)k] = k;
      if ((rc = ensure_all(ctx, ctx->idx, 8 * (size_t)n)) || (rc = ensure_all(ctx, ctx->keep, (size_t)n)))
        return rc;
      HIPCHK(hipMemcpy(ctx->idx.p, idx.data(), 8 * (size_t)n, hipMemcpyHostToDevice));
      ctx->iota_n = n;
    }
    HIPCHK(hipEventRecord(ctx->ev[6], ctx->s));
    launch_interval_filter(ctx->U.as<uint8_t>(), ctx->rec_lin.as<int64_t>(), ctx->soa(),
                           ctx->idx.as<int64_t>(), n, ctx->iv_ref.as<int32_t>(),
                           ctx->iv_start.as<int32_t>(), ctx->iv_end.as<int32_t>(),
                           ctx->iv_begin.as<int32_t>(), ctx->n_ref, ctx->keep.as<uint8_t>(), ctx->s);
    HIPCHK(hipEventRecord(ctx->ev[7], ctx->s));
    HIPCHK(hipEventSynchronize(ctx->ev[7]));
    S.ms_filter = ev_ms(ctx->ev[6], ctx->ev[7]);
    std::vector<uint8_t> keep((size_t)n);
    HIPCHK(hipMemcpy(keep.data(), ctx->keep.p, (size_t)n, hipMemcpyDeviceToHost));
    int64_t kept = 0;
    for (int64_t k = 0; k < n; k++) kept += keep[(size_t)k] != 0;
    S.n_filtered = kept;
  }
  if (stats) *stats = S;
  return 0;
}

int dq_debug_inflated(dq_ctx* ctx, uint8_t* host_out, int64_t cap, int64_t* len) {
  if (!ctx) return DQ_EINVAL;
  ON_DEVICE(ctx);
  int rc = run_pipeline(ctx);
  if (rc) return rc;
  if (len) *len = ctx->ulen;
  if (host_out && cap > 0)
    HIPCHK(hipMemcpy(host_out, ctx->U.p, (size_t)std::min(cap, ctx->ulen), hipMemcpyDeviceToHost));
  return 0;
}

int dq_debug_guess_all(dq_ctx* ctx, uint64_t* voffs, int64_t cap, int64_t* n) {
  if (!ctx || !n) return DQ_EINVAL;
  ON_DEVICE(ctx);
  if (ctx->shard || ctx->chunk_mode) RET(DQ_EINVAL, "dq_debug_guess_all checks a whole resident file");
  int rc = run_pipeline(ctx);
  if (rc) return rc;
  const int64_t ulen = ctx->ulen;
  DevBuf d;
  HIPCHK(d.ensure((size_t)std::max<int64_t>(ulen, 1)));
  launch_guess_all(ctx->U.as<uint8_t>(), ulen, 1, ctx->d_ref_len.as<int32_t>(), ctx->n_ref,
                   d.as<uint8_t>(), ctx->s);
  HIPCHK(hipGetLastError());
  std::vector<uint8_t> f((size_t)ulen);
  std::vector<int64_t> uo((size_t)ctx->nblk + 1), bp((size_t)ctx->nblk);
  HIPCHK(hipMemcpyAsync(f.data(), d.p, (size_t)ulen, hipMemcpyDeviceToHost, ctx->s));
  HIPCHK(hipMemcpyAsync(uo.data(), ctx->uoff.p, 8 * uo.size(), hipMemcpyDeviceToHost, ctx->s));
  HIPCHK(hipMemcpyAsync(bp.data(), ctx->blk_pos.p, 8 * bp.size(), hipMemcpyDeviceToHost, ctx->s));
  HIPCHK(hipStreamSynchronize(ctx->s));
  int64_t k = 0;
  size_t j = 0;
  for (int64_t x = 0; x < ulen; x++) {
    if (f[(size_t)x] == 4) RET(DQ_EFORMAT, "guesser needed data past the end of a whole file");
    if (f[(size_t)x] != 1) continue;
    while (j + 1 < bp.size() && uo[j + 1] <= x) j++;
    if (k < cap && voffs) voffs[k] = ((uint64_t)bp[j] << 16) | (uint64_t)(x - uo[j]);
    k++;
  }
  *n = k;
  return 0;
}

int dq_text_set_index(dq_ctx* ctx, const uint8_t* tbi, int64_t len) {
  if (!ctx) return DQ_EINVAL;
  ctx->have_text = false;
  if (!tbi) {
    ctx->have_tbi = false;
    return 0;
  }
  Bai x;
  std::vector<std::string> names;
  if (parse_tbi(tbi, len, x, names)) RET(DQ_EFORMAT, "invalid tabix index (expects the decompressed .tbi bytes)");
  ctx->tbi = std::move(x);
  ctx->tbi_names = std::move(names);
  ctx->have_tbi = true;
  return 0;
}

int dq_text_set_intervals(dq_ctx* ctx, const char* const* contig, const int32_t* start,
                          const int32_t* end, int64_t n) {
  if (!ctx) return DQ_EINVAL;
  ON_DEVICE(ctx);
  ctx->have_text = false;
  ctx->tiv_contig.clear();
  ctx->tiv_cid.clear();
  ctx->tiv_start.clear();
  ctx->tiv_end.clear();
  if (!contig || n < 0) {
    ctx->text_iv = false;
    return 0;
  }
  if (n > 0 && (!start || !end)) return DQ_EINVAL;
  for (int64_t i = 0; i < n; i++) {
    if (!contig[i]) RET(DQ_EINVAL, "interval may not be null");
    const std::string c(contig[i]);
    auto it = std::find(ctx->tiv_contig.begin(), ctx->tiv_contig.end(), c);
    int32_t id = (int32_t)(it - ctx->tiv_contig.begin());
    if (it == ctx->tiv_contig.end()) ctx->tiv_contig.push_back(c);
    ctx->tiv_cid.push_back(id);
    ctx->tiv_start.push_back(start[i]);
    ctx->tiv_end.push_back(end[i]);
  }
  // device form: intervals grouped by contig, sorted by start, with running maximum ends
  const int32_t nc = (int32_t)ctx->tiv_contig.size();
  std::vector<int32_t> beg((size_t)nc + 1, 0), st, en, mx, noff((size_t)nc + 1, 0);
  std::string names;
  for (int32_t c = 0; c < nc; c++) {
    std::vector<std::pair<int32_t, int32_t>> v;
    for (size_t i = 0; i < ctx->tiv_cid.size(); i++)
      if (ctx->tiv_cid[i] == c) v.push_back({ctx->tiv_start[i], ctx->tiv_end[i]});
    std::sort(v.begin(), v.end());
    int32_t m = INT32_MIN;
    for (const auto& x : v) {
      st.push_back(x.first);
      en.push_back(x.second);
      m = std::max(m, x.second);
      mx.push_back(m);
    }
    beg[(size_t)c + 1] = (int32_t)st.size();
    names += ctx->tiv_contig[(size_t)c];
    noff[(size_t)c + 1] = (int32_t)names.size();
  }
  int rc;
  const size_t ni = std::max<size_t>(1, st.size());
  if ((rc = ensure_all(ctx, ctx->t_ivnames, std::max<size_t>(1, names.size()))) ||
      (rc = ensure_all(ctx, ctx->t_ivnoff, 4 * noff.size())) ||
      (rc = ensure_all(ctx, ctx->t_ivbeg, 4 * beg.size())) ||
      (rc = ensure_all(ctx, ctx->t_ivstart, 4 * ni)) || (rc = ensure_all(ctx, ctx->t_ivend, 4 * ni)) ||
      (rc = ensure_all(ctx, ctx->t_ivmaxend, 4 * ni)))
    return rc;
  if (!names.empty()) HIPCHK(hipMemcpy(ctx->t_ivnames.p, names.data(), names.size(), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(ctx->t_ivnoff.p, noff.data(), 4 * noff.size(), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(ctx->t_ivbeg.p, beg.data(), 4 * beg.size(), hipMemcpyHostToDevice));
  if (!st.empty()) {
    HIPCHK(hipMemcpy(ctx->t_ivstart.p, st.data(), 4 * st.size(), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(ctx->t_ivend.p, en.data(), 4 * en.size(), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(ctx->t_ivmaxend.p, mx.data(), 4 * mx.size(), hipMemcpyHostToDevice));
  }
  ctx->text_iv = true;
  return 0;
}

int dq_text_open_memory(dq_ctx* ctx, const uint8_t* bytes, int64_t len) {
  int rc = dq_open_memory(ctx, bytes, len);
  if (rc == 0) ctx->text_mode = true;
  return rc;
}

int dq_text_open_path(dq_ctx* ctx, const char* path) {
  int rc = dq_open_path(ctx, path);
  if (rc == 0) ctx->text_mode = true;
  return rc;
}

int dq_text_run(dq_ctx* ctx, int32_t drop_header_lines, dq_stats* stats) {
  if (!ctx) return DQ_EINVAL;
  ON_DEVICE(ctx);
  // a re-run times the whole pipeline again
  ctx->have_pipeline = false;
  ctx->have_text = false;
  int rc = text_run(ctx, drop_header_lines ? 1 : 0);
  if (rc) return rc;
  if (stats) *stats = ctx->stats;
  return 0;
}

int dq_text_read(dq_ctx* ctx, int32_t drop_header_lines, dq_text_batch** out) {
  if (!ctx || !out) return DQ_EINVAL;
  ON_DEVICE(ctx);
  *out = nullptr;
  int rc = text_run(ctx, drop_header_lines ? 1 : 0);
  if (rc) return rc;
  hipStream_t s = ctx->s;
  const int64_t n = ctx->t_nkept, nsplit = (int64_t)ctx->tplans_h.size();
  const size_t n1 = (size_t)std::max<int64_t>(1, n);
  DevBuf o_start, o_len, o_hash, o_off, o_data, tmp;
  HIPCHK(o_start.ensure(8 * n1));
  HIPCHK(o_len.ensure(4 * n1));
  HIPCHK(o_hash.ensure(8 * n1));
  HIPCHK(o_off.ensure(8 * (n1 + 1)));
  HIPCHK(tmp.ensure(sizeof(int64_t) * (size_t)(4 * ((int64_t)n1 / 1024 + 1) + 4096)));
  launch_text_export(ctx->t_kept.as<int64_t>(), n, ctx->t_vs.as<int64_t>(), ctx->t_vl.as<int32_t>(),
                     ctx->t_hash.as<uint64_t>(), o_start.as<int64_t>(), o_len.as<int32_t>(),
                     o_hash.as<uint64_t>(), s);
  if (n > 0) launch_exclusive_scan_i32(o_len.as<int32_t>(), o_off.as<int64_t>(), n, tmp.as<int64_t>(), s);
  int64_t nbytes = 0;
  if (n > 0 && (rc = get_i64(ctx, o_off.as<int64_t>() + n, &nbytes))) return rc;
  HIPCHK(o_data.ensure((size_t)std::max<int64_t>(1, nbytes)));
  launch_text_gather(ctx->U.as<uint8_t>(), ctx->t_vs.as<int64_t>(), ctx->t_vl.as<int32_t>(),
                     ctx->t_kept.as<int64_t>(), o_off.as<int64_t>(), n, o_data.as<uint8_t>(), s);
  dq_text_batch* b = (dq_text_batch*)calloc(1, sizeof(dq_text_batch));
  if (!b) return DQ_ENOMEM;
  b->n_lines = n;
  b->n_partitions = nsplit;
  b->line_offset = (int64_t*)malloc(8 * n1);
  b->line_len = (int32_t*)malloc(4 * n1);
  b->hash = (uint64_t*)malloc(8 * n1);
  b->data_offset = (int64_t*)malloc(8 * (n1 + 1));
  b->data = (uint8_t*)malloc((size_t)std::max<int64_t>(1, nbytes));
  b->part_offset = (int64_t*)malloc(8 * (size_t)(nsplit + 1));
  b->part_digest = (uint64_t*)malloc(8 * (size_t)std::max<int64_t>(1, nsplit));
  if (!b->line_offset || !b->line_len || !b->hash || !b->data_offset || !b->data || !b->part_offset ||
      !b->part_digest) {
    dq_text_batch_free(b);
    return DQ_ENOMEM;
  }
  if (n > 0) {
    HIPCHK(hipMemcpyAsync(b->line_offset, o_start.p, 8 * (size_t)n, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(b->line_len, o_len.p, 4 * (size_t)n, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(b->hash, o_hash.p, 8 * (size_t)n, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(b->data_offset, o_off.p, 8 * (size_t)(n + 1), hipMemcpyDeviceToHost, s));
  } else {
    b->data_offset[0] = 0;
  }
  if (nbytes > 0) HIPCHK(hipMemcpyAsync(b->data, o_data.p, (size_t)nbytes, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  b->n_bytes = nbytes;
  for (int64_t i = 0; i < nsplit; i++) {
    b->part_offset[i] = ctx->parts_h[(size_t)i].begin;
    b->part_digest[i] = ctx->parts_h[(size_t)i].digest;
  }
  b->part_offset[nsplit] = n;
  *out = b;
  return 0;
}

void dq_text_batch_free(dq_text_batch* b) {
  if (!b) return;
  free(b->line_offset);
  free(b->line_len);
  free(b->hash);
  free(b->data_offset);
  free(b->data);
  free(b->part_offset);
  free(b->part_digest);
  free(b);
}

int dq_bgzf_compress(dq_ctx* ctx, const uint8_t* data, int64_t len, uint8_t** out, int64_t* out_len) {
  if (!ctx || !out || !out_len || len < 0 || (!data && len > 0)) return DQ_EINVAL;
  ON_DEVICE(ctx);
  *out = nullptr;
  *out_len = 0;
  int rc;
  if ((rc = ensure_all(ctx, ctx->z_in, (size_t)len + 64))) return rc;
  if (len) HIPCHK(hipMemcpy(ctx->z_in.p, data, (size_t)len, hipMemcpyHostToDevice));
  double ms = 0;
  if ((rc = bgzf_compress_dev(ctx, ctx->z_in.as<uint8_t>(), len, &ms))) return rc;
  uint8_t* b = (uint8_t*)malloc((size_t)std::max<int64_t>(1, ctx->z_len));
  if (!b) return DQ_ENOMEM;
  if (ctx->z_len) HIPCHK(hipMemcpy(b, ctx->z_out.p, (size_t)ctx->z_len, hipMemcpyDeviceToHost));
  *out = b;
  *out_len = ctx->z_len;
  return 0;
}

int dq_bgzf_compress_resident(dq_ctx* ctx, int64_t* out_len, double* ms) {
  if (!ctx) return DQ_EINVAL;
  ON_DEVICE(ctx);
  int rc = ctx->text_mode ? text_run(ctx, ctx->text_drop < 0 ? 1 : ctx->text_drop) : run_pipeline(ctx);
  if (rc) return rc;
  double t = 0;
  if ((rc = bgzf_compress_dev(ctx, ctx->U.as<uint8_t>(), ctx->ulen, &t))) return rc;
  if (out_len) *out_len = ctx->z_len;
  if (ms) *ms = t;
  return 0;
}

int dq_bgzf_fetch(dq_ctx* ctx, uint8_t* host_out, int64_t cap) {
  if (!ctx || (!host_out && cap > 0)) return DQ_EINVAL;
  ON_DEVICE(ctx);
  if (cap < ctx->z_len) RET(DQ_EINVAL, "buffer smaller than the compressed stream");
  if (ctx->z_len) HIPCHK(hipMemcpy(host_out, ctx->z_out.p, (size_t)ctx->z_len, hipMemcpyDeviceToHost));
  return 0;
}

int dq_set_export_arena(dq_ctx* ctx, int64_t bytes) {
  if (!ctx || bytes < 0) return DQ_EINVAL;
  ON_DEVICE(ctx);
  if (!ctx->ah) ctx->ah = new ArenaHold();
  {
    std::lock_guard<std::mutex> lk(ctx->ah->mu);
    if (ctx->ah->live)
      RET(DQ_EINVAL, "the export arena still holds a batch: dq_batch_free it before resizing the arena");
  }
  if (ctx->s) HIPCHK(hipStreamSynchronize(ctx->s));
  if (ctx->sx) HIPCHK(hipStreamSynchronize(ctx->sx));
  if (ctx->arena) (void)hipHostFree(ctx->arena);
  ctx->arena = ctx->ah->arena = nullptr;
  ctx->arena_cap = 0;
  if (bytes == 0) return 0;
  HIPCHK(hipHostMalloc((void**)&ctx->arena, (size_t)bytes, hipHostMallocDefault));
  ctx->ah->arena = ctx->arena;
  ctx->arena_cap = (size_t)bytes;
  return ensure_pinned(ctx);  // the upload staging too: every long-lived host buffer up front
}

void dq_batch_free(dq_batch* b) {
  if (!b) return;
  if (b->in_arena) {  // the arrays live in the context's export arena: give it back
    if (ArenaHold* h = static_cast<ArenaHold*>(b->arena_hold)) {
      bool last;
      {
        std::lock_guard<std::mutex> lk(h->mu);
        h->live = false;
        last = h->orphan;
      }
      if (last) {  // the context is gone: this batch owned the arena
        if (h->arena) (void)hipHostFree(h->arena);
        delete h;
      }
    }
    free(b->part_offset);
    free(b->part_digest);
    free(b);
    return;
  }
  free(b->voffset);
  free(b->block_size);
  free(b->ref_id);
  free(b->pos);
  free(b->l_seq);
  free(b->next_ref_id);
  free(b->next_pos);
  free(b->tlen);
  free(b->flag);
  free(b->bin);
  free(b->n_cigar);
  free(b->mapq);
  free(b->l_read_name);
  free(b->hash);
  free(b->raw_offset);
  free(b->raw);
  free(b->part_offset);
  free(b->part_digest);
  free(b);
}

void dq_free(void* p) { free(p); }

int dq_checked_report(uint64_t words[4]) {
  if (!words) return DQ_EINVAL;
  words[0] = dq::dq_chk_take_kernels();
  words[1] = dq::dq_chk_take_inflate();
  words[2] = dq::dq_chk_take_text();
  words[3] = dq::dq_chk_take_deflate();
#ifdef DQ_CHECKED
  return 1;
#else
  return 0;
#endif
}

}  // extern "C"
