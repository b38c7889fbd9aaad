// dq_internal.h -- shared device helpers and kernel launch wrappers of libdisq_gpu.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// ------------------------------------------------------------------ status codes (per block/record)
enum : int32_t {
  ST_OK = 0,
  ST_BAD_HEADER = 1,      // BGZF header: not 1f 8b 08 04 / XLEN != 6 (htsjdk BlockGunzipper)
  ST_BAD_BLOCKTYPE = 2,
  ST_BAD_STORED = 3,
  ST_BAD_TABLE = 4,       // over-subscribed / incomplete Huffman code, bad header counts
  ST_BAD_CODE = 5,        // invalid literal/length/distance code
  ST_BAD_DIST = 6,        // distance too far back
  ST_SHORT = 7,           // "Did not inflate expected amount"
  ST_OVERREAD = 8,        // read past the block's deflate data
  ST_CRC = 9,             // CRC32 mismatch (verify_crc)
  ST_ISIZE = 10,          // ISIZE > 65536
  ST_HANG = 11,           // internal: batch loop made no progress
  ST_TEXT_START = 12,     // text split: no block start in the split and none at its end
};

// ------------------------------------------------------------------ DQ_CHECKED
// The device bounds-checked build (`make -C disq_amd/csrc checked` -> libdisq_gpu_checked.so, picked
// up through DQ_GPU_LIB): DQ_CHK(cond, site) counts a failed check and sets bit `site` in this
// translation unit's check words; the access itself goes ahead unchanged (the checks observe the
// kernels, they do not alter them, and nothing traps: a trap would take the GPU down with it).
// dq_checked_report (dq_api.hip) collects every unit's words after a run.  In the product build
// DQ_CHK compiles to nothing.
enum : int {
  CHK_K1_SLOT = 0,   // K1: a candidate's slot outside its chunk's CAP slots
  CHK_K2_BITS = 1,   // K2: the bit reader loads a word past the member's deflate data (+ slack)
  CHK_K2_IMAGE = 2,  // K2: an emit / stored-copy store outside the LDS output image
  CHK_K2_TABLE = 3,  // K2: a second-level table read outside its alphabet's area
  CHK_K2_LANES = 4,  // K2: per-lane arrays / redo list outside the image tail
  CHK_K2_BM = 5,     // K2: a match-start bitmap word outside the bitmap
  CHK_K2_NXT = 6,    // K2: a resolve next pointer outside the batch window
  CHK_K2_SRC = 7,    // K2: a resolve copy source outside [0, isize)
  CHK_K3_STAGE = 8,  // K3: a record's staged bytes (or their reads) outside the LDS staging
  CHK_K2_LAST = 9,   // K2: a last_start index outside the table
  CHK_Z_BL = 10,     // deflate: a bucket-list slot outside the chunk's position list
  CHK_Z_STAGE = 11,  // deflate: a staged symbol word outside its lane's staging
  CHK_Z_IMAGE = 12,  // deflate: an emitted word outside the LDS deflate image
  CHK_K3_SPEC = 13,  // K3: the LDS-filtered segment speculation differs from seg_spec_kernel<64>
};
#ifdef DQ_CHECKED
namespace {
// failed checks, OR of their site bits, the largest excess a failed check reported (this unit)
__device__ unsigned int g_dq_chk[3];
}
#define DQ_CHKV(cond, site, excess)                              \
  do {                                                           \
    if (__builtin_expect(!(cond), 0)) {                          \
      atomicAdd(&g_dq_chk[0], 1u);                               \
      atomicOr(&g_dq_chk[1], 1u << (site));                      \
      atomicMax(&g_dq_chk[2], (unsigned int)(excess));           \
    }                                                            \
  } while (0)
#define DQ_CHK(cond, site) DQ_CHKV(cond, site, 0)
// Host: this unit's words (count << 32 | excess << 16 | site bits), reset; the current device.
#define DQ_CHK_UNIT(name)                                                              \
  uint64_t dq_chk_take_##name() {                                                      \
    unsigned int w[3] = {0, 0, 0}, z[3] = {0, 0, 0};                                   \
    if (hipMemcpyFromSymbol(w, HIP_SYMBOL(g_dq_chk), sizeof w) != hipSuccess) return ~0ull; \
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_dq_chk), z, sizeof z);                        \
    return (uint64_t)w[0] << 32 | (uint64_t)(w[2] & 0xffff) << 16 | (w[1] & 0xffff); \
  }
#else
#define DQ_CHKV(cond, site, excess) ((void)0)
#define DQ_CHK(cond, site) ((void)0)
#define DQ_CHK_UNIT(name) \
  uint64_t dq_chk_take_##name() { return 0; }
#endif

// ------------------------------------------------------------------ hashing
__host__ __device__ inline uint64_t dq_mix64(uint64_t z) {
  z ^= z >> 30;
  z *= 0xBF58476D1CE4E5B9ULL;
  z ^= z >> 27;
  z *= 0x94D049BB133111EBULL;
  z ^= z >> 31;
  return z;
}
#define DQ_K_LEN 0x9E3779B97F4A7C15ULL
#define DQ_K_WORD 0xD6E8FEB86659FD93ULL

// ------------------------------------------------------------------ launch wrappers
// All pointers are device pointers; all launches go on `s`.
namespace dq {

struct Cand {          // a BgzfBlockGuesser-visible magic position
  int64_t pos;
  int32_t csize;       // guesser cSize (BSIZE + 1 via the BC subfield)
  int32_t usize;       // ISIZE
  int32_t valid;       // 1 = guessNextBGZFPos would return this block; 0 = magic only
  int32_t pad;
};

constexpr int SCAN_CHUNK = 16384;  // bytes of C per scan workgroup
constexpr int SCAN_CAP = 32;       // candidate slots per chunk in the first scan pass
constexpr int SCAN_CAP_BIG = 640;  // slots of a re-scanned chunk (BGZF members are >= 28 bytes)
constexpr int SCAN_OVER_MAX = 1 << 22;  // chunks the second pass can take

// Kernel 1: BGZF candidate scan of C[0, n) (file offsets; L = readable bytes).  Writes each
// chunk's candidates sorted into slots[chunk * SCAN_CAP ...] and its count.
void launch_bgzf_scan(const uint8_t* C, int64_t n, int64_t L, Cand* slots, int64_t cap,
                      int32_t* chunk_counts, int64_t n_chunks, int64_t* d_count,
                      int32_t* over_list, hipStream_t s);
// Second pass over the chunks listed in over_list[1..over_list[0]] (more than SCAN_CAP hits).
void launch_bgzf_scan_listed(const uint8_t* C, int64_t n, int64_t L, Cand* big, int64_t n_over,
                             int32_t* chunk_counts, int32_t* over_list, int32_t* over_map,
                             hipStream_t s);
void launch_gather_slots(const Cand* slots, const int32_t* counts, const int64_t* offs,
                         int64_t nchunks, Cand* out, int64_t cap, const int32_t* over_map,
                         const Cand* big, hipStream_t s);
void launch_valid_flags(const Cand* cand, const int64_t* ncand, int64_t cap, int32_t* flags,
                        hipStream_t s);
// Chain check: valid candidates must be htsjdk blocks linked by pos + BSIZE + 1.
void launch_chain2(const uint8_t* C, int64_t L, const Cand* cand, const int64_t* ncand, int64_t cap,
                   const int64_t* voff, int64_t* blk_pos, int32_t* blk_csize, int32_t* blk_usize,
                   int64_t blk_cap, int64_t* d_nblk, int32_t* d_broken, int32_t eof_in_buf,
                   hipStream_t s);
// out[0] = min pos of the valid candidates (out initialised to all ones), out[1] = blk_pos[0].
void launch_chain_check(const Cand* cand, const int64_t* d_ncand, int64_t cap, const int64_t* blk_pos,
                        const int64_t* d_nblk, unsigned long long* out, hipStream_t s);
// out[0] = the first block index (through sel when given) whose status is not ST_OK.
void launch_first_bad(const int32_t* status, const int32_t* sel, int64_t n, unsigned long long* out,
                      hipStream_t s);
// Serial fallback chain walk (one lane) over htsjdk headers from `start`.
void launch_chain_serial(const uint8_t* C, int64_t clen, int64_t start, int64_t* blk_pos,
                         int32_t* blk_csize, int32_t* blk_usize, int64_t cap, int64_t* d_nblk,
                         int32_t* d_status, hipStream_t s);

// Exclusive prefix sums; out has n + 1 entries (out[n] = total).  tmp >= 4*ceil(n/1024)+256.
void launch_exclusive_scan_i32(const int32_t* in, int64_t* out, int64_t n, int64_t* tmp,
                               hipStream_t s);
void launch_exclusive_scan_i64(const int64_t* in, int64_t* out, int64_t n, int64_t* tmp,
                               hipStream_t s);

// Kernel 2: fused inflate + CRC32, one workgroup per block (dq_inflate3.hip).  The CRC tables
// live in each device's memory: inflate3_tables(device) initialises them once per device (thread
// safe) and returns that device's table of x^(8n) * ~0 mod P, n = 0..65536 (nullptr on failure).
const uint32_t* inflate3_tables(int device);
// tails: 16 bytes of device scratch per launched block (the tail kernel's descriptors; nullptr:
// the block kernel decodes every deflate block itself)
constexpr size_t INFLATE_TAIL_BYTES = 16;
void launch_inflate3(const uint8_t* C, const int64_t* blk_pos, const int32_t* blk_csize,
                     const int32_t* blk_usize, const int64_t* uoff, int64_t nblk, uint8_t* U,
                     int32_t* status, int32_t verify_crc, const uint32_t* crc_init, uint64_t* tim,
                     hipStream_t s, const int32_t* sel, int64_t nsel, void* tails);

// out[0] = sum of (csize - 26) over the blocks; out[1] / out[2] = uoff of the first block starting
// after / at or after x (ulen if none); out[3] = the index of the first block starting after x.
void launch_block_stats(const int64_t* blk_pos, const int32_t* blk_cs, const int64_t* uoff,
                        int64_t nblk, int64_t ulen, int64_t x, uint64_t* out, hipStream_t s);

// Split planning (a2-a4).
constexpr int64_t SPLIT_FROM_SBI = -2;  // SplitPlan.first_blk of a chunk taken from a .sbi
struct SplitPlan {
  int64_t split_start, split_end;
  int64_t first_blk;     // chain index of the first guessed block (-1 none)
  int64_t u_lo, u_hi;    // linear U range scanned by the guesser
  int64_t rec_lin;       // linear U offset of the first record (-1 = empty partition)
  uint64_t vstart, vend;
  int32_t status;        // 0 ok; 100 = needs more data; else error
  int32_t rec_span;      // bytes of the <= 10 records chained from rec_lin (segment sizing)
};
void launch_plan_blocks(const Cand* cand, const int64_t* d_ncand, const int64_t* blk_pos,
                        const int32_t* blk_usize, const int64_t* uoff, const int64_t* d_nblk,
                        SplitPlan* plans, int64_t nsplit, hipStream_t s);
void launch_guess_all(const uint8_t* U, int64_t ulen, int32_t u_is_eof, const int32_t* ref_len,
                      int32_t n_ref, uint8_t* flag, hipStream_t s);
// best: 2 * nsplit words of device scratch
void launch_first_record(const uint8_t* U, int64_t ulen, int32_t u_is_eof, const int32_t* ref_len,
                         int32_t n_ref, const int64_t* blk_pos, const int64_t* uoff,
                         const int64_t* d_nblk, SplitPlan* plans, int64_t nsplit,
                         unsigned long long* best, hipStream_t s);

// Kernel 3: record chain over U from `start_lin`.
struct Seg {
  int64_t start;   // speculated / exact first chain position in the segment (-1 none)
  int64_t exit;    // first chain position >= segment end reached from `start`
  int64_t count;   // records started in [start, segment end)
  int32_t exact;   // bit 1: seg_walk recorded the record starts (SEG_OFF_CAP u16 offsets from the
                   // segment start); a re-walk by seg_fix clears it
  int32_t status;
};
constexpr int SEG_OFF_CAP = 512;  // record starts one segment's walk records (64 KiB segments)
// Segments cover [start_lin, chain_end) (record starts wanted); ulen bounds the readable bytes.
void launch_seg_spec(const uint8_t* U, int64_t ulen, int32_t u_is_eof, int64_t chain_end,
                     const int32_t* ref_len, int32_t n_ref, Seg* segs, int64_t nseg,
                     int64_t seg_bytes, int64_t start_lin, uint16_t* offs, hipStream_t s);
void launch_seg_link(const Seg* segs, int64_t nseg, int64_t seg_bytes, int64_t start_lin,
                     int64_t ulen, int32_t* d_broken, hipStream_t s);
void launch_seg_fix2(const uint8_t* U, int64_t ulen, int32_t u_is_eof, int64_t chain_end,
                     Seg* segs, int64_t nseg,
                     int64_t seg_bytes, int64_t start_lin, int32_t* d_status, hipStream_t s);
void launch_seg_counts(const Seg* segs, int64_t nseg, int64_t* counts, hipStream_t s);
void launch_seg_emit2(const uint8_t* U, int64_t ulen, const Seg* segs, const int64_t* base,
                      int64_t nseg, int64_t* rec_lin, hipStream_t s, const uint16_t* offs = nullptr,
                      int64_t seg_bytes = 0, int64_t start_lin = 0);

// Sparse (windowed) record chains: every window is a run of inflated U bytes (whole-file layout)
// with an exact first record start; segments [seg0, next window's seg0) belong to it.
struct Win {
  int64_t u_start;      // exact first record start
  int64_t u_chain_end;  // record starts wanted: < u_chain_end
  int64_t u_limit;      // end of the inflated bytes (reads past it: status 4, needs more)
  int64_t seg0;         // first segment of the window
  int32_t at_eof;       // the window runs to the end of the file
  int32_t pad;
};
void launch_wseg(const uint8_t* U, const int32_t* ref_len, int32_t n_ref, const Win* wins,
                 int64_t nwin, Seg* segs, int64_t nseg, int64_t seg_bytes, int32_t* d_broken,
                 hipStream_t s);
void launch_wseg_fix(const uint8_t* U, Seg* segs, const Win* wins, int64_t nwin, int64_t nseg,
                     int64_t seg_bytes, int32_t* d_status, hipStream_t s);

struct RecSoA {
  uint64_t* voffset;
  int32_t* block_size;
  int32_t* ref_id;
  int32_t* pos;
  int32_t* l_seq;
  int32_t* next_ref_id;
  int32_t* next_pos;
  int32_t* tlen;
  uint16_t* flag;
  uint16_t* bin;
  uint16_t* n_cigar;
  uint8_t* mapq;
  uint8_t* l_read_name;
  uint64_t* hash;
};
// pt: (ulen >> 16) + 1 int32 scratch (block page table); long_ent: long_list_cap(ulen, nrec)
// entries (the pieces of the records hashed by many threads), long_cnt: one device counter
int64_t long_list_cap(int64_t ulen, int64_t nrec);
void launch_decode_records(const uint8_t* U, int64_t ulen, const int64_t* rec_lin, int64_t nrec,
                           const int64_t* blk_pos, const int64_t* uoff, int64_t nblk, int32_t* pt,
                           RecSoA soa, int32_t* d_status, uint64_t* long_ent, int64_t long_cap,
                           unsigned long long* long_cnt, hipStream_t s);

struct PartRange {
  int64_t begin, end;   // record index range in the chain
  uint64_t digest;
};
void launch_sbi_sample(const uint64_t* voffset, int64_t nrec, int64_t g, uint64_t* out,
                       hipStream_t s);
void launch_partition_ranges(const SplitPlan* plans, int64_t nsplit, const int64_t* rec_lin,
                             const uint64_t* voffset, int64_t nrec, PartRange* parts,
                             int32_t* d_status, hipStream_t s);
void launch_bs_plus4(const int32_t* bs, int64_t n, int32_t* out, hipStream_t s);
void launch_add_u64(const uint64_t* in, int64_t n, uint64_t add, uint64_t* out, hipStream_t s);
void launch_partition_digest2(const uint64_t* hash, PartRange* parts, int64_t nparts,
                              hipStream_t s);
void launch_partition_digest_idx(const uint64_t* hash, const int64_t* kept, PartRange* parts,
                                 int64_t nparts, hipStream_t s);

// Record export: record-index ranges -> index list; SoA rows and raw bytes gathered by index into
// compact buffers (idx == nullptr in gather_raw: records first .. first + n - 1).
void launch_ranges_to_idx(const int64_t* begin, const int64_t* out_off, int64_t nranges,
                          int64_t* idx, hipStream_t s);
void launch_gather_soa(const int64_t* idx, int64_t n, const RecSoA src, RecSoA dst, hipStream_t s);
void launch_gather_raw(const uint8_t* U, const int64_t* rec_lin, const int32_t* block_size,
                       const int64_t* idx, int64_t first, int64_t n, const int64_t* out_off,
                       uint8_t* out, hipStream_t s);

// Interval traversal over .bai span chunks (partition order): record range of every chunk, keep
// flags -> compact kept index list, per-partition digests over an index list.
void launch_span_ranges(const uint64_t* voffset, int64_t nrec, const uint64_t* cbeg,
                        const uint64_t* cend, int64_t nchunk, int64_t* first, int64_t* count,
                        hipStream_t s);
void launch_keep_to_i32(const uint8_t* keep, int64_t n, int32_t* out, hipStream_t s);
// Span-run unplaced tail: keep flags of chunk k's entries (idx[off[k]..off[k+1])) = from the first
// record with refID == -1 on (*first: device scratch, initialised to all ones).
void launch_tail_keep(const int64_t* idx, const int64_t* off, int k, const int32_t* ref,
                      unsigned long long* first, uint8_t* keep, int64_t max_n, hipStream_t s);
void launch_gather_i64(const int64_t* src, const int64_t* pos, int64_t n, int64_t* dst,
                       hipStream_t s);
void launch_compact_kept(const int64_t* idx, const uint8_t* keep, const int64_t* off, int64_t n,
                         int64_t* kept, hipStream_t s);

// Kernel 4: interval filter; keep[t] for record idx[t] (or t when idx == NULL).
void launch_interval_filter(const uint8_t* U, const int64_t* rec_lin, const RecSoA soa,
                            const int64_t* idx, int64_t n, const int32_t* iv_ref,
                            const int32_t* iv_start, const int32_t* iv_end,
                            const int32_t* ref_iv_begin, int32_t n_ref, uint8_t* keep,
                            hipStream_t s);

// ------------------------------------------------------------------ BGZF text (VCF) path
struct TextPlan {
  int64_t split_start, split_end;
  int64_t k0, k1;   // the split's lines: indices [k0, k1)
  int64_t b0;       // the split stream's first block (-1 none)
  int32_t status;
  int32_t bom;      // line k0 == 0 starts with a UTF-8 BOM that LineRecordReader strips
};
int64_t text_tiles(int64_t ulen);
void launch_text_terms(const uint8_t* U, int64_t ulen, int32_t* tile_count, const int64_t* tile_off,
                       int64_t* term_pos, bool emit, hipStream_t s);
void launch_text_cr_fills(const uint8_t* U, const int64_t* uoff, const int32_t* blk_us, int64_t nblk,
                          int64_t* last_cr_fill, hipStream_t s);
void launch_text_plan(const Cand* cand, const int64_t* ncand, const int64_t* blk_pos,
                      const int32_t* blk_us, const int64_t* uoff, int64_t nblk, int64_t flen,
                      const uint8_t* U, int64_t ulen, const int64_t* term, int64_t nterm,
                      const int64_t* last_cr_fill, TextPlan* plans, int64_t nsplit, hipStream_t s);
void launch_text_values(const uint8_t* U, int64_t ulen, const int64_t* term, int64_t nterm,
                        const int64_t* idx, int64_t n, int32_t bom, int32_t drop_hash,
                        int64_t* vstart, int32_t* vlen, uint64_t* hash, uint8_t* keep,
                        hipStream_t s);
void launch_text_parts(const int64_t* out_off, const int64_t* koff, int64_t nsplit, PartRange* parts,
                       hipStream_t s);
void launch_text_export(const int64_t* kept, int64_t n, const int64_t* vstart, const int32_t* vlen,
                        const uint64_t* hash, int64_t* o_start, int32_t* o_len, uint64_t* o_hash,
                        hipStream_t s);
void launch_vcf_overlap(const uint8_t* U, const int64_t* vstart, const int32_t* vlen, int64_t n,
                        const uint8_t* names, const int32_t* noff, int32_t nnames,
                        const int32_t* ivbeg, const int32_t* ivstart, const int32_t* ivmaxend,
                        uint8_t* keep, hipStream_t s);
void launch_text_gather(const uint8_t* U, const int64_t* vstart, const int32_t* vlen,
                        const int64_t* kept, const int64_t* out_off, int64_t n, uint8_t* out,
                        hipStream_t s);

// DQ_CHECKED: each kernel unit's check words (count << 32 | site bits), read and reset
uint64_t dq_chk_take_kernels();
uint64_t dq_chk_take_inflate();
uint64_t dq_chk_take_text();
uint64_t dq_chk_take_deflate();

// ------------------------------------------------------------------ BGZF deflate (write path)
int64_t bgzf_block_count(int64_t n);
size_t bgzf_stage_bytes(int64_t nblk);
size_t bgzf_meta_bytes(int64_t nblk);
size_t bgzf_slot_bytes(int64_t nblk);  // the blocks' output slots
bool deflate_tables(int device);
// Blocks [blk0, blk0 + nblk) of src[0, n_in) (65280 bytes each) into fixed-size slots: the
// chunk parse kernel, the Huffman kernel, then the code/emit kernel.  tim (DQ_DEFLATE_TIMING): 8
// words per parse workgroup (2 per block), then 8 per block for each of the other two kernels.
void launch_bgzf_deflate(const uint8_t* src, int64_t n_in, int64_t blk0, int64_t nblk,
                         uint32_t* stage, uint32_t* meta, uint8_t* out_slots, int32_t* out_size,
                         uint64_t* tim, hipStream_t s);
// Packs the slots at offsets scanned on the device from the sizes on top of *total (the stream's
// length so far, updated).
void launch_bgzf_pack(const uint8_t* slots, const int32_t* size, int64_t* off, int64_t* total,
                      int64_t nblk, uint8_t* out, hipStream_t s);

}  // namespace dq
