/*
 * disq_oracle.h -- CPU restatement of Disq's BAM read path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libdisq_gpu.so, disq_amd/) links or calls
 * this code.  It is the checker used by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg.
 *
 * Parity pinning: the restatement is checked against the reference's own fixtures
 * (src/test/resources/1.bam, 1-with-splitting-index.bam.sbi) and the numbers its tests assert
 * (BgzfBlockSourceTest.java:31-35, BamRecordGuesserCheckerTest.java:16-70).  The reference is
 * Java (Disq + htsjdk 2.16.0 + Hadoop 2.7 + Spark 2.2); no JVM exists in this image, so the
 * reference itself cannot be run here (see DESIGN.md "Oracle").
 */
#ifndef DISQ_ORACLE_H
#define DISQ_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Error codes (mirror include/disq_gpu.h). */
#define DQO_OK 0
#define DQO_EIO (-1)
#define DQO_EFORMAT (-2)
#define DQO_EINVAL (-3)
#define DQO_ENOMEM (-5)
#define DQO_ESHORT (-6) /* a shard window ended before the bytes a partition needed */

/* One decoded record (a8 of SURVEY.md §8). */
typedef struct dqo_rec {
  uint64_t voffset;     /* htsjdk start file pointer (normalised, BAMFileReader2.java:962-971) */
  int64_t lin;          /* offset in the linearised decompressed stream */
  int32_t block_size;   /* BAM block_size (record length - 4) */
  int32_t ref_id;
  int32_t pos;          /* 0-based, as stored */
  int32_t l_seq;
  int32_t next_ref_id;
  int32_t next_pos;
  int32_t tlen;
  int32_t align_end;    /* htsjdk getAlignmentEnd() (1-based, 0 if unmapped) */
  uint16_t flag;
  uint16_t bin;
  uint16_t n_cigar;
  uint8_t mapq;
  uint8_t l_read_name;
  uint64_t hash;        /* dqo_record_hash of the 4+block_size raw bytes */
} dqo_rec;

typedef struct dqo_file dqo_file;

/* Wrap an in-memory BAM (not copied; caller keeps it alive). */
dqo_file* dqo_open_mem(const uint8_t* data, int64_t len, int verify_crc);
void dqo_close(dqo_file* f);
const char* dqo_last_error(dqo_file* f);

/* a1: PathSplitSource.getPathSplits (PathSplitSource.java:26-64) for one file.
 * nio=1: ceil(len/splitSize) splits; nio=0: Hadoop 2.7 FileInputFormat.getSplits with
 * SPLIT_MAXSIZE=split_size (if >0) and the local block size.  Returns #splits or <0. */
int64_t dqo_path_splits(int64_t file_len, int32_t split_size, int nio, int64_t local_block_size,
                        int64_t* starts, int64_t* ends, int64_t cap);

/* a2: BgzfBlockGuesser.guessNextBGZFPos(p, end) (BgzfBlockGuesser.java:76-149).
 * Returns 1 and fills the block, or 0 for "null". */
int dqo_guess_next_bgzf(dqo_file* f, int64_t p, int64_t end, int64_t* pos, int32_t* csize,
                        int32_t* usize);

/* a3: BgzfBlockSource iterator over one split (BgzfBlockSource.java:63-84).  Returns #blocks. */
int64_t dqo_split_blocks(dqo_file* f, int64_t split_start, int64_t split_end, int64_t* pos,
                         int32_t* csize, int32_t* usize, int64_t cap);

/* a10: BAM header (BAMFileReader2.java:747-821).  Must be called before record functions.
 * Fills n_ref and the first-record voffset; ref_lengths receives up to cap lengths. */
int dqo_read_header(dqo_file* f, int32_t* n_ref, uint64_t* first_record_voffset,
                    int32_t* ref_lengths, int32_t cap);
/* Reference name lookup (for interval preparation). Returns index or -1. */
int32_t dqo_ref_index(dqo_file* f, const char* name);

/* a5: BamRecordGuesser.checkRecordStart(vPos) (BamRecordGuesser.java:34-194). 1/0, <0 error. */
int dqo_check_record_start(dqo_file* f, uint64_t vpos);

/* a4: BamSource.getFirstReadInPartition (BamSource.java:110-153) for one split.
 * Returns 1 with the chunk, 0 for an empty partition, <0 on error. */
int dqo_first_read_in_split(dqo_file* f, int64_t split_start, int64_t split_end, uint64_t* vstart,
                            uint64_t* vend);

/* BamRecordGuesserChecker (granularity 1): every position of one split's blocks where the
 * guesser fires.  Returns the count (positions written up to cap). */
int64_t dqo_scan_record_starts(dqo_file* f, int64_t split_start, int64_t split_end, uint64_t* out,
                               int64_t cap);

/* a6-a8: BAMFileIndexIterator over one chunk (BAMFileReader2.java:1063-1096).
 * Returns #records written (records whose start pointer < vend), or <0. If out==NULL only
 * counts. */
int64_t dqo_read_chunk(dqo_file* f, uint64_t vstart, uint64_t vend, dqo_rec* out, int64_t cap);

/* queryUnmapped from a given start pointer (BAMFileReader2.java:715-738,1199-1206). */
int64_t dqo_read_unmapped(dqo_file* f, uint64_t start, dqo_rec* out, int64_t cap);

/* Whole-file sequential walk from the first record (BAMSBIIndexer.java:45-66 semantics). */
int64_t dqo_read_all(dqo_file* f, dqo_rec* out, int64_t cap);

/* .bai facts used by AbstractBinarySamSource.java:92-94. */
int dqo_bai_info(const uint8_t* bai, int64_t len, int32_t* n_ref, int64_t* start_of_last_linear_bin,
                 int64_t* no_coordinate_count);

/* .bai span of optimized intervals (getFileSpan) clipped to a partition chunk [vstart, vend)
 * (AbstractBinarySamSource.java:105-107).  Returns the chunk count (up to cap written), or <0. */
int64_t dqo_bai_span(const uint8_t* bai, int64_t len, const int32_t* ref, const int32_t* start,
                     const int32_t* end, int64_t n_iv, uint64_t vstart, uint64_t vend,
                     uint64_t* out_beg, uint64_t* out_end, int64_t cap);

/* Interval preparation: QueryInterval.optimizeIntervals (htsjdk 2.16, via
 * BoundedTraversalUtil.java:10-27).  In-place on (ref, start, end) arrays; returns new count. */
int64_t dqo_optimize_intervals(int32_t* ref, int32_t* start, int32_t* end, int64_t n);

/* BAMQueryMultipleIntervalsIteratorFilter overlap test (contained=false) for one record. */
int dqo_record_overlaps(const dqo_rec* r, const int32_t* ref, const int32_t* start,
                        const int32_t* end, int64_t n);

/* Hashes shared with the GPU path (definition in DESIGN.md). */
uint64_t dqo_record_hash(const uint8_t* bytes, int64_t n);
uint64_t dqo_stream_digest(const uint64_t* hashes, int64_t n, uint64_t start_index);

/* Inflate every BGZF block of the file in order from offset 0 (real headers, htsjdk
 * BlockCompressedInputStream semantics).  Returns decompressed length, or <0.  If out==NULL,
 * returns the required length. */
/* BGZF text (VCF) path: the lines Hadoop's LineRecordReader returns for split [start, end) of a
 * BGZF text file read through Disq's BGZFCodec (value offsets in the decompressed stream and
 * value lengths); drop_hash drops lines starting with '#' (VcfSource.getVariants). */
int64_t dqo_text_split_lines(dqo_file* f, int64_t start, int64_t end, int drop_hash,
                             int64_t* vstart, int64_t* vlen, int64_t cap);

int64_t dqo_inflate_file(dqo_file* f, uint8_t* out, int64_t cap);

/* CPU baseline: Disq's per-partition work (a4 + a6..a8 + hash) for a list of splits on
 * nthreads threads (one partition per task, like Spark local[N]).  Writes per-split record
 * counts and stream digests (digest indices restart at 0 per split). */
int dqo_run_partitions(const uint8_t* data, int64_t len, const int64_t* starts,
                       const int64_t* ends, int64_t n_splits, int nthreads, int64_t* counts,
                       uint64_t* digests, int64_t* ubytes);
/* The same over a shard window: bytes [base, base + len) of a file_len-byte file, `header` its
 * decompressed BAM header (the window lacks the file's first blocks).  DQO_ESHORT: a partition
 * needed bytes past the window (a halo too small). */
dqo_file* dqo_open_window(const uint8_t* data, int64_t base, int64_t len, int64_t file_len);
int dqo_set_header(dqo_file* f, const uint8_t* u, int64_t n);
int dqo_run_partitions_window(const uint8_t* data, int64_t base, int64_t len, int64_t file_len,
                              const uint8_t* header, int64_t header_len, const int64_t* starts,
                              const int64_t* ends, int64_t n, int nthreads, int64_t* counts,
                              uint64_t* digests, int64_t* ubytes);
/* Interval traversal of every partition on nthreads threads: per partition the records of the
 * .bai span of the optimized intervals q (sorted, disjoint; spans = 0: the whole chunk) that
 * overlap q, plus the unplaced-unmapped tail when `unplaced`; count + ordered digest. */
int dqo_run_partitions_traversal(const uint8_t* data, int64_t len, const int64_t* starts,
                                 const int64_t* ends, int64_t n, int nthreads,
                                 const uint8_t* bai, int64_t bai_len, const int32_t* q_ref,
                                 const int32_t* q_start, const int32_t* q_end, int64_t nq,
                                 int unplaced, int spans, int64_t* counts, uint64_t* digests);

#ifdef __cplusplus
}
#endif
#endif
