/*
 * disq_gpu.h -- C ABI of libdisq_gpu.so, the MI355X (gfx950) BAM read path for Disq.
 *
 * Drop-in boundary.  A JNI / Panama shim implements the three
 * template methods of D/impl/formats/sam/AbstractBinarySamSource.java:138-150 on top of these
 * calls; callers of HtsjdkReadsRddStorage.read() (D/HtsjdkReadsRddStorage.java:83-131) are
 * unchanged.  No HIP or torch types cross this boundary: plain pointers and sizes only.
 *
 *   reference interface                                         replaced by
 *   ---------------------------------------------------------   -------------------------------
 *   BamSource.getPathChunks (D/impl/formats/bam/BamSource.java:61-104)
 *     = PathSplitSource.getPathSplits (D/impl/file/PathSplitSource.java:26-64)
 *     + BgzfBlockSource/BgzfBlockGuesser (D/impl/formats/bgzf/BgzfBlockSource.java:34-84,
 *       BgzfBlockGuesser.java:76-149)
 *     + getFirstReadInPartition/BamRecordGuesser (BamSource.java:110-153,
 *       D/impl/formats/bam/BamRecordGuesser.java:34-194)                    dq_plan
 *   BamSource.getIterator(SamReader, SAMFileSpan) (BamSource.java:172-175), one Spark task
 *                                                      dq_decode_chunk (dq_decode on a resident file)
 *   BamSource.createIndexIterator + queryUnmapped tail
 *     (BamSource.java:177-182; AbstractBinarySamSource.java:86-134)
 *                                    dq_decode_chunk_filtered (dq_decode_filtered on a resident file)
 *   AbstractBinarySamSource.getReads, whole RDD (AbstractBinarySamSource.java:42-136)  dq_read
 *   AbstractSamSource.getFileHeader (D/impl/formats/sam/AbstractSamSource.java:32-49)
 *                                                                           dq_read_header
 *
 * Error mapping (Java side): DQ_EIO -> IOException; DQ_EFORMAT -> htsjdk SAMFormatException;
 * DQ_EINVAL -> IllegalArgumentException; DQ_EDEVICE / DQ_ENOMEM -> RuntimeException.
 * Threading: a dq_ctx is used by one thread at a time (one per Spark task thread); each ctx owns
 * its own HIP stream.  Every call is synchronous with respect to its results.
 */
#ifndef DISQ_GPU_H
#define DISQ_GPU_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI version: 2 = dq_batch with the trailing arena_hold pointer (round 5) and the export modes
 * below (round 6).  A JNI / FFM binding compares dq_abi_version() with the value it was built
 * against before it maps dq_batch. */
#define DQ_ABI_VERSION 2

#define DQ_OK 0
#define DQ_EIO (-1)
#define DQ_EFORMAT (-2)
#define DQ_EINVAL (-3)
#define DQ_EDEVICE (-4)
#define DQ_ENOMEM (-5)

/* ValidationStringency (htsjdk); recorded, see DESIGN.md "STRICT validation". */
#define DQ_STRINGENCY_STRICT 0
#define DQ_STRINGENCY_LENIENT 1
#define DQ_STRINGENCY_SILENT 2

typedef struct dq_ctx dq_ctx;

/* HtsjdkReadsRddStorage builder state (D/HtsjdkReadsRddStorage.java:19-73) + device knobs. */
typedef struct dq_opts {
  int32_t device;            /* HIP device ordinal */
  int32_t split_size;        /* splitSize(int); 0 = Hadoop default (one split per block) */
  int32_t use_nio;           /* useNio(boolean): NIO ceil(len/splitSize) splits */
  int32_t verify_crc;        /* check each BGZF block's CRC32 (stricter than htsjdk default) */
  int32_t stringency;        /* validationStringency (recorded) */
  int32_t full_traversal;    /* 1: interval runs inflate and filter the whole file; 0 (default):
                                only the .bai spans of the intervals (dq_run_resident) */
  int64_t hadoop_block_size; /* fs.local.block.size; 0 = 32 MiB */
  int32_t compat;            /* DQ_COMPAT_DISQ_EXACT (default) or DQ_COMPAT_DEDUPE */
  int32_t reserved;
} dq_opts;

/* dq_opts.compat.  DISQ_EXACT reproduces Disq's chunk ends, (splitEnd << 16) | 0xffff
 * (BamSource.java:136-143): when a BGZF block starts exactly at a split end, the records starting
 * in it are read by that partition and again by the next one (BgzfBlockSource includes a block at
 * pos == splitEnd in both splits).  DEDUPE ends guessed chunks at splitEnd << 16 instead, so each
 * record belongs to exactly one partition (the one whose split holds its start block); .sbi chunks
 * are unaffected (they never overlap). */
#define DQ_COMPAT_DISQ_EXACT 0
#define DQ_COMPAT_DEDUPE 1

/* One Spark partition of the BAM read plan: a PathChunk (D/impl/file/PathChunk.java). */
typedef struct dq_chunk {
  int64_t split_start;  /* PathSplit [start, end) */
  int64_t split_end;
  uint64_t vstart;      /* Chunk virtual start (first record found by the guesser) */
  uint64_t vend;        /* Chunk virtual end = (split_end << 16) | 0xffff */
  int32_t has_chunk;    /* 0: getFirstReadInPartition returned null (empty partition) */
  int32_t reserved;
} dq_chunk;

/* Records as structure-of-arrays (fixed BAM fields, SAMv1 §4.2), host memory owned by the
 * library.  raw holds each record's 4 + block_size bytes (what htsjdk's
 * SAMRecordFactory.createBAMRecord needs as restOfData) at raw_offset[i].
 *
 * Export modes (the `with_raw` argument of the decode calls):
 *   DQ_EXPORT_FIELDS  every SoA field, hash and raw_offset; raw = NULL
 *   DQ_EXPORT_RAW     the same plus the raw bytes
 *   DQ_EXPORT_LEAN    voffset and raw only (every other pointer NULL, partition digests kept): the
 *                     fields are the first 36 bytes of each record's raw bytes (block_size, refID,
 *                     pos, bin_mq_nl, flag_nc, l_seq, next_refID, next_pos, tlen: what htsjdk's
 *                     BAMRecordCodec.decode reads, H/BAMFileReader2.java:929-931), and record i+1
 *                     starts 4 + block_size bytes after record i.  52 fewer bytes per record
 *                     cross PCIe.
 * dq_batch_free may release pinned memory (an arena batch) after dq_ctx_destroy: a JNI consumer
 * must free its batches before the HIP runtime shuts down (not from a JVM shutdown hook that can
 * run after it). */
#define DQ_EXPORT_FIELDS 0
#define DQ_EXPORT_RAW 1
#define DQ_EXPORT_LEAN 2
typedef struct dq_batch {
  int64_t n_records;
  uint64_t* voffset;     /* htsjdk start file pointer of the record */
  int32_t* block_size;
  int32_t* ref_id;
  int32_t* pos;          /* 0-based as stored; SAMRecord alignmentStart = pos + 1 */
  int32_t* l_seq;
  int32_t* next_ref_id;
  int32_t* next_pos;
  int32_t* tlen;
  uint16_t* flag;
  uint16_t* bin;
  uint16_t* n_cigar;
  uint8_t* mapq;
  uint8_t* l_read_name;
  uint64_t* hash;        /* per-record raw-byte hash */
  int64_t* raw_offset;
  uint8_t* raw;          /* may be NULL when the caller asked for fields only */
  int64_t raw_len;
  int64_t n_partitions;
  int64_t* part_offset;  /* n_partitions + 1 entries: partition p = [part_offset[p], [p+1]) */
  uint64_t* part_digest; /* ordered digest of each partition's record hashes */
  int32_t in_arena;      /* 1: the arrays live in the context's export arena (dq_set_export_arena) */
  int32_t reserved;
  void* arena_hold;      /* library-internal: the arena's ownership record (NULL off the arena) */
} dq_batch;

/* Interval traversal (HtsjdkReadsTraversalParameters, D/HtsjdkReadsTraversalParameters.java):
 * intervals already converted to (reference index, 1-based start, 1-based end) as in
 * BoundedTraversalUtil.convertSimpleIntervalToQueryInterval (BoundedTraversalUtil.java:36-53).
 * intervals == NULL means getIntervalsForTraversal() == null. */
typedef struct dq_traversal {
  const int32_t* ref;
  const int32_t* start;
  const int32_t* end;
  int64_t n;
  int32_t has_intervals;            /* 0: null interval list */
  int32_t traverse_unplaced_unmapped;
} dq_traversal;

typedef struct dq_header_info {
  int32_t n_ref;
  int32_t reserved;
  uint64_t first_record_voffset;
  int64_t header_bytes;   /* l_text etc. total, uncompressed */
} dq_header_info;

/* Timings / counters of the last pipeline run on the device (for benchmarks). */
typedef struct dq_stats {
  int64_t compressed_bytes;
  int64_t decompressed_bytes;
  int64_t n_blocks;
  int64_t n_records;        /* records emitted over all partitions (duplicates included) */
  int64_t n_partitions;
  double ms_total;          /* device time of the whole pipeline (HIP events) */
  double ms_scan;           /* kernel 1: BGZF scan + chain */
  double ms_inflate;        /* kernel 2: the inflate kernel alone */
  double ms_records;        /* kernel 3: record starts + SoA decode + hash */
  double ms_filter;         /* kernel 4: interval filter */
  double ms_plan;           /* split planning (guesser) */
  uint64_t digest;          /* digest over partition digests, in partition order */
  double ms_crc;            /* CRC32 verification kernel */
  int64_t deflate_bytes;    /* compressed DEFLATE payload bytes (sum of BSIZE + 1 - 26) */
  int64_t n_filtered;       /* records kernel 4 kept (dq_run_resident with intervals), else -1 */
  int64_t h2d_bytes;        /* compressed bytes the last open/decode copied host -> device */
  int64_t owned_bytes;      /* decompressed bytes of the blocks starting inside the splits (the
                               whole stream for a whole file; the shards of a file sum to it) */
  int64_t blocks_inflated;  /* BGZF blocks the last run inflated (fewer than n_blocks in a
                               .bai span run) */
  double ms_span;           /* .bai span run: device time of the sparse inflate + chains + filter */
} dq_stats;

int dq_ctx_create(dq_ctx** out, const dq_opts* opts);
void dq_ctx_destroy(dq_ctx* ctx);
const char* dq_last_error(const dq_ctx* ctx);
const char* dq_version(void);
int32_t dq_abi_version(void); /* DQ_ABI_VERSION of the library */

/* Open a BAM from host memory (copied to HBM) or from a path.  The resident file is used by
 * every call below until the next open. */
int dq_open_memory(dq_ctx* ctx, const uint8_t* bam, int64_t len);
int dq_open_path(dq_ctx* ctx, const char* path);

/* Byte-range shard of one file (multi-GPU): `bytes` are the file's bytes
 * [base, base + len) -- from the start of split p0 through the end of split p1 - 1, plus a halo
 * long enough to hold the last partition's straddling record (the end of the halo may cut a
 * BGZF block).  `file_len` is the whole file's length (split arithmetic) and the shard owns Disq
 * partitions [p0, p1).  `header` is the decompressed BAM header (dq_read_header of the file's
 * first bytes), which the record guesser needs.  Every later call reports file coordinates
 * (split offsets and virtual offsets), exactly as for the whole file.  A halo that is too short
 * fails with DQ_EFORMAT "shard halo too small" (retry with more bytes). */
int dq_open_shard(dq_ctx* ctx, const uint8_t* bytes, int64_t len, int64_t base, int64_t file_len,
                  int64_t p0, int64_t p1, const uint8_t* header, int64_t header_len);

/* The same with the shard's bytes already in device memory (multi-GPU: a rank's own byte range
 * stays resident in HBM and the halo arrives from the next rank over RCCL/xGMI).  dev_bytes is a
 * caller-owned device pointer on this context's device with at least len + 4096 readable bytes,
 * the last 4096 zero; it must stay valid and unchanged until the next open. */
int dq_open_shard_device(dq_ctx* ctx, const void* dev_bytes, int64_t len, int64_t base,
                         int64_t file_len, int64_t p0, int64_t p1, const uint8_t* header,
                         int64_t header_len);

/* The same, reading the shard's bytes [base, base + len) from `path` itself (pinned staging,
 * parallel reads from the page cache overlapped with the copies to the device): the streaming
 * (out-of-core) reader's windows and multi-GPU ranks that read a shared file. */
int dq_open_shard_path(dq_ctx* ctx, const char* path, int64_t base, int64_t len, int64_t p0,
                       int64_t p1, const uint8_t* header, int64_t header_len);

/* Whole-node mode in one process (the benchmark entry of SURVEY.md section 8(b)): the file's
 * partitions in contiguous groups, one per device of `devices` (by the even byte range holding
 * each split's first byte, as disq_amd.parallel.shard_plan), each group decoded on its own
 * context and host thread from the file alone (dq_open_shard_path with a halo grown x4 while too
 * short + dq_run_resident; records stay in HBM and are freed).  `ctx` supplies the options and
 * reads the header once.  digest folds every partition's digest in partition order: it equals
 * dq_stats.digest of a one-device run of the whole file. */
typedef struct dq_multi_result {
  int32_t n_devices;
  int32_t reserved;
  int64_t n_partitions;
  int64_t n_records;
  int64_t compressed_bytes;    /* file length */
  int64_t decompressed_bytes;  /* sum of the shards' owned bytes (= the file's stream) */
  uint64_t digest;
  double ms_wall;              /* header read + all shards (open, upload, pipeline), host clock */
  double ms_shard_wall_max;    /* slowest shard, host clock */
  double ms_device_max;        /* slowest shard's device pipeline (HIP events) */
} dq_multi_result;
int dq_decode_file_multi(dq_ctx* ctx, const char* path, const int32_t* devices, int32_t n_devices,
                         dq_multi_result* out);

/* The decompressed BAM header (AbstractSamSource.getFileHeader, D/impl/formats/sam/
 * AbstractSamSource.java:32-49) from the first `len` bytes of a file: enough BGZF blocks to hold
 * it (the last one may be cut).  Writes up to cap bytes to out; *out_len = header length.  Used
 * by the multi-GPU path: one rank reads it and broadcasts it to the others' dq_open_shard. */
int dq_header_from_prefix(dq_ctx* ctx, const uint8_t* bytes, int64_t len, uint8_t* out,
                          int64_t cap, int64_t* out_len);

/* .bai bytes for interval traversal (AbstractSamSource.findIndex: path.bai or .bam->.bai). */
int dq_set_index(dq_ctx* ctx, const uint8_t* bai, int64_t len);

int dq_read_header(dq_ctx* ctx, dq_header_info* info, uint8_t* header_bytes, int64_t cap);

/* .sbi splitting index bytes (htsjdk SBIIndex.load, M/htsjdk/samtools/SBIIndex.java:117-165:
 * magic "SBI\1", ascending virtual offsets).  Disq's getPathChunks loads it and then discards the
 * result (D/impl/formats/bam/BamSource.java:69-87), so with use_for_planning = 0 (Disq-exact,
 * the default) it is validated and ignored.  With use_for_planning = 1 dq_plan gives each split
 * the chunk SBIIndex.getChunk(splitStart, splitEnd) returns (SBIIndex.java:244-264: from the
 * first indexed record at or after the split start to the first at or after the split end) and
 * no record guessing runs.  NULL clears it. */
int dq_set_splitting_index(dq_ctx* ctx, const uint8_t* sbi, int64_t len, int32_t use_for_planning);

/* BAMSBIIndexer.createIndex (M/htsjdk/samtools/BAMSBIIndexer.java:45-66) + SBIIndexWriter
 * (SBIIndexWriter.java:84-151) for the open (whole) file: every granularity-th record's virtual
 * offset from the first record, then the final pointer; zero MD5 and UUID.  *out is
 * library-allocated (dq_free); granularity <= 0 means htsjdk's default 4096. */
int dq_write_sbi(dq_ctx* ctx, int64_t granularity, uint8_t** out, int64_t* out_len);

/* getPathChunks: all splits of the open file, in Disq partition order.  *chunks is
 * library-allocated; free with dq_free. */
int dq_plan(dq_ctx* ctx, dq_chunk** chunks, int64_t* n);

/* getIterator(span): the records of one chunk (start pointer < vend), in file order. */
int dq_decode(dq_ctx* ctx, uint64_t vstart, uint64_t vend, int32_t with_raw, dq_batch** out);

/* BamSource.getIterator(SamReader, SAMFileSpan) as a Spark task runs it (BamSource.java:172-175),
 * with no resident file: reads from `path` only the compressed bytes of the chunk's blocks
 * [vstart >> 16, first block past vend >> 16] plus what the last record needs (the window grows
 * until that record is whole), inflates them and walks the records from the exact start pointer
 * while start < vend.  The file's header is read once per context and path.  Afterwards the
 * context holds no open file (dq_plan / dq_read need an open again).  stats.h2d_bytes
 * (dq_get_stats) reports the compressed bytes copied to the device. */
int dq_decode_chunk(dq_ctx* ctx, const char* path, uint64_t vstart, uint64_t vend, int32_t with_raw,
                    dq_batch** out);

/* createIndexIterator(intervals, contained=false) + the unplaced-unmapped tail for one task
 * (AbstractBinarySamSource.java:86-134) with no resident file: the .bai span of the optimized
 * intervals (dq_set_index first) clipped to the chunk is the only part of `path` read -- span
 * chunks closer than 1 MiB are read as one window, each decoded from its exact start pointer --
 * then kernel 4 keeps the overlapping records; if the chunk holds the .bai's start of the last
 * linear bin and traverse_unplaced_unmapped is set, the records with refID -1 from there to EOF
 * follow (queryUnmapped).  One partition in the batch. */
int dq_decode_chunk_filtered(dq_ctx* ctx, const char* path, uint64_t vstart, uint64_t vend,
                             const dq_traversal* tr, int32_t with_raw, dq_batch** out);

/* createIndexIterator(intervals, contained=false) over one chunk, plus the unplaced-unmapped
 * tail when the chunk contains the .bai's start of the last linear bin. */
int dq_decode_filtered(dq_ctx* ctx, uint64_t vstart, uint64_t vend, const dq_traversal* tr,
                       int32_t with_raw, dq_batch** out);

/* getReads for the whole file: every partition, in order (tr may be NULL). */
int dq_read(dq_ctx* ctx, const dq_traversal* tr, int32_t with_raw, dq_batch** out);

/* Run the whole device pipeline on the resident file without copying records back (records
 * stay in HBM); fills stats.  This is the benchmark entry point.  With intervals in tr (needs
 * dq_set_index, as createIndexIterator does; AbstractBinarySamSource.java:86-112), the traversal
 * of every partition as Disq runs it: the .bai span of the optimized intervals clipped to each
 * partition chunk is the only part of the file inflated (the partition plans come from a full run
 * of the open file, made first if there is none); records of the spans are filtered by kernel 4
 * (overlap, contained=false).  stats.n_records = records in the spans, stats.n_filtered = kept,
 * stats.blocks_inflated, stats.ms_span; dq_partition_digests gives the kept count and digest per
 * partition.  With opts.full_traversal, or traverse_unplaced_unmapped, every record of the file is
 * filtered instead (stats.ms_filter; the unplaced tail is not included). */
int dq_run_resident(dq_ctx* ctx, const dq_traversal* tr, dq_stats* stats);

/* Stats of the last pipeline run (the ones dq_run_resident returns). */
int dq_get_stats(dq_ctx* ctx, dq_stats* stats);

/* Per-partition record counts and digests of the last pipeline run, in partition order (the
 * shard's partitions p0..p1-1 for a shard): *n = number of partitions; up to cap entries written.
 * The whole-file digest folds them. */
int dq_partition_digests(dq_ctx* ctx, int64_t* counts, uint64_t* digests, int64_t cap, int64_t* n);

/* Device pointer of the resident decompressed stream (for tests), and its length. */
int dq_debug_inflated(dq_ctx* ctx, uint8_t* host_out, int64_t cap, int64_t* len);

/* Test hook: the GPU record guesser (BamRecordGuesser.checkRecordStart) evaluated at EVERY
 * decompressed position of a whole resident file, as BamRecordGuesserChecker does with a
 * granularity-1 index (D/impl/formats/bam/BamRecordGuesserChecker.java:104-120).  Writes the
 * virtual offsets where it fires, ascending, up to cap; *n = how many there are. */
int dq_debug_guess_all(dq_ctx* ctx, uint64_t* voffs, int64_t cap, int64_t* n);

/* ---- BGZF text (VCF) path ----------------------------------
 * Replaces, for a BGZF-compressed text file, Hadoop's TextInputFormat record reader running over
 * Disq's splittable codecs: BGZFCodec / BGZFEnhancedGzipCodec.createInputStream
 * (D/impl/formats/bgzf/BGZFCodec.java:57-68, BGZFEnhancedGzipCodec.java:41-74) and
 * BGZFSplitCompressionInputStream (BGZFSplitCompressionInputStream.java:14-106) under Hadoop 2.7
 * LineRecordReader, as VcfSource.getVariants uses them (D/impl/formats/vcf/VcfSource.java:88-113).
 * A partition is one FileInputFormat split (same arithmetic as the BAM path); its lines are the
 * values LineRecordReader returns, terminators excluded; drop_header_lines drops the values
 * starting with '#' (VcfSource.java:108).  Parsing a line into a VariantContext is the caller's. */
typedef struct dq_text_batch {
  int64_t n_lines;
  int64_t* line_offset;   /* value offset in the file's decompressed stream */
  int32_t* line_len;      /* value length in bytes */
  uint64_t* hash;         /* hash of the value bytes (same function as the record hash) */
  int64_t* data_offset;   /* value k = data[data_offset[k], data_offset[k] + line_len[k]) */
  uint8_t* data;
  int64_t n_bytes;
  int64_t n_partitions;
  int64_t* part_offset;   /* lines of partition p: [part_offset[p], part_offset[p + 1]) */
  uint64_t* part_digest;  /* ordered digest of the partition's line hashes */
} dq_text_batch;

int dq_text_open_memory(dq_ctx* ctx, const uint8_t* bytes, int64_t len);
/* VcfSource.getVariants with intervals (D/impl/formats/vcf/VcfSource.java:88-113, 144-168): the
 * tabix index (the DECOMPRESSED bytes of the .tbi; NULL clears) and the intervals (contig names,
 * 1-based closed starts and ends; contig == NULL or n < 0 clears, n == 0 keeps nothing).  With
 * intervals set, dq_text_run / dq_text_read keep only the splits whose [start, end] overlaps an
 * index block of some interval (TribbleIndexIntervalFilteringTextInputFormat.getSplits) and only
 * the lines whose variant (CHROM, POS .. POS + len(REF) - 1 or INFO END) overlaps an interval
 * (OverlapDetector.overlapsAny); '#' lines are always dropped then.  stats.n_partitions counts
 * the kept splits. */
int dq_text_set_index(dq_ctx* ctx, const uint8_t* tbi, int64_t len);
int dq_text_set_intervals(dq_ctx* ctx, const char* const* contig, const int32_t* start,
                          const int32_t* end, int64_t n);
int dq_text_open_path(dq_ctx* ctx, const char* path);
/* Scan, inflate, line planning and digests; the lines stay in HBM.  stats: n_records = lines
 * kept, n_filtered = '#' lines dropped, digest = whole-file digest of the partition digests. */
int dq_text_run(dq_ctx* ctx, int32_t drop_header_lines, dq_stats* stats);
int dq_text_read(dq_ctx* ctx, int32_t drop_header_lines, dq_text_batch** out);
void dq_text_batch_free(dq_text_batch* b);

/* ---- BGZF compression: the write path -----------------------
 * Replaces htsjdk BlockCompressedOutputStream under HeaderlessBamOutputFormat.BamRecordWriter
 * (D/impl/formats/bam/HeaderlessBamOutputFormat.java:26-50) and BamSink's header file
 * (BAMFileWriter.writeHeader, D/impl/formats/bam/BamSink.java:46-50): `data` is cut into blocks
 * of 65280 bytes (htsjdk DEFAULT_UNCOMPRESSED_BLOCK_SIZE, the last one shorter), each compressed
 * on the GPU into one BGZF member ('BC' extra field, BSIZE, CRC32, ISIZE).  No EOF terminator is
 * written (BamSink appends BlockCompressedStreamConstants.EMPTY_GZIP_BLOCK once, after all parts).
 * The DEFLATE bit stream is this library's own (LZ77 + a dynamic Huffman code per block, the
 * fixed code when that is shorter, stored when neither fits): the blocks inflate to exactly
 * htsjdk's block contents; the compressed bytes differ from java.util.zip.Deflater's.  *out is
 * malloc'ed (dq_free). */
int dq_bgzf_compress(dq_ctx* ctx, const uint8_t* data, int64_t len, uint8_t** out, int64_t* out_len);
/* The same over the resident decompressed stream of the open file (benchmark / round trip): the
 * result stays in HBM (dq_bgzf_fetch copies it out); *ms = device time. */
int dq_bgzf_compress_resident(dq_ctx* ctx, int64_t* out_len, double* ms);
int dq_bgzf_fetch(dq_ctx* ctx, uint8_t* host_out, int64_t cap);

/* Export arena: batches of this context (dq_read, dq_decode*) place their arrays in `bytes` of
 * pinned host memory, copied by DMA with no staging copies (a batch that does not fit takes heap
 * memory as before): a streaming consumer's recycled buffers, one Spark task's records at a time.
 * The arena holds ONE batch: while it is alive (until dq_batch_free), a batch that would go to
 * the arena and dq_set_export_arena return DQ_EINVAL, and dq_ctx_destroy leaves the arena to the
 * batch, whose dq_batch_free releases it (per-task ownership with auto-close,
 * AutocloseIteratorWrapper.java:26-36).  bytes = 0 releases the arena. */
int dq_set_export_arena(dq_ctx* ctx, int64_t bytes);
void dq_batch_free(dq_batch* b);
void dq_free(void* p);

/* Debug: the device bounds-checked build (`make -C disq_amd/csrc checked` ->
 * libdisq_gpu_checked.so, compiled with -DDQ_CHECKED).  Writes each kernel unit's failed-check
 * count << 32 | largest reported excess << 16 | site bits (K1/K3 kernels, K2 inflate, text,
 * deflate: 4 words) for the current
 * device and resets them; returns 1 in the checked build, 0 in the product build (words all 0). */
int dq_checked_report(uint64_t words[4]);

#ifdef __cplusplus
}
#endif
#endif
