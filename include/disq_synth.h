/* disq_synth.h -- synthetic BAM workload generator (tests and bench.py; not the read path). */
#ifndef DISQ_SYNTH_H
#define DISQ_SYNTH_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  DQ_SYNTH_WGS = 0,      /* 2x150 bp pairs, GRCh38-like dictionary (configs C2/C3) */
  DQ_SYNTH_ANYSAM = 1,   /* T/AnySamTestUtil.java:37-105 shape; n_records = number of pairs */
  DQ_SYNTH_LONGREAD = 2  /* ONT-like 10-100 kb reads, 1% at 0.5-2 Mb (config C5) */
};

typedef struct dq_synth_opts {
  int64_t n_records;          /* records (pairs for ANYSAM) */
  uint64_t seed;
  int32_t shape;
  int32_t level;              /* deflate level; htsjdk default 5 */
  int32_t nthreads;
  int32_t write_bai;
  int64_t sbi_granularity;    /* 0 = no .sbi */
  int64_t records_per_chunk;  /* 0 = default */
  double unplaced_fraction;   /* trailing unplaced-unmapped records (WGS/LONGREAD) */
  /* Byte range of one logical file (multi-GPU benchmark: each rank generates only its shard).
   * The file is the concatenation of ceil(n_records / records_per_chunk) independently seeded
   * chunks, each ending on a BGZF block boundary (chunk 0 starts with the header), then the EOF
   * block.  chunk_hi > 0 generates chunks [chunk_lo, chunk_hi) only (plus the EOF block when
   * chunk_hi is the last chunk); their bytes are the file's bytes at the offset equal to the
   * total length of chunks [0, chunk_lo).  No .bai/.sbi in that mode. */
  int64_t chunk_lo;
  int64_t chunk_hi;
} dq_synth_opts;

typedef struct dq_synth_result {
  uint8_t* bam;
  int64_t bam_len;
  uint8_t* bai;
  int64_t bai_len;
  uint8_t* sbi;
  int64_t sbi_len;
  int64_t n_records;
  int64_t n_blocks;      /* including the EOF block */
  int64_t record_bytes;  /* decompressed bytes of records (excludes the header) */
  int64_t n_chunks;      /* chunks of the whole logical file */
} dq_synth_result;

int dq_synth_bam(const dq_synth_opts* opts, dq_synth_result* res);
void dq_synth_free(dq_synth_result* res);

#ifdef __cplusplus
}
#endif
#endif
