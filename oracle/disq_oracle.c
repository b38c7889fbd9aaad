/*
 * disq_oracle.c -- CPU restatement of Disq's BAM read path (TEST INFRASTRUCTURE ONLY).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this code, and only
 * as the checker; the product path (libdisq_gpu.so) never links it.
 *
 * Each function cites the reference file:line it restates.  Abbreviations:
 *   D/  = /root/reference/src/main/java/org/disq_bio/disq/
 *   H/  = /root/reference/src/main/java/htsjdk/samtools/   (vendored htsjdk shims)
 * htsjdk 2.16.0 classes that are NOT vendored (BlockCompressedInputStream, BlockGunzipper,
 * BAMRecordCodec, QueryInterval, BAMQueryMultipleIntervalsIteratorFilter) are restated from their
 * published 2.16.0 behaviour; their call sites in the reference are cited instead.
 *
 * Stream model.  htsjdk's BlockCompressedInputStream reads BGZF blocks one after another by the
 * BSIZE field at header offset 16 (BLOCK_HEADER_LENGTH = 18) and raw-inflates exactly ISIZE
 * bytes from each (BlockGunzipper.unzipBlock).  A file pointer is (block address << 16 | offset);
 * a pointer at the end of a non-empty block reads as (next block address, 0) -- confirmed by the
 * final offset (597454, 0) of the reference fixture 1-with-splitting-index.bam.sbi.  Empty BGZF
 * blocks in the middle of a stream are treated as transparent (documented limitation).
 */
#include "disq_oracle.h"

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#define MAX_USIZE 65536
#define NCACHE 4
#define R_EOF 11      /* java.io.EOFException */
#define R_IOERR 12    /* other java.io.IOException */
#define R_FORMAT 13   /* htsjdk SAMFormatException / RuntimeIOException (not caught by Disq) */

struct dqo_file {
  const uint8_t* data; /* the file's bytes [base, len) (a whole file: base 0, len = file_len) */
  int64_t len;         /* end of the held bytes, in file coordinates */
  int64_t base;        /* file offset of data[0] (a shard window of a larger file) */
  int64_t file_len;    /* the whole file's length (where EOF is) */
  int short_window;    /* a read needed bytes past a shard window that ends before EOF */
  int verify_crc;
  /* header */
  int have_header;
  int32_t n_ref;
  int32_t* ref_len;
  char** ref_name;
  uint64_t first_record;
  char err[256];
};

static void set_err(dqo_file* f, const char* msg) {
  if (f) snprintf(f->err, sizeof f->err, "%s", msg);
}

static inline uint16_t rd16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static inline int32_t rd32(const uint8_t* p) {
  return (int32_t)((uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
                   ((uint32_t)p[3] << 24));
}
static inline uint64_t rd64(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; i--) v = (v << 8) | p[i];
  return v;
}
/* Java int32 wrap-around arithmetic. */
static inline int32_t jadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
static inline int32_t jmul(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }
static inline int32_t jdiv2(int32_t a) { return a / 2; } /* Java truncates toward zero, as C99 */

/* ------------------------------------------------------------------ hashes */
static inline uint64_t mix64(uint64_t z) {
  z ^= z >> 30;
  z *= 0xBF58476D1CE4E5B9ULL;
  z ^= z >> 27;
  z *= 0x94D049BB133111EBULL;
  z ^= z >> 31;
  return z;
}

uint64_t dqo_record_hash(const uint8_t* b, int64_t n) {
  uint64_t h = (uint64_t)n * 0x9E3779B97F4A7C15ULL;
  int64_t nw = (n + 7) / 8;
  for (int64_t i = 0; i < nw; i++) {
    uint64_t w = 0;
    for (int k = 7; k >= 0; k--) {
      int64_t j = i * 8 + k;
      w = (w << 8) | (j < n ? b[j] : 0);
    }
    h += mix64(w ^ ((uint64_t)(i + 1) * 0xD6E8FEB86659FD93ULL));
  }
  return mix64(h);
}

uint64_t dqo_stream_digest(const uint64_t* hs, int64_t n, uint64_t start_index) {
  uint64_t d = 0;
  for (int64_t k = 0; k < n; k++)
    d += mix64(hs[k] + (start_index + (uint64_t)k + 1) * 0x9E3779B97F4A7C15ULL);
  return d;
}

/* ------------------------------------------------------------------ file */
dqo_file* dqo_open_mem(const uint8_t* data, int64_t len, int verify_crc) {
  dqo_file* f = (dqo_file*)calloc(1, sizeof(dqo_file));
  if (!f) return NULL;
  f->data = data;
  f->len = len;
  f->file_len = len;
  f->verify_crc = verify_crc;
  return f;
}

/* A shard window: bytes [base, base + len) of a file of file_len bytes (test infrastructure for
 * the multi-GPU bench's per-rank parity: a rank holds only its byte range plus the halo).  Reads
 * past the window's end, when it is not the file's end, set short_window instead of reading EOF. */
dqo_file* dqo_open_window(const uint8_t* data, int64_t base, int64_t len, int64_t file_len) {
  dqo_file* f = dqo_open_mem(data, base + len, 0);
  if (!f) return NULL;
  f->base = base;
  f->file_len = file_len;
  return f;
}

void dqo_close(dqo_file* f) {
  if (!f) return;
  if (f->ref_name)
    for (int i = 0; i < f->n_ref; i++) free(f->ref_name[i]);
  free(f->ref_name);
  free(f->ref_len);
  free(f);
}

const char* dqo_last_error(dqo_file* f) { return f ? f->err : "null file"; }

/* ------------------------------------------------------------------ a1 splits */
/* PathSplitSource.getPathSplits: D/impl/file/PathSplitSource.java:26-64.
 * NIO branch :32-42; Hadoop branch :44-62 -> Hadoop 2.7 FileInputFormat.getSplits
 * (computeSplitSize = max(minSize=1, min(maxSize, blockSize)); SPLIT_SLOP = 1.1). */
int64_t dqo_path_splits(int64_t len, int32_t split_size, int nio, int64_t local_block_size,
                        int64_t* starts, int64_t* ends, int64_t cap) {
  int64_t n = 0;
  if (nio) {
    if (split_size <= 0) return DQO_EINVAL; /* ceil(len/0) is undefined in the reference */
    int64_t ns = (len + split_size - 1) / split_size;
    for (int64_t i = 0; i < ns; i++) {
      int64_t s = i * (int64_t)split_size;
      int64_t e = s + split_size > len ? len : s + split_size;
      if (n < cap) { starts[n] = s; ends[n] = e; }
      n++;
    }
    return n;
  }
  int64_t max_size = split_size > 0 ? split_size : INT64_MAX;
  int64_t ss = local_block_size < max_size ? local_block_size : max_size;
  if (ss < 1) ss = 1;
  if (len == 0) {
    if (n < cap) { starts[n] = 0; ends[n] = 0; }
    return 1;
  }
  int64_t rem = len;
  while (((double)rem) / ss > 1.1) {
    if (n < cap) { starts[n] = len - rem; ends[n] = len - rem + ss; }
    n++;
    rem -= ss;
  }
  if (rem != 0) {
    if (n < cap) { starts[n] = len - rem; ends[n] = len; }
    n++;
  }
  return n;
}

/* ------------------------------------------------------------------ a2/a3 block guesser */
/* BgzfBlockGuesser.guessNextBGZFPos: D/impl/formats/bgzf/BgzfBlockGuesser.java:76-149.
 * Any read past EOF is an IOException caught at :146-148 -> null. */
int dqo_guess_next_bgzf(dqo_file* f, int64_t p, int64_t end, int64_t* opos, int32_t* ocsize,
                        int32_t* ousize) {
  const uint8_t* d = f->data; /* indexed as d[x - B]: x in file coordinates */
  const int64_t L = f->len, B = f->base;
#define NEED(q, n) \
  do {             \
    if ((q) < B || (q) + (n) > L) {                          \
      if ((q) + (n) > L && L < f->file_len) f->short_window = 1; \
      return 0;                                             \
    }                                                       \
  } while (0)
  for (;;) {
    for (;;) { /* :79-92 */
      NEED(p, 4);
      uint32_t n = (uint32_t)rd32(d + (p - B));
      if (n == 0x04088b1fu) break;
      if ((n >> 8) == 0x00088b1fu) p += 1;
      else if ((n >> 16) == 0x8b1fu) p += 2;
      else p += 3;
      if (p >= end) return 0;
    }
    const int64_t p0 = p; /* :95 */
    p += 10;
    NEED(p, 2);
    int32_t xlen = rd16(d + (p - B));
    p += 2;
    const int64_t sub_end = p + xlen;
    int64_t q = p; /* stream position */
    int cancelled = 0;
    while (p < sub_end) { /* :103 */
      NEED(q, 4);
      uint32_t id = (uint32_t)rd32(d + (q - B));
      if (id != 0x00024342u) {
        p += 4 + rd16(d + (q - B) + 2);
        q = p;
        continue;
      }
      NEED(q + 4, 2);
      int32_t bsize = rd16(d + (q - B) + 4); /* :117-118 */
      p += 6;                          /* :121 */
      while (p < sub_end) {            /* :122-126 */
        NEED(p, 4);
        p += 4 + rd16(d + (p - B) + 2);
      }
      if (p != sub_end) { /* :127-131 */
        cancelled = 1;
        break;
      }
      p += (int64_t)bsize - xlen - 19 + 4; /* :134 */
      NEED(p, 4);
      *opos = p0;
      *ocsize = (int32_t)(p + 4 - p0);
      *ousize = rd32(d + (p - B));
      return 1;
    }
    (void)cancelled;
    p = p0 + 4; /* :144 -- note: the inner loop tests this position before any end check */
  }
#undef NEED
}

/* BgzfBlockSource iterator: D/impl/formats/bgzf/BgzfBlockSource.java:63-84. */
int64_t dqo_split_blocks(dqo_file* f, int64_t s, int64_t e, int64_t* pos, int32_t* cs, int32_t* us,
                         int64_t cap) {
  int64_t n = 0;
  int64_t start = s;
  for (;;) {
    if (start > e) break; /* :70 */
    int64_t bp;
    int32_t bc, bu;
    if (!dqo_guess_next_bgzf(f, start, e, &bp, &bc, &bu)) break;
    if (n < cap) { pos[n] = bp; cs[n] = bc; us[n] = bu; }
    n++;
    start = bp + bc; /* :79 */
  }
  return n;
}

/* ------------------------------------------------------------------ block reader */
typedef struct {
  int64_t addr;
  int32_t csize; /* 0 for the EOF pseudo-block */
  int32_t len;
  int valid;
  uint64_t stamp;
  uint8_t data[MAX_USIZE];
} blkbuf;

typedef struct {
  dqo_file* f;
  blkbuf* c[NCACHE];
  uint64_t clock;
  blkbuf* cur;
  int32_t off;
  z_stream zs;
  int zinit;
} rdr;

static int rdr_init(rdr* r, dqo_file* f) {
  memset(r, 0, sizeof *r);
  r->f = f;
  for (int i = 0; i < NCACHE; i++) {
    r->c[i] = (blkbuf*)calloc(1, sizeof(blkbuf));
    if (!r->c[i]) return DQO_ENOMEM;
  }
  if (inflateInit2(&r->zs, -15) != Z_OK) return DQO_ENOMEM;
  r->zinit = 1;
  return 0;
}

static void rdr_free(rdr* r) {
  for (int i = 0; i < NCACHE; i++) free(r->c[i]);
  if (r->zinit) inflateEnd(&r->zs);
}

/* htsjdk BlockCompressedInputStream.processNextBlock + BlockGunzipper.unzipBlock (htsjdk 2.16.0,
 * not vendored; used through BamSource.java:158,174). Returns 0 or R_IOERR / R_FORMAT. */
static int inflate_block(rdr* r, int64_t addr, blkbuf* b) {
  const uint8_t* d = r->f->data;
  const int64_t L = r->f->len;
  b->addr = addr;
  b->valid = 1;
  if (addr >= r->f->file_len) { /* headerByteCount == 0: "no empty gzip block at end" -> empty block */
    b->csize = 0;
    b->len = 0;
    return 0;
  }
  if (addr < r->f->base ||
      (L < r->f->file_len && (L - addr < 18 || L - addr < rd16(d + (addr - r->f->base) + 16) + 1))) {
    /* a shard window that does not hold the whole block (and does not end at EOF) */
    r->f->short_window = 1;
    set_err(r->f, "read outside the shard window");
    b->valid = 0;
    return R_IOERR;
  }
  if (L - addr < 18) { set_err(r->f, "incorrect header size"); b->valid = 0; return R_IOERR; }
  const uint8_t* h = d + (addr - r->f->base);
  int32_t blen = rd16(h + 16) + 1;
  if (blen < 18 || blen > 65536) { set_err(r->f, "unexpected block length"); b->valid = 0; return R_IOERR; }
  if (L - addr < blen) { set_err(r->f, "premature end of file"); b->valid = 0; return R_IOERR; }
  if (h[0] != 0x1f || h[1] != 0x8b || h[2] != 8 || h[3] != 4 || rd16(h + 10) != 6) {
    set_err(r->f, "Invalid GZIP header");
    b->valid = 0;
    return R_FORMAT;
  }
  int32_t defl = blen - 18 - 8;
  uint32_t crc_exp = (uint32_t)rd32(h + 18 + defl);
  int32_t isize = rd32(h + 18 + defl + 4);
  if (isize < 0 || isize > MAX_USIZE) { set_err(r->f, "ISIZE out of range"); b->valid = 0; return R_FORMAT; }
  inflateReset(&r->zs);
  r->zs.next_in = (Bytef*)(h + 18);
  r->zs.avail_in = (uInt)defl;
  r->zs.next_out = b->data;
  r->zs.avail_out = (uInt)isize;
  int zr = Z_OK;
  while (r->zs.avail_out > 0) {
    zr = inflate(&r->zs, Z_SYNC_FLUSH);
    if (zr != Z_OK) break;
  }
  if (zr == Z_DATA_ERROR || zr == Z_MEM_ERROR || zr == Z_NEED_DICT) {
    set_err(r->f, "inflate data error");
    b->valid = 0;
    return R_FORMAT;
  }
  if ((int32_t)((uint8_t*)r->zs.next_out - b->data) != isize) {
    set_err(r->f, "Did not inflate expected amount");
    b->valid = 0;
    return R_FORMAT;
  }
  if (r->f->verify_crc) {
    uint32_t c = (uint32_t)crc32(0L, b->data, (uInt)isize);
    if (c != crc_exp) { set_err(r->f, "CRC mismatch"); b->valid = 0; return R_FORMAT; }
  }
  b->csize = blen;
  b->len = isize;
  return 0;
}

static int rdr_load(rdr* r, int64_t addr, blkbuf** out) {
  blkbuf* victim = NULL;
  for (int i = 0; i < NCACHE; i++) {
    if (r->c[i]->valid && r->c[i]->addr == addr) {
      r->c[i]->stamp = ++r->clock;
      *out = r->c[i];
      return 0;
    }
  }
  for (int i = 0; i < NCACHE; i++) {
    if (r->c[i] == r->cur) continue;
    if (!victim || !r->c[i]->valid || r->c[i]->stamp < victim->stamp) victim = r->c[i];
  }
  int e = inflate_block(r, addr, victim);
  if (e) return e;
  victim->stamp = ++r->clock;
  *out = victim;
  return 0;
}

/* Move to the following block, skipping empty mid-stream blocks (documented limitation). */
static int rdr_next_block(rdr* r) {
  for (;;) {
    if (r->cur->csize == 0) return R_EOF; /* EOF pseudo-block */
    blkbuf* nb;
    int e = rdr_load(r, r->cur->addr + r->cur->csize, &nb);
    if (e) return e;
    r->cur = nb;
    r->off = 0;
    if (nb->len > 0 || nb->csize == 0) return nb->len > 0 ? 0 : R_EOF;
  }
}

/* BlockCompressedInputStream.seek.  An offset beyond the block is "Invalid file pointer",
 * which BamRecordGuesser.seek turns into EOFException (BamRecordGuesser.java:206-216). */
static int rdr_seek(rdr* r, uint64_t v) {
  blkbuf* b;
  int e = rdr_load(r, (int64_t)(v >> 16), &b);
  if (e) return e;
  r->cur = b;
  r->off = (int32_t)(v & 0xffff);
  if (b->len == 0 && b->csize != 0) { /* empty mid-stream block: available() reads the next */
    if (r->off != 0) return R_EOF;
    e = rdr_next_block(r);
    if (e && e != R_EOF) return e;
    return 0;
  }
  if (r->off > b->len) return R_EOF;
  return 0;
}

static int rdr_read(rdr* r, uint8_t* dst, int64_t n) {
  while (n > 0) {
    if (r->off >= r->cur->len) {
      int e = rdr_next_block(r);
      if (e) return e;
    }
    int64_t a = r->cur->len - r->off;
    if (a > n) a = n;
    if (dst) {
      memcpy(dst, r->cur->data + r->off, (size_t)a);
      dst += a;
    }
    r->off += (int32_t)a;
    n -= a;
  }
  return 0;
}

/* BlockCompressedInputStream.getFilePointer (end-of-block normalisation). */
static uint64_t rdr_ptr(const rdr* r) {
  if (r->off > 0 && r->off == r->cur->len)
    return (uint64_t)(r->cur->addr + r->cur->csize) << 16;
  return ((uint64_t)r->cur->addr << 16) | (uint32_t)r->off;
}

/* ------------------------------------------------------------------ a10 header */
/* BAMFileReader2.readHeader / readSequenceRecord: H/BAMFileReader2.java:747-821. */
int dqo_read_header(dqo_file* f, int32_t* n_ref, uint64_t* first, int32_t* lens, int32_t cap) {
  rdr r;
  int e = rdr_init(&r, f);
  if (e) { rdr_free(&r); return e; }
  int rc = DQO_OK;
  uint8_t b4[4];
  char* text = NULL;
  if (rdr_seek(&r, 0) || rdr_read(&r, b4, 4) || memcmp(b4, "BAM\1", 4) != 0) {
    set_err(f, "Invalid BAM file header");
    rc = DQO_EFORMAT;
    goto out;
  }
  if (rdr_read(&r, b4, 4)) { rc = DQO_EFORMAT; goto out; }
  int32_t l_text = rd32(b4);
  if (l_text < 0) { rc = DQO_EFORMAT; goto out; }
  if (rdr_read(&r, NULL, l_text)) { rc = DQO_EFORMAT; goto out; }
  if (rdr_read(&r, b4, 4)) { rc = DQO_EFORMAT; goto out; }
  int32_t nr = rd32(b4);
  if (nr < 0) { rc = DQO_EFORMAT; goto out; }
  if (f->ref_name) {
    for (int i = 0; i < f->n_ref; i++) free(f->ref_name[i]);
    free(f->ref_name);
    free(f->ref_len);
  }
  f->n_ref = nr;
  f->ref_len = (int32_t*)calloc((size_t)nr + 1, sizeof(int32_t));
  f->ref_name = (char**)calloc((size_t)nr + 1, sizeof(char*));
  for (int32_t i = 0; i < nr; i++) {
    if (rdr_read(&r, b4, 4)) { rc = DQO_EFORMAT; goto out; }
    int32_t ln = rd32(b4);
    if (ln <= 1) { set_err(f, "missing sequence name"); rc = DQO_EFORMAT; goto out; }
    f->ref_name[i] = (char*)calloc((size_t)ln, 1);
    if (rdr_read(&r, (uint8_t*)f->ref_name[i], ln)) { rc = DQO_EFORMAT; goto out; }
    f->ref_name[i][ln - 1] = 0;
    if (rdr_read(&r, b4, 4)) { rc = DQO_EFORMAT; goto out; }
    f->ref_len[i] = rd32(b4);
  }
  f->first_record = rdr_ptr(&r);
  f->have_header = 1;
  *n_ref = nr;
  *first = f->first_record;
  for (int32_t i = 0; i < nr && i < cap; i++) lens[i] = f->ref_len[i];
out:
  free(text);
  rdr_free(&r);
  return rc;
}

/* The same header from its decompressed bytes (a shard window does not hold the file's first
 * blocks: the multi-GPU bench broadcasts the decompressed header, as the GPU shards use it). */
int dqo_set_header(dqo_file* f, const uint8_t* u, int64_t n) {
  int64_t p = 0;
#define TAKE(k) do { if (p + (k) > n) { set_err(f, "short header"); return DQO_EFORMAT; } } while (0)
  TAKE(8);
  if (memcmp(u, "BAM\1", 4) != 0) { set_err(f, "Invalid BAM file header"); return DQO_EFORMAT; }
  const int32_t l_text = rd32(u + 4);
  if (l_text < 0) return DQO_EFORMAT;
  p = 8 + (int64_t)l_text;
  TAKE(4);
  const int32_t nr = rd32(u + p);
  if (nr < 0) return DQO_EFORMAT;
  p += 4;
  if (f->ref_name) {
    for (int i = 0; i < f->n_ref; i++) free(f->ref_name[i]);
    free(f->ref_name);
    free(f->ref_len);
  }
  f->n_ref = nr;
  f->ref_len = (int32_t*)calloc((size_t)nr + 1, sizeof(int32_t));
  f->ref_name = (char**)calloc((size_t)nr + 1, sizeof(char*));
  for (int32_t i = 0; i < nr; i++) {
    TAKE(4);
    const int32_t ln = rd32(u + p);
    p += 4;
    if (ln <= 1) { set_err(f, "missing sequence name"); return DQO_EFORMAT; }
    TAKE(ln + 4);
    f->ref_name[i] = (char*)calloc((size_t)ln, 1);
    memcpy(f->ref_name[i], u + p, (size_t)ln);
    f->ref_name[i][ln - 1] = 0;
    p += ln;
    f->ref_len[i] = rd32(u + p);
    p += 4;
  }
#undef TAKE
  f->first_record = 0; /* not known without the compressed header blocks (unused by a window) */
  f->have_header = 1;
  return DQO_OK;
}

int32_t dqo_ref_index(dqo_file* f, const char* name) {
  for (int32_t i = 0; i < f->n_ref; i++)
    if (strcmp(f->ref_name[i], name) == 0) return i;
  return -1;
}

/* ------------------------------------------------------------------ a5 record guesser */
static int valid_name_char(uint8_t c) {
  int8_t b = (int8_t)c; /* Java byte comparison: BamRecordGuesser.java:196-198 */
  return ((int8_t)'!' <= b && b <= (int8_t)'?') || ((int8_t)'A' <= b && b <= (int8_t)'~');
}

/* checkRecordStartInternal: D/impl/formats/bam/BamRecordGuesser.java:79-194.
 * Returns 1 (start, *next set), 0 (no start), or R_EOF / R_IOERR / R_FORMAT. */
static int check_internal(rdr* r, uint64_t v, uint64_t* next) {
  dqo_file* f = r->f;
  uint8_t b[36];
  uint8_t name[256];
  int e = rdr_seek(r, v);
  if (e) return e;
  if ((e = rdr_read(r, b, 36))) return e; /* :98-99 */
  int32_t remaining = rd32(b);
  int32_t id = rd32(b + 4), pos = rd32(b + 8);
  if (id < -1 || id >= f->n_ref || pos < -1) return 0;  /* :110 */
  if (id >= 0 && pos > f->ref_len[id]) return 0;        /* :114 */
  int32_t nid = rd32(b + 24), npos = rd32(b + 28);
  if (nid < -1 || nid >= f->n_ref || npos < -1) return 0; /* :125 */
  if (nid >= 0 && npos > f->ref_len[nid]) return 0;       /* :129 */
  int32_t name_len = rd32(b + 12) & 0xff;
  if (name_len < 2) return 0; /* :138 */
  uint32_t flag_nc = (uint32_t)rd32(b + 16);
  int32_t flags = (int32_t)(flag_nc >> 16);
  int32_t n_cig = (int32_t)(flag_nc & 0xffff);
  int32_t cig_len = jmul(n_cig, 4);
  int32_t l_seq = rd32(b + 20);
  int32_t seq_len = jadd(l_seq, jdiv2(jadd(l_seq, 1))); /* :146 */
  if ((flags & 4) == 0 && (seq_len == 0 || n_cig == 0)) return 0;
  if ((e = rdr_read(r, name, name_len))) return e; /* :153-155 */
  if (name[name_len - 1] != 0) return 0;
  for (int i = 0; i < name_len - 1; i++)
    if (!valid_name_char(name[i])) return 0;
  for (int i = 0; i < n_cig; i++) { /* :167-176 */
    uint8_t c[4];
    if ((e = rdr_read(r, c, 4))) return e;
    int32_t op = rd32(c);
    if (op == -1) return R_EOF;
    if ((op & 0xf) > 8) return 0;
  }
  int32_t zero_min = jadd(jadd(jadd(32, name_len), cig_len), seq_len); /* :186 */
  if (remaining >= zero_min) {
    if ((e = rdr_seek(r, v))) return e; /* :189 */
    int32_t skip = jadd(4, remaining); /* int arithmetic, widened to long by skipFully */
    if (skip > 0 && (e = rdr_read(r, NULL, skip))) return e;
    *next = rdr_ptr(r);
    return 1;
  }
  return 0;
}

/* checkRecordStart: BamRecordGuesser.java:34-52 (READS_TO_CHECK = 10 at :16). */
static int check_record_start(rdr* r, uint64_t v) {
  for (int k = 0; k < 10; k++) {
    uint64_t nv = 0;
    int res = check_internal(r, v, &nv);
    if (res == 1) { v = nv; continue; }
    if (res == 0) return 0;
    if (res == R_EOF) return k > 0;
    if (res == R_IOERR) return 0;
    return DQO_EFORMAT; /* runtime exception escapes Disq */
  }
  return 1;
}

int dqo_check_record_start(dqo_file* f, uint64_t v) {
  if (!f->have_header) return DQO_EINVAL;
  rdr r;
  if (rdr_init(&r, f)) { rdr_free(&r); return DQO_ENOMEM; }
  int res = check_record_start(&r, v);
  rdr_free(&r);
  return res;
}

/* ------------------------------------------------------------------ a4 first read */
/* BamSource.getFirstReadInPartition: D/impl/formats/bam/BamSource.java:110-153,
 * MAX_READ_SIZE = 10_000_000 at :44. */
static int first_read(rdr* r, int64_t s, int64_t e, uint64_t* vs, uint64_t* ve) {
  dqo_file* f = r->f;
  int64_t index = 0;
  int64_t start = s;
  for (;;) { /* lazy BgzfBlockSource iterator, BgzfBlockSource.java:63-84 */
    if (start > e) break;
    int64_t bp;
    int32_t bc, bu;
    if (!dqo_guess_next_bgzf(f, start, e, &bp, &bc, &bu)) break;
    start = bp + bc;
    for (int32_t up = 0; up < bu; up++) {
      index++;
      if (index > 10000000) return 0;
      if (up > 0xffff) return DQO_EFORMAT; /* makeFilePointer rejects offsets > 0xffff */
      uint64_t v = ((uint64_t)bp << 16) | (uint32_t)up;
      int res = check_record_start(r, v);
      if (res < 0) return res;
      if (res) {
        *vs = v;
        *ve = ((uint64_t)e << 16) | 0xffff;
        return 1;
      }
    }
  }
  return 0;
}

int dqo_first_read_in_split(dqo_file* f, int64_t s, int64_t e, uint64_t* vs, uint64_t* ve) {
  if (!f->have_header) return DQO_EINVAL;
  rdr r;
  if (rdr_init(&r, f)) { rdr_free(&r); return DQO_ENOMEM; }
  int res = first_read(&r, s, e, vs, ve);
  rdr_free(&r);
  return res;
}


/* BamRecordGuesserChecker.check with granularity 1 (D/impl/formats/bam/BamRecordGuesserChecker.java:
 * 96-124): run the guesser at every uncompressed position of every block of one split and
 * return the positions where it fires. */
int64_t dqo_scan_record_starts(dqo_file* f, int64_t s, int64_t e, uint64_t* out, int64_t cap) {
  if (!f->have_header) return DQO_EINVAL;
  rdr r;
  if (rdr_init(&r, f)) { rdr_free(&r); return DQO_ENOMEM; }
  int64_t n = 0;
  int64_t start = s;
  for (;;) {
    if (start > e) break;
    int64_t bp;
    int32_t bc, bu;
    if (!dqo_guess_next_bgzf(f, start, e, &bp, &bc, &bu)) break;
    start = bp + bc;
    for (int32_t up = 0; up < bu; up++) {
      uint64_t v = ((uint64_t)bp << 16) | (uint32_t)up;
      int res = check_record_start(&r, v);
      if (res < 0) { n = res; goto out; }
      if (res) {
        if (out && n < cap) out[n] = v;
        n++;
      }
    }
  }
out:
  rdr_free(&r);
  return n;
}

/* ------------------------------------------------------------------ a6-a8 decode */
static int32_t cigar_ref_len(const uint8_t* cig, int n) {
  int32_t len = 0;
  for (int i = 0; i < n; i++) {
    uint32_t op = (uint32_t)rd32(cig + 4 * i);
    uint32_t o = op & 0xf;
    if (o == 0 || o == 2 || o == 3 || o == 7 || o == 8) len += (int32_t)(op >> 4);
  }
  return len;
}

/* htsjdk BAMRecordCodec.decode field layout (SAMv1 §4.2); BAMRecord.getAlignmentEnd. */
static void fill_rec(dqo_rec* o, uint64_t v, const uint8_t* rec, int32_t block_size) {
  const uint8_t* p = rec + 4;
  o->voffset = v;
  o->lin = -1;
  o->block_size = block_size;
  o->ref_id = rd32(p + 0);
  o->pos = rd32(p + 4);
  uint32_t bmn = (uint32_t)rd32(p + 8);
  o->l_read_name = (uint8_t)(bmn & 0xff);
  o->mapq = (uint8_t)((bmn >> 8) & 0xff);
  o->bin = (uint16_t)(bmn >> 16);
  uint32_t fnc = (uint32_t)rd32(p + 12);
  o->n_cigar = (uint16_t)(fnc & 0xffff);
  o->flag = (uint16_t)(fnc >> 16);
  o->l_seq = rd32(p + 16);
  o->next_ref_id = rd32(p + 20);
  o->next_pos = rd32(p + 24);
  o->tlen = rd32(p + 28);
  if (o->flag & 4) {
    o->align_end = 0;
  } else {
    int64_t cig_off = 32 + (int64_t)o->l_read_name;
    int32_t rl = 0;
    if (cig_off + 4 * (int64_t)o->n_cigar <= block_size)
      rl = cigar_ref_len(p + cig_off, o->n_cigar);
    o->align_end = o->pos + 1 + rl - 1;
  }
  o->hash = dqo_record_hash(rec, 4 + (int64_t)block_size);
}

/* Read one record at the current position.  Returns 1 record, 0 end, <0 error. */
static int read_record(rdr* r, uint8_t** buf, int64_t* bufcap, int32_t* bs_out) {
  uint8_t b4[4];
  int e = rdr_read(r, b4, 4);
  if (e == R_EOF) return 0; /* BinaryCodec.readInt -> RuntimeEOFException -> decode() null */
  if (e) return DQO_EFORMAT;
  int32_t bs = rd32(b4);
  if (bs < 32) { set_err(r->f, "Invalid record length"); return DQO_EFORMAT; }
  if (*bufcap < 4 + (int64_t)bs) {
    int64_t nc = 4 + (int64_t)bs + 1024;
    uint8_t* nb = (uint8_t*)realloc(*buf, (size_t)nc);
    if (!nb) return DQO_ENOMEM;
    *buf = nb;
    *bufcap = nc;
  }
  memcpy(*buf, b4, 4);
  e = rdr_read(r, *buf + 4, bs);
  if (e) { set_err(r->f, "truncated record"); return DQO_EFORMAT; }
  *bs_out = bs;
  return 1;
}

/* BAMFileIndexIterator.getNextRecord: H/BAMFileReader2.java:1082-1095 with one chunk. */
int64_t dqo_read_chunk(dqo_file* f, uint64_t vs, uint64_t ve, dqo_rec* out, int64_t cap) {
  rdr r;
  if (rdr_init(&r, f)) { rdr_free(&r); return DQO_ENOMEM; }
  uint8_t* buf = NULL;
  int64_t bufcap = 0, n = 0;
  int e = rdr_seek(&r, vs);
  if (e == R_EOF) goto done;
  if (e) { n = DQO_EFORMAT; goto done; }
  for (;;) {
    uint64_t v = rdr_ptr(&r);
    if (v >= ve) break;
    int32_t bs;
    int res = read_record(&r, &buf, &bufcap, &bs);
    if (res < 0) { n = res; break; }
    if (res == 0) break;
    if (out && n < cap) fill_rec(&out[n], v, buf, bs);
    n++;
  }
done:
  free(buf);
  rdr_free(&r);
  return n;
}

/* BAMFileIndexUnmappedIterator: H/BAMFileReader2.java:1199-1206 (skip until refID == -1, then
 * everything to EOF), after queryUnmapped's seek (:715-738). */
int64_t dqo_read_unmapped(dqo_file* f, uint64_t start, dqo_rec* out, int64_t cap) {
  rdr r;
  if (rdr_init(&r, f)) { rdr_free(&r); return DQO_ENOMEM; }
  uint8_t* buf = NULL;
  int64_t bufcap = 0, n = 0;
  int skipping = 1;
  int e = rdr_seek(&r, start);
  if (e == R_EOF) goto done;
  if (e) { n = DQO_EFORMAT; goto done; }
  for (;;) {
    uint64_t v = rdr_ptr(&r);
    int32_t bs;
    int res = read_record(&r, &buf, &bufcap, &bs);
    if (res < 0) { n = res; break; }
    if (res == 0) break;
    if (skipping && rd32(buf + 4) != -1) continue;
    skipping = 0;
    if (out && n < cap) fill_rec(&out[n], v, buf, bs);
    n++;
  }
done:
  free(buf);
  rdr_free(&r);
  return n;
}

/* BAMSBIIndexer.createIndex walk (H/BAMSBIIndexer.java:45-66): every record from the first. */
int64_t dqo_read_all(dqo_file* f, dqo_rec* out, int64_t cap) {
  if (!f->have_header) return DQO_EINVAL;
  return dqo_read_chunk(f, f->first_record, UINT64_MAX, out, cap);
}

/* ------------------------------------------------------------------ a9 intervals */
/* AbstractBAMFileIndex.getStartOfLastLinearBin / getNoCoordinateCount (htsjdk 2.16.0), used at
 * D/impl/formats/sam/AbstractBinarySamSource.java:92-94. */
int dqo_bai_info(const uint8_t* b, int64_t len, int32_t* n_ref, int64_t* solb, int64_t* ncc) {
  int64_t p = 0;
#define NEED(n) do { if (p + (n) > len) return DQO_EFORMAT; } while (0)
  NEED(8);
  if (memcmp(b, "BAI\1", 4) != 0) return DQO_EFORMAT;
  int32_t nr = rd32(b + 4);
  p = 8;
  int64_t last = -1;
  for (int32_t i = 0; i < nr; i++) {
    NEED(4);
    int32_t nbin = rd32(b + p);
    p += 4;
    for (int32_t j = 0; j < nbin; j++) {
      NEED(8);
      int32_t nch = rd32(b + p + 4);
      p += 8 + 16 * (int64_t)nch;
    }
    NEED(4);
    int32_t nint = rd32(b + p);
    p += 4;
    if (nint > 0) {
      NEED(8 * (int64_t)nint);
      last = (int64_t)rd64(b + p + 8 * ((int64_t)nint - 1));
      p += 8 * (int64_t)nint;
    }
  }
  *n_ref = nr;
  *solb = last;
  *ncc = (p + 8 <= len) ? (int64_t)rd64(b + p) : -1; /* null for old indexes */
#undef NEED
  return 0;
}

/* .bai span of a list of optimized intervals, clipped to one partition chunk:
 *   BAMFileReader.getFileSpan (H/BAMFileReader2.java:1004-1019) -> per interval htsjdk 2.16.0
 *   CachingBAMFileIndex.getSpanOverlapping (bins from GenomicIndexUtil.regionToBins, their
 *   chunks, Chunk.optimizeChunkList with LinearIndex.getMinimumOffset(start)), then
 *   BAMFileSpan.merge (optimizeChunkList(all, 0)); then removeContentsBefore / removeContentsAfter
 *   of the partition chunk (D/impl/formats/sam/AbstractBinarySamSource.java:105-107).
 * htsjdk is not vendored (pom.xml:13), so this restates its published algorithm. */
typedef struct { uint64_t b, e; } dchunk;
static int dchunk_cmp(const void* x, const void* y) {
  const dchunk* a = (const dchunk*)x;
  const dchunk* c = (const dchunk*)y;
  if (a->b != c->b) return a->b < c->b ? -1 : 1;
  if (a->e != c->e) return a->e < c->e ? -1 : 1;
  return 0;
}
/* Chunk.overlaps / isAdjacentTo (block-address adjacency) */
static int dchunk_touch(const dchunk* l, const dchunk* r) {
  if (l->b == r->b && l->e == r->e) return 1;
  const dchunk* lo = dchunk_cmp(l, r) < 0 ? l : r;
  const dchunk* hi = lo == l ? r : l;
  if (lo->e > hi->b) return 1; /* overlap */
  return (l->e >> 16) == (r->b >> 16) || (l->b >> 16) == (r->e >> 16);
}
/* Chunk.optimizeChunkList: sort, drop chunks ending at or before min_off, coalesce. */
static int64_t optimize_chunks(dchunk* c, int64_t n, uint64_t min_off) {
  qsort(c, (size_t)n, sizeof(dchunk), dchunk_cmp);
  int64_t m = 0;
  for (int64_t i = 0; i < n; i++) {
    if (c[i].e <= min_off) continue;
    if (m == 0 || !dchunk_touch(&c[m - 1], &c[i])) {
      c[m++] = c[i];
    } else if (c[i].e > c[m - 1].e) {
      c[m - 1].e = c[i].e;
    }
  }
  return m;
}

int64_t dqo_bai_span(const uint8_t* b, int64_t len, const int32_t* ref, const int32_t* start,
                     const int32_t* end, int64_t n_iv, uint64_t vstart, uint64_t vend,
                     uint64_t* out_beg, uint64_t* out_end, int64_t cap) {
  if (len < 8 || memcmp(b, "BAI\1", 4) != 0) return DQO_EFORMAT;
  const int32_t nr = rd32(b + 4);
  /* offsets of each reference's section */
  int64_t* refp = (int64_t*)malloc(sizeof(int64_t) * (size_t)(nr + 1));
  int64_t p = 8;
  for (int32_t i = 0; i < nr; i++) {
    refp[i] = p;
    if (p + 4 > len) { free(refp); return DQO_EFORMAT; }
    const int32_t nbin = rd32(b + p);
    p += 4;
    for (int32_t j = 0; j < nbin; j++) {
      if (p + 8 > len) { free(refp); return DQO_EFORMAT; }
      p += 8 + 16 * (int64_t)rd32(b + p + 4);
    }
    if (p + 4 > len) { free(refp); return DQO_EFORMAT; }
    p += 4 + 8 * (int64_t)rd32(b + p);
  }
  int64_t cap_all = 1024, n_all = 0;
  dchunk* all = (dchunk*)malloc(sizeof(dchunk) * (size_t)cap_all);
  for (int64_t k = 0; k < n_iv; k++) {
    const int32_t r = ref[k];
    if (r < 0 || r >= nr) continue;
    /* GenomicIndexUtil.regionToBins(startPos, endPos) */
    const int32_t maxp = 0x1FFFFFFF;
    const int32_t s0 = start[k] <= 0 ? 0 : (start[k] - 1) & maxp;
    const int32_t e0 = end[k] <= 0 ? maxp : (end[k] - 1) & maxp;
    if (s0 > e0) continue;
    int64_t q = refp[r];
    const int32_t nbin = rd32(b + q);
    q += 4;
    int64_t cap_c = 64, n_c = 0;
    dchunk* cl = (dchunk*)malloc(sizeof(dchunk) * (size_t)cap_c);
    for (int32_t j = 0; j < nbin; j++) {
      const uint32_t bin = (uint32_t)rd32(b + q);
      const int32_t nch = rd32(b + q + 4);
      const int64_t cq = q + 8;
      q = cq + 16 * (int64_t)nch;
      if (bin == 37450) continue; /* pseudo-bin (metadata) */
      int in = bin == 0;
      if (!in && bin >= 1 && bin <= 8) in = bin >= 1 + (uint32_t)(s0 >> 26) && bin <= 1 + (uint32_t)(e0 >> 26);
      if (!in && bin >= 9 && bin <= 72) in = bin >= 9 + (uint32_t)(s0 >> 23) && bin <= 9 + (uint32_t)(e0 >> 23);
      if (!in && bin >= 73 && bin <= 584) in = bin >= 73 + (uint32_t)(s0 >> 20) && bin <= 73 + (uint32_t)(e0 >> 20);
      if (!in && bin >= 585 && bin <= 4680) in = bin >= 585 + (uint32_t)(s0 >> 17) && bin <= 585 + (uint32_t)(e0 >> 17);
      if (!in && bin >= 4681) in = bin >= 4681 + (uint32_t)(s0 >> 14) && bin <= 4681 + (uint32_t)(e0 >> 14);
      if (!in) continue;
      for (int32_t c = 0; c < nch; c++) {
        if (n_c == cap_c) { cap_c *= 2; cl = (dchunk*)realloc(cl, sizeof(dchunk) * (size_t)cap_c); }
        cl[n_c].b = rd64(b + cq + 16 * (int64_t)c);
        cl[n_c].e = rd64(b + cq + 16 * (int64_t)c + 8);
        n_c++;
      }
    }
    /* LinearIndex.getMinimumOffset(startPos) */
    const int32_t nint = rd32(b + q);
    const int32_t lb = s0 >> 14;
    const uint64_t min_off = lb < nint ? rd64(b + q + 4 + 8 * (int64_t)lb) : 0;
    n_c = optimize_chunks(cl, n_c, min_off);
    for (int64_t c = 0; c < n_c; c++) {
      if (n_all == cap_all) { cap_all *= 2; all = (dchunk*)realloc(all, sizeof(dchunk) * (size_t)cap_all); }
      all[n_all++] = cl[c];
    }
    free(cl);
  }
  free(refp);
  n_all = optimize_chunks(all, n_all, 0); /* BAMFileSpan.merge */
  int64_t m = 0;
  for (int64_t i = 0; i < n_all; i++) {
    dchunk c = all[i];
    if (c.e <= vstart) continue;          /* removeContentsBefore */
    if (c.b < vstart) c.b = vstart;
    if (c.b >= vend) continue;            /* removeContentsAfter */
    if (c.e > vend) c.e = vend;
    if (m < cap) { out_beg[m] = c.b; out_end[m] = c.e; }
    m++;
  }
  free(all);
  return m;
}

/* QueryInterval compareTo / overlaps / abuts and optimizeIntervals (htsjdk 2.16.0), called from
 * D/impl/formats/BoundedTraversalUtil.java:26.  end <= 0 means "to the end of the contig". */
typedef struct { int32_t ref, start, end; } qiv;
static int32_t qend(int32_t e) { return e <= 0 ? INT32_MAX : e; }
static int qcmp(const void* a, const void* b) {
  const qiv* x = (const qiv*)a;
  const qiv* y = (const qiv*)b;
  if (x->ref != y->ref) return x->ref < y->ref ? -1 : 1;
  if (x->start != y->start) return x->start < y->start ? -1 : 1;
  int32_t ex = qend(x->end), ey = qend(y->end);
  if (ex != ey) return ex < ey ? -1 : 1;
  return 0;
}

int64_t dqo_optimize_intervals(int32_t* ref, int32_t* start, int32_t* end, int64_t n) {
  if (n <= 0) return 0;
  qiv* v = (qiv*)malloc(sizeof(qiv) * (size_t)n);
  for (int64_t i = 0; i < n; i++) { v[i].ref = ref[i]; v[i].start = start[i]; v[i].end = end[i]; }
  qsort(v, (size_t)n, sizeof(qiv), qcmp);
  int64_t m = 0;
  qiv prev = v[0];
  for (int64_t i = 1; i < n; i++) {
    qiv nx = v[i];
    int same = prev.ref == nx.ref;
    int64_t pe = qend(prev.end), ne = qend(nx.end);
    int ovl = same && prev.start <= ne && nx.start <= pe;
    int abut = same && (pe + 1 == nx.start || ne + 1 == prev.start);
    if (ovl || abut) {
      if (ne > pe) prev.end = nx.end;
    } else {
      ref[m] = prev.ref; start[m] = prev.start; end[m] = prev.end; m++;
      prev = nx;
    }
  }
  ref[m] = prev.ref; start[m] = prev.start; end[m] = prev.end; m++;
  free(v);
  return m;
}

/* BAMQueryMultipleIntervalsIteratorFilter.compareIntervalToRecord with contained=false: a record
 * matches iff some interval is neither BEFORE nor AFTER it.  The filter's running interval index
 * only skips intervals that are BEFORE every later record of a coordinate-sorted file, so the
 * stateless test below selects the same records. */
int dqo_record_overlaps(const dqo_rec* r, const int32_t* ref, const int32_t* start,
                        const int32_t* end, int64_t n) {
  int32_t astart = r->pos + 1;
  int32_t aend = ((r->flag & 4) && astart != 0) ? astart : r->align_end;
  for (int64_t i = 0; i < n; i++) {
    if (ref[i] != r->ref_id) continue;
    int32_t ie = qend(end[i]);
    if (ie < astart) continue;      /* BEFORE */
    if (aend < start[i]) continue;  /* AFTER */
    return 1;
  }
  return 0;
}

/* ------------------------------------------------------------------ whole-file inflate */
int64_t dqo_inflate_file(dqo_file* f, uint8_t* out, int64_t cap) {
  rdr r;
  if (rdr_init(&r, f)) { rdr_free(&r); return DQO_ENOMEM; }
  int64_t addr = 0, n = 0;
  while (addr < f->len) {
    blkbuf* b;
    int e = rdr_load(&r, addr, &b);
    if (e) { n = e == R_FORMAT ? DQO_EFORMAT : DQO_EIO; break; }
    if (out) {
      if (n + b->len > cap) { n = DQO_EINVAL; break; }
      memcpy(out + n, b->data, (size_t)b->len);
    }
    n += b->len;
    addr += b->csize;
  }
  rdr_free(&r);
  return n;
}

/* ------------------------------------------------------------------ CPU baseline */
typedef struct {
  const uint8_t* data;
  int64_t len;
  int64_t base, file_len;   /* a shard window (dqo_run_partitions_window); base 0 otherwise */
  const uint8_t* header;    /* its decompressed header, or NULL: read from the file */
  int64_t header_len;
  const int64_t* starts;
  const int64_t* ends;
  int64_t n;
  int64_t* counts;
  uint64_t* digests;
  int64_t* ubytes;
  int64_t next;
  pthread_mutex_t mu;
  int err, short_window;
} job_t;

static void* worker(void* arg) {
  job_t* j = (job_t*)arg;
  dqo_file* f = j->header ? dqo_open_window(j->data, j->base, j->len, j->file_len)
                          : dqo_open_mem(j->data, j->len, 0);
  int32_t nr;
  uint64_t first;
  int32_t dummy;
  if (j->header ? dqo_set_header(f, j->header, j->header_len) != 0
                : dqo_read_header(f, &nr, &first, &dummy, 0) != 0) {
    j->err = 1;
    dqo_close(f);
    return NULL;
  }
  rdr r;
  rdr_init(&r, f);
  uint8_t* buf = NULL;
  int64_t bufcap = 0;
  for (;;) {
    pthread_mutex_lock(&j->mu);
    int64_t i = j->next++;
    pthread_mutex_unlock(&j->mu);
    if (i >= j->n) break;
    uint64_t vs, ve;
    int64_t cnt = 0, ub = 0;
    uint64_t dig = 0;
    int res = first_read(&r, j->starts[i], j->ends[i], &vs, &ve);
    if (res < 0) { j->err = 1; break; }
    if (res == 1 && rdr_seek(&r, vs) == 0) {
      for (;;) {
        uint64_t v = rdr_ptr(&r);
        if (v >= ve) break;
        int32_t bs;
        int rr = read_record(&r, &buf, &bufcap, &bs);
        if (rr <= 0) { if (rr < 0) j->err = 1; break; }
        uint64_t h = dqo_record_hash(buf, 4 + (int64_t)bs);
        dig += mix64(h + ((uint64_t)cnt + 1) * 0x9E3779B97F4A7C15ULL);
        cnt++;
        ub += 4 + (int64_t)bs;
      }
    }
    j->counts[i] = cnt;
    j->digests[i] = dig;
    if (j->ubytes) j->ubytes[i] = ub;
  }
  if (f->short_window) j->short_window = 1;
  free(buf);
  rdr_free(&r);
  dqo_close(f);
  return NULL;
}

int dqo_run_partitions(const uint8_t* data, int64_t len, const int64_t* starts,
                       const int64_t* ends, int64_t n, int nthreads, int64_t* counts,
                       uint64_t* digests, int64_t* ubytes) {
  if (nthreads < 1) nthreads = 1;
  job_t j;
  memset(&j, 0, sizeof j);
  j.data = data; j.len = len; j.starts = starts; j.ends = ends; j.n = n;
  j.counts = counts; j.digests = digests; j.ubytes = ubytes;
  pthread_mutex_init(&j.mu, NULL);
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
  for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, worker, &j);
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  free(th);
  pthread_mutex_destroy(&j.mu);
  return j.err ? DQO_EFORMAT : 0;
}

/* dqo_run_partitions over a shard window: bytes [base, base + len) of a file of file_len bytes
 * whose decompressed header is `header` (the multi-GPU bench's per-rank parity: a rank's resident
 * bytes plus its halo).  Returns DQO_ESHORT when some partition needed bytes past the window. */
int dqo_run_partitions_window(const uint8_t* data, int64_t base, int64_t len, int64_t file_len,
                              const uint8_t* header, int64_t header_len, const int64_t* starts,
                              const int64_t* ends, int64_t n, int nthreads, int64_t* counts,
                              uint64_t* digests, int64_t* ubytes) {
  if (nthreads < 1) nthreads = 1;
  if (!header || base < 0 || len < 0 || base + len > file_len) return DQO_EINVAL;
  job_t j;
  memset(&j, 0, sizeof j);
  j.data = data; j.len = len; j.base = base; j.file_len = file_len;
  j.header = header; j.header_len = header_len;
  j.starts = starts; j.ends = ends; j.n = n;
  j.counts = counts; j.digests = digests; j.ubytes = ubytes;
  pthread_mutex_init(&j.mu, NULL);
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
  for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, worker, &j);
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  free(th);
  pthread_mutex_destroy(&j.mu);
  return j.short_window ? DQO_ESHORT : j.err ? DQO_EFORMAT : 0;
}

/* ------------------------------------------------------------------ interval traversal, all
 * partitions (bench-scale parity of the GPU span runs): per partition, the records of the .bai span
 * of the optimized intervals clipped to the partition chunk (AbstractBinarySamSource.java:102-112;
 * spans = 0 reads the whole chunk) that overlap an interval (the filter of :113-115), then, when
 * asked, the unplaced-unmapped tail of the partition holding the start of the last linear bin
 * (:116-129).  q = optimized intervals (sorted, disjoint per reference), so the overlap test is a
 * binary search equal to dqo_record_overlaps.  Per-partition count + ordered digest, as
 * dqo_run_partitions. */
typedef struct {
  const uint8_t* data;
  int64_t len;
  const int64_t *starts, *ends;
  int64_t n;
  const uint8_t* bai;
  int64_t bai_len;
  const int32_t *qr, *qs, *qe;
  int64_t nq;
  int unplaced, spans;
  int64_t solb, ncc;
  int64_t* counts;
  uint64_t* digests;
  int64_t next;
  pthread_mutex_t mu;
  int err;
} tjob_t;

static int q_overlaps(const tjob_t* j, const dqo_rec* r) {
  const int32_t astart = r->pos + 1;
  const int32_t aend = ((r->flag & 4) && astart != 0) ? astart : r->align_end;
  /* first interval of r's reference whose end >= astart */
  int64_t lo = 0, hi = j->nq;
  while (lo < hi) {
    const int64_t mid = (lo + hi) / 2;
    if (j->qr[mid] < r->ref_id || (j->qr[mid] == r->ref_id && qend(j->qe[mid]) < astart)) lo = mid + 1;
    else hi = mid;
  }
  return lo < j->nq && j->qr[lo] == r->ref_id && j->qs[lo] <= aend;
}

static void* tworker(void* arg) {
  tjob_t* j = (tjob_t*)arg;
  dqo_file* f = dqo_open_mem(j->data, j->len, 0);
  int32_t nr, dummy;
  uint64_t first;
  if (dqo_read_header(f, &nr, &first, &dummy, 0) != 0) {
    j->err = 1;
    dqo_close(f);
    return NULL;
  }
  rdr r;
  rdr_init(&r, f);
  uint8_t* buf = NULL;
  int64_t bufcap = 0, spcap = 0;
  uint64_t *sb = NULL, *se = NULL;
  for (;;) {
    pthread_mutex_lock(&j->mu);
    int64_t i = j->next++;
    pthread_mutex_unlock(&j->mu);
    if (i >= j->n) break;
    uint64_t vs, ve;
    int64_t cnt = 0;
    uint64_t dig = 0;
    int res = first_read(&r, j->starts[i], j->ends[i], &vs, &ve);
    if (res < 0) { j->err = 1; break; }
    if (res == 1) {
      /* the chunks to read: the clipped span, or the whole chunk */
      int64_t nsp = 1;
      if (j->nq > 0 && j->spans) {
        nsp = dqo_bai_span(j->bai, j->bai_len, j->qr, j->qs, j->qe, j->nq, vs, ve, NULL, NULL, 0);
        if (nsp < 0) { j->err = 1; break; }
      }
      if (nsp > spcap) {
        spcap = nsp + 16;
        sb = (uint64_t*)realloc(sb, sizeof(uint64_t) * (size_t)spcap);
        se = (uint64_t*)realloc(se, sizeof(uint64_t) * (size_t)spcap);
      }
      if (j->nq > 0 && j->spans) dqo_bai_span(j->bai, j->bai_len, j->qr, j->qs, j->qe, j->nq, vs, ve, sb, se, nsp);
      else { sb[0] = vs; se[0] = ve; }
      for (int64_t k = 0; j->nq > 0 && k < nsp; k++) {
        if (rdr_seek(&r, sb[k]) != 0) continue;
        for (;;) {
          uint64_t v = rdr_ptr(&r);
          if (v >= se[k]) break;
          int32_t bs;
          int rr = read_record(&r, &buf, &bufcap, &bs);
          if (rr <= 0) { if (rr < 0) j->err = 1; break; }
          dqo_rec rec;
          fill_rec(&rec, v, buf, bs);
          if (!q_overlaps(j, &rec)) continue;
          dig += mix64(rec.hash + ((uint64_t)cnt + 1) * 0x9E3779B97F4A7C15ULL);
          cnt++;
        }
      }
      if (j->unplaced && j->solb != -1 && j->ncc >= 1 && vs <= (uint64_t)j->solb &&
          (uint64_t)j->solb < ve && rdr_seek(&r, (uint64_t)j->solb) == 0) {
        int skipping = 1;  /* BAMFileIndexUnmappedIterator */
        for (;;) {
          uint64_t v = rdr_ptr(&r);
          int32_t bs;
          int rr = read_record(&r, &buf, &bufcap, &bs);
          if (rr <= 0) { if (rr < 0) j->err = 1; break; }
          if (skipping && rd32(buf + 4) != -1) continue;
          skipping = 0;
          (void)v;
          uint64_t h = dqo_record_hash(buf, 4 + (int64_t)bs);
          dig += mix64(h + ((uint64_t)cnt + 1) * 0x9E3779B97F4A7C15ULL);
          cnt++;
        }
      }
    }
    j->counts[i] = cnt;
    j->digests[i] = dig;
  }
  free(sb);
  free(se);
  free(buf);
  rdr_free(&r);
  dqo_close(f);
  return NULL;
}

int dqo_run_partitions_traversal(const uint8_t* data, int64_t len, const int64_t* starts,
                                 const int64_t* ends, int64_t n, int nthreads,
                                 const uint8_t* bai, int64_t bai_len, const int32_t* q_ref,
                                 const int32_t* q_start, const int32_t* q_end, int64_t nq,
                                 int unplaced, int spans, int64_t* counts, uint64_t* digests) {
  if (nthreads < 1) nthreads = 1;
  tjob_t j;
  memset(&j, 0, sizeof j);
  j.data = data; j.len = len; j.starts = starts; j.ends = ends; j.n = n;
  j.bai = bai; j.bai_len = bai_len; j.qr = q_ref; j.qs = q_start; j.qe = q_end; j.nq = nq;
  j.unplaced = unplaced; j.spans = spans; j.counts = counts; j.digests = digests;
  int32_t nref;
  if (dqo_bai_info(bai, bai_len, &nref, &j.solb, &j.ncc) != 0) return DQO_EFORMAT;
  pthread_mutex_init(&j.mu, NULL);
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
  for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, tworker, &j);
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  free(th);
  pthread_mutex_destroy(&j.mu);
  return j.err ? DQO_EFORMAT : 0;
}

/* ================================================================== BGZF text (VCF) path
 * TextInputFormat over a BGZF file with Disq's splittable codecs: per split, the lines Hadoop's
 * LineRecordReader returns.  Restated, as a literal simulation:
 *   D/impl/formats/bgzf/BGZFCodec.java:57-68 (and BGZFEnhancedGzipCodec.java:41-74 for BGZF
 *     data): adjustedStart = guessNextBGZFPos(start, end).pos, or end when there is none;
 *   D/impl/formats/bgzf/BGZFSplitCompressionInputStream.java:14-106: reads within one block;
 *     at a block end it reports END_OF_BLOCK, then returns ONE byte of the next block and
 *     advertises getPos = adjustedStart + (block address relative to adjustedStart) + 1;
 *   htsjdk 2.16.0 BlockCompressedInputStream (stream mode; not vendored): available(),
 *     endOfBlock(), getPosition() with the end-of-block pointer normalisation;
 *   Hadoop 2.7 (not vendored): LineRecordReader.initialize/nextKeyValue/skipUtfByteOrderMark,
 *     CompressedSplitLineReader.fillBuffer/readLine/needAdditionalRecordAfterSplit,
 *     LineReader.readDefaultLine (CR, LF and CRLF terminators) with io.file.buffer.size = 4096;
 *   D/impl/formats/vcf/VcfSource.java:103-113: lines starting with '#' are dropped. */
#define TX_BUF 4096
typedef struct {
  rdr r;              /* block loader (inflate_block) */
  int64_t start_pos;  /* adjustedStart: stream address 0 */
  int have;           /* mCurrentBlock != null */
  int64_t addr;       /* absolute address of the current block */
  int32_t csize, len, off;
  const uint8_t* data;
  int64_t processed;  /* processedPosition (relative) */
  int64_t cpos;       /* compressedStreamPosition */
  int advertise;
  int64_t u_base;     /* absolute decompressed offset of the current block's first byte */
  const int64_t* chain_pos; const int64_t* chain_u; int64_t nchain;
  int err;
} tstream;

static int64_t tx_u_of(tstream* t, int64_t addr) {
  int64_t lo = 0, hi = t->nchain;
  while (lo < hi) {
    int64_t m = (lo + hi) / 2;
    if (t->chain_pos[m] < addr) lo = m + 1; else hi = m;
  }
  if (lo < t->nchain && t->chain_pos[lo] == addr) return t->chain_u[lo];
  return -1;
}

/* BlockCompressedInputStream.readBlock: the next block at the stream position */
static int tx_read_block(tstream* t) {
  int64_t a = t->have ? t->addr + t->csize : t->start_pos;
  blkbuf* b;
  int e = rdr_load(&t->r, a, &b);
  if (e) { t->err = e == R_FORMAT ? DQO_EFORMAT : DQO_EIO; return -1; }
  t->have = 1;
  t->r.cur = b;  /* keep it cached while other blocks load */
  t->addr = a;
  t->csize = b->csize;
  t->len = b->len;
  t->off = 0;
  t->data = b->data;
  if (b->len > 0) {
    t->u_base = tx_u_of(t, a);
    if (t->u_base < 0) { set_err(t->r.f, "text block off the BGZF chain"); t->err = DQO_EFORMAT; return -1; }
  }
  return 0;
}
static int tx_available(tstream* t) {
  if (!t->have || t->off == t->len)
    if (tx_read_block(t)) return -1;
  return t->len - t->off;
}
static int tx_end_of_block(const tstream* t) { return t->have && t->off == t->len; }
static int64_t tx_position_block(const tstream* t) { /* getPosition() >> 16, relative */
  if (!t->have) return 0;
  if (t->off > 0 && t->off == t->len) return t->addr + t->csize - t->start_pos;
  return t->addr - t->start_pos;
}
/* readWithinBlock: n > 0 bytes, -1 end of stream, -2 end of block; *u0 = offset of byte 0 */
static int tx_read_within(tstream* t, uint8_t* dst, int n, int64_t* u0) {
  if (tx_end_of_block(t)) {
    int av = tx_available(t);
    if (av < 0) return -3;
    t->processed = tx_position_block(t);
    return av == 0 ? -1 : -2;
  }
  int av = tx_available(t);
  if (av < 0) return -3;
  int k = av < n ? av : n;
  if (k == 0) return 0;  /* an empty first block: read(b, off, 0) == 0, EOF to LineReader */
  memcpy(dst, t->data + t->off, (size_t)k);
  *u0 = t->u_base + t->off;
  t->off += k;
  return k;
}
/* BGZFSplitCompressionInputStream.read(b, 0, n) */
static int tx_read(tstream* t, uint8_t* dst, int n, int64_t* u0) {
  int res = tx_read_within(t, dst, n, u0);
  if (res == -3) return -3;
  if (res == -2) t->advertise = 1;
  if (t->advertise) {
    res = tx_read_within(t, dst, 1, u0);
    if (res == -3) return -3;
    t->cpos = t->start_pos + t->processed + 1;
    t->advertise = 0;
  }
  return res;
}

typedef struct {
  tstream* s;
  uint8_t buf[TX_BUF];
  int64_t bu0;        /* absolute decompressed offset of buf[0] */
  int blen, bpos;
  int need_additional, finished;
  int64_t end;        /* getAdjustedEnd */
} lreader;

static int lr_fill(lreader* L, int in_delim) {
  int64_t u0 = 0;
  int n = tx_read(L->s, L->buf, TX_BUF, &u0);
  if (n == -3) return -3;
  if (n > 0) L->bu0 = u0;
  if (in_delim && n > 0) L->need_additional = L->buf[0] != '\n';
  return n;
}

typedef struct {
  int64_t start;      /* absolute decompressed offset of the line's first byte (-1: none) */
  int64_t len;        /* value length (terminator excluded) */
  uint8_t head[3];    /* the value's first bytes */
  int nhead;
} tline;

/* LineReader.readDefaultLine (maxLineLength, maxBytesToConsume = Integer.MAX_VALUE): returns the
 * bytes consumed; the value is the line's first `len` bytes. */
static int64_t lr_read_line(lreader* L, tline* o) {
  int64_t consumed = 0;
  int nl_len = 0, prev_cr = 0;
  o->start = -1;
  o->len = 0;
  o->nhead = 0;
  do {
    int startp = L->bpos;
    if (L->bpos >= L->blen) {
      startp = L->bpos = 0;
      if (prev_cr) ++consumed;
      L->blen = lr_fill(L, prev_cr);
      if (L->blen == -3) return -3;
      if (L->blen <= 0) break;
    }
    if (o->start < 0) o->start = L->bu0 + startp;
    for (; L->bpos < L->blen; ++L->bpos) {
      if (L->buf[L->bpos] == '\n') { nl_len = prev_cr ? 2 : 1; ++L->bpos; break; }
      if (prev_cr) { nl_len = 1; break; }
      prev_cr = L->buf[L->bpos] == '\r';
    }
    int rl = L->bpos - startp;
    if (prev_cr && nl_len == 0) --rl;
    consumed += rl;
    int app = rl - nl_len;
    for (int i = 0; i < app && o->nhead < 3; i++) o->head[o->nhead++] = L->buf[startp + i];
    if (app > 0) o->len += app;
  } while (nl_len == 0);
  return consumed;
}
/* CompressedSplitLineReader.readLine */
static int64_t csl_read_line(lreader* L, tline* o) {
  if (L->finished) { o->start = -1; o->len = 0; o->nhead = 0; return 0; }
  if (L->s->cpos > L->end) L->finished = 1;
  return lr_read_line(L, o);
}

/* Block chain of a whole BGZF file: positions and decompressed offsets (test helper). */
static int64_t tx_chain(dqo_file* f, int64_t** pos, int64_t** uo) {
  int64_t cap = f->len / 26 + 2, n = 0, u = 0, a = 0;
  *pos = (int64_t*)malloc(sizeof(int64_t) * (size_t)cap);
  *uo = (int64_t*)malloc(sizeof(int64_t) * (size_t)cap);
  if (!*pos || !*uo) return DQO_ENOMEM;
  while (a + 18 <= f->len && n < cap) {
    const uint8_t* h = f->data + a;
    if (h[0] != 0x1f || h[1] != 0x8b) break;
    int32_t cs = rd16(h + 16) + 1;
    if (cs < 26 || a + cs > f->len) break;
    (*pos)[n] = a;
    (*uo)[n] = u;
    u += rd32(h + cs - 4);
    n++;
    a += cs;
  }
  return n;
}

/* The lines of split [start, end): value offsets (absolute in the decompressed stream) and
 * lengths, in order; drop_hash drops values starting with '#' (VcfSource.java:108).  Returns the
 * count (entries written up to cap) or a negative DQO_ error. */
int64_t dqo_text_split_lines(dqo_file* f, int64_t start, int64_t end, int drop_hash,
                             int64_t* vstart, int64_t* vlen, int64_t cap) {
  int64_t *cp = NULL, *cu = NULL;
  int64_t nchain = tx_chain(f, &cp, &cu);
  tstream* t = (tstream*)calloc(1, sizeof(tstream));
  lreader* L = (lreader*)calloc(1, sizeof(lreader));
  int64_t n = 0;
  if (nchain < 0) { n = nchain; goto out; }
  if (!t || !L || rdr_init(&t->r, f)) { n = DQO_ENOMEM; goto out; }
  t->chain_pos = cp; t->chain_u = cu; t->nchain = nchain;
  {
    /* BGZFCodec.createInputStream */
    int64_t gp = 0; int32_t gc = 0, gu = 0;
    const int64_t adj = dqo_guess_next_bgzf(f, start, end, &gp, &gc, &gu) ? gp : end;
    t->start_pos = adj;
    t->cpos = adj;  /* updatePos(false), processedPosition 0 */
    L->s = t;
    L->end = end;
    tline ln;
    int64_t pos = adj;
    /* LineRecordReader.initialize: start = adjustedStart; unless 0, the first line is dropped */
    if (adj != 0) {
      int64_t k = csl_read_line(L, &ln);
      if (k < 0) { n = t->err ? t->err : DQO_EFORMAT; goto out; }
      pos += k;
    }
    /* one nextKeyValue call per iteration */
    for (;;) {
      if (!(t->cpos <= end || (!L->finished && L->need_additional))) break;
      int64_t k = csl_read_line(L, &ln);
      if (k < 0) { n = t->err ? t->err : DQO_EFORMAT; goto out; }
      int64_t vs = ln.start, vl = ln.len;
      const uint8_t* hd = ln.head;
      int nh = ln.nhead;
      if (pos == 0 && vl >= 3 && hd[0] == 0xEF && hd[1] == 0xBB && hd[2] == 0xBF) {
        vs += 3;  /* skipUtfByteOrderMark */
        vl -= 3;
        k -= 3;
        hd += 3;
        nh = 0;
      }
      pos += k;
      if (k == 0) break;
      if (drop_hash && vl > 0) {
        uint8_t c0;
        if (nh > 0) c0 = hd[0];
        else { /* after a BOM: the value's first byte */
          int64_t lo = 0, hi = nchain;
          while (lo + 1 < hi) { int64_t m = (lo + hi) / 2; if (cu[m] <= vs) lo = m; else hi = m; }
          blkbuf* b;
          if (rdr_load(&t->r, cp[lo], &b)) { n = DQO_EFORMAT; goto out; }
          c0 = b->data[vs - cu[lo]];
        }
        if (c0 == '#') continue;
      }
      if (vstart && n < cap) { vstart[n] = vs; vlen[n] = vl; }
      n++;
    }
  }
out:
  if (t) rdr_free(&t->r);
  free(t); free(L); free(cp); free(cu);
  return n;
}
