// synth_bam.cpp -- deterministic synthetic coordinate-sorted BAM generator (+ .bai, .sbi).
//
// Workload generator for tests and bench.py, not part of the read
// path.  Output follows the htsjdk writer conventions the reference fixtures show:
//   * BGZF blocks of 65498 uncompressed bytes (1.bam block 0: cSize 14146, uSize 65498), records
//     straddling block boundaries, raw deflate level 5 (htsjdk Defaults.COMPRESSION_LEVEL),
//     XLEN = 6 with the BC subfield first, and the 28-byte EOF block;
//   * .sbi in the layout of H/SBIIndexWriter.java:120-151;
//   * .bai with bins, chunks, a 16 kb linear index and the trailing n_no_coor (SAMv1 §5.2).
// Chunks of records are generated and compressed on independent threads; each chunk starts a new
// BGZF block (as htslib's writer does at flush points), so only a chunk's last block is short.
#include <zlib.h>

#include <algorithm>
#include <cmath>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "../../include/disq_synth.h"

namespace {

constexpr int kBlockU = 65498;

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed) {}
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
  }
  uint32_t u32(uint32_t n) { return (uint32_t)((next() >> 32) * n >> 32); }
  double unif() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
};

// SAMv1 reg2bin for [beg, end) 0-based.
int reg2bin(int beg, int end) {
  --end;
  if (beg >> 14 == end >> 14) return ((1 << 15) - 1) / 7 + (beg >> 14);
  if (beg >> 17 == end >> 17) return ((1 << 12) - 1) / 7 + (beg >> 17);
  if (beg >> 20 == end >> 20) return ((1 << 9) - 1) / 7 + (beg >> 20);
  if (beg >> 23 == end >> 23) return ((1 << 6) - 1) / 7 + (beg >> 23);
  if (beg >> 26 == end >> 26) return ((1 << 3) - 1) / 7 + (beg >> 26);
  return 0;
}

struct Ref {
  std::string name;
  int32_t len;
};

std::vector<Ref> grch38_dict() {
  static const int32_t L[24] = {248956422, 242193529, 198295559, 190214555, 181538259, 170805979,
                                159345973, 145138636, 138394717, 133797422, 135086622, 133275309,
                                114364328, 107043718, 101991189, 90338345,  83257441,  80373285,
                                58617616,  64444167,  46709983,  50818468,  156040895, 57227415};
  std::vector<Ref> d;
  for (int i = 0; i < 24; i++) {
    std::string n = i < 22 ? "chr" + std::to_string(i + 1) : (i == 22 ? "chrX" : "chrY");
    d.push_back({n, L[i]});
  }
  return d;
}

// SAMRecordSetBuilder's default dictionary: chr1..chr22, chrX, chrY, chrM (chr21 is index 20, as
// T/HtsjdkReadsRddTest.java:170 relies on).
std::vector<Ref> anysam_dict() {
  std::vector<Ref> d;
  for (int i = 1; i <= 22; i++) d.push_back({"chr" + std::to_string(i), 101000000});
  d.push_back({"chrX", 101000000});
  d.push_back({"chrY", 101000000});
  d.push_back({"chrM", 101000000});
  return d;
}

struct Rec {  // staged record (bytes) plus index facts
  int32_t ref, beg, end;  // end exclusive, for binning
  bool mapped;
};

void put32(std::vector<uint8_t>& o, int32_t v) {
  uint8_t b[4] = {(uint8_t)v, (uint8_t)(v >> 8), (uint8_t)(v >> 16), (uint8_t)(v >> 24)};
  o.insert(o.end(), b, b + 4);
}

struct CigarOp {
  uint32_t len;
  char op;
};

uint32_t op_code(char c) {
  const char* s = "MIDNSHP=X";
  return (uint32_t)(strchr(s, c) - s);
}

int ref_len_of(const std::vector<CigarOp>& c) {
  int n = 0;
  for (auto& o : c)
    if (o.op == 'M' || o.op == 'D' || o.op == 'N' || o.op == '=' || o.op == 'X') n += o.len;
  return n;
}

// Append one BAM record; returns its reference span facts.
Rec emit_record(std::vector<uint8_t>& out, const std::string& name, int32_t ref, int32_t pos,
                uint8_t mapq, uint16_t flag, const std::vector<CigarOp>& cigar, int l_seq,
                const uint8_t* seq4, const uint8_t* qual, int32_t nref, int32_t npos, int32_t tlen,
                const std::vector<uint8_t>& aux) {
  bool mapped = !(flag & 4);
  int rl = mapped ? ref_len_of(cigar) : 0;
  int beg = pos, end = mapped ? pos + (rl > 0 ? rl : 1) : pos + 1;
  int bin = reg2bin(beg < 0 ? 0 : beg, end <= 0 ? 1 : end);
  if (ref < 0) bin = 4680;  // reg2bin(-1, 0)
  int32_t lrn = (int32_t)name.size() + 1;
  int32_t bs = 32 + lrn + 4 * (int32_t)cigar.size() + (l_seq + 1) / 2 + l_seq + (int32_t)aux.size();
  put32(out, bs);
  put32(out, ref);
  put32(out, pos);
  put32(out, (int32_t)((uint32_t)bin << 16 | (uint32_t)mapq << 8 | (uint32_t)lrn));
  put32(out, (int32_t)((uint32_t)flag << 16 | (uint32_t)cigar.size()));
  put32(out, l_seq);
  put32(out, nref);
  put32(out, npos);
  put32(out, tlen);
  out.insert(out.end(), name.begin(), name.end());
  out.push_back(0);
  for (auto& c : cigar) put32(out, (int32_t)(c.len << 4 | op_code(c.op)));
  out.insert(out.end(), seq4, seq4 + (l_seq + 1) / 2);
  out.insert(out.end(), qual, qual + l_seq);
  out.insert(out.end(), aux.begin(), aux.end());
  return Rec{ref, beg, end, mapped && ref >= 0};
}

void aux_z(std::vector<uint8_t>& a, const char* tag, const std::string& v) {
  a.push_back(tag[0]);
  a.push_back(tag[1]);
  a.push_back('Z');
  a.insert(a.end(), v.begin(), v.end());
  a.push_back(0);
}
void aux_i(std::vector<uint8_t>& a, const char* tag, int v) {
  a.push_back(tag[0]);
  a.push_back(tag[1]);
  if (v >= 0 && v < 256) {
    a.push_back('C');
    a.push_back((uint8_t)v);
  } else {
    a.push_back('i');
    put32(a, v);
  }
}

std::string cigar_str(const std::vector<CigarOp>& c) {
  std::string s;
  for (auto& o : c) s += std::to_string(o.len) + o.op;
  return s;
}

// Illumina-like binned qualities with a first-order Markov chain.
void gen_qual(Rng& r, uint8_t* q, int n) {
  static const uint8_t bins[4] = {2, 12, 23, 37};
  int st = 3;
  for (int i = 0; i < n; i++) {
    double u = r.unif();
    if (u < 0.08) st = (int)r.u32(4);
    else if (u < 0.12 && st > 0) st--;
    else if (u < 0.20 && st < 3) st++;
    if (i > n - 10 && r.unif() < 0.1 && st > 0) st--;
    q[i] = bins[st];
  }
}

void gen_seq(Rng& r, uint8_t* s4, int n) {
  static const uint8_t code[5] = {1, 2, 4, 8, 15};  // A C G T N
  for (int i = 0; i < (n + 1) / 2; i++) s4[i] = 0;
  for (int i = 0; i < n; i++) {
    uint32_t x = r.u32(1000);
    uint8_t b = x == 0 ? code[4] : code[x & 3];
    s4[i / 2] |= (uint8_t)(i & 1 ? b : b << 4);
  }
}

struct Chunk {
  std::vector<uint8_t> comp;          // compressed blocks
  std::vector<int32_t> blk_csize;     // per block
  std::vector<int32_t> blk_usize;
  // index facts (only when indexing): per record (local block, offset) and span
  std::vector<uint32_t> rec_blk;
  std::vector<uint16_t> rec_off;
  std::vector<Rec> recs;
  uint32_t end_blk = 0;  // position right after the last record
  uint16_t end_off = 0;
  int64_t n_records = 0;
  int64_t ubytes = 0;
};

int compress_block(z_stream* zs, const uint8_t* src, int n, std::vector<uint8_t>& out,
                   int level) {
  uint8_t tmp[65536 + 1024];
  deflateReset(zs);
  zs->next_in = (Bytef*)src;
  zs->avail_in = (uInt)n;
  zs->next_out = tmp + 18;
  zs->avail_out = 65536 - 26;
  int rc = deflate(zs, Z_FINISH);
  int clen;
  if (rc != Z_STREAM_END) {  // did not fit: store uncompressed (htsjdk's noCompressionDeflater)
    z_stream z0;
    memset(&z0, 0, sizeof z0);
    deflateInit2(&z0, 0, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY);
    z0.next_in = (Bytef*)src;
    z0.avail_in = (uInt)n;
    z0.next_out = tmp + 18;
    z0.avail_out = 65536 - 26;
    if (deflate(&z0, Z_FINISH) != Z_STREAM_END) {
      deflateEnd(&z0);
      return -1;
    }
    clen = (int)(65536 - 26 - z0.avail_out);
    deflateEnd(&z0);
  } else {
    clen = (int)(65536 - 26 - zs->avail_out);
  }
  (void)level;
  int bsize = clen + 26;
  static const uint8_t hdr[16] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 'B', 'C', 2, 0};
  memcpy(tmp, hdr, 16);
  tmp[16] = (uint8_t)((bsize - 1) & 0xff);
  tmp[17] = (uint8_t)((bsize - 1) >> 8);
  uint32_t crc = (uint32_t)crc32(0L, src, (uInt)n);
  uint8_t* t = tmp + 18 + clen;
  for (int i = 0; i < 4; i++) t[i] = (uint8_t)(crc >> (8 * i));
  for (int i = 0; i < 4; i++) t[4 + i] = (uint8_t)((uint32_t)n >> (8 * i));
  out.insert(out.end(), tmp, tmp + bsize);
  return bsize;
}

struct Gen {
  dq_synth_opts o;
  std::vector<Ref> dict;
  std::vector<uint8_t> header;  // uncompressed BAM header
  int64_t total_records = 0;    // mapped + unplaced
  int64_t n_unplaced = 0;
  int64_t per_chunk = 0;
  int64_t n_chunks = 0;
  double spacing = 5.0;         // short-read genome offset step
};

void build_header(Gen& g) {
  std::string text = "@HD\tVN:1.6\tSO:coordinate\n";
  for (auto& r : g.dict) text += "@SQ\tSN:" + r.name + "\tLN:" + std::to_string(r.len) + "\n";
  text += "@RG\tID:grp1\tSM:synthetic\tPL:ILLUMINA\n@PG\tID:disq_amd_synth\tPN:synth_bam\n";
  auto& h = g.header;
  h.insert(h.end(), {'B', 'A', 'M', 1});
  put32(h, (int32_t)text.size());
  h.insert(h.end(), text.begin(), text.end());
  put32(h, (int32_t)g.dict.size());
  for (auto& r : g.dict) {
    put32(h, (int32_t)r.name.size() + 1);
    h.insert(h.end(), r.name.begin(), r.name.end());
    h.push_back(0);
    put32(h, r.len);
  }
}

// Genome layout for the WGS shapes: record i sits at genome offset i*spacing (+jitter < spacing).
void locate(const std::vector<Ref>& d, int64_t g, int32_t* ref, int32_t* pos) {
  for (size_t i = 0; i < d.size(); i++) {
    if (g < d[i].len - 200000) {
      *ref = (int32_t)i;
      *pos = (int32_t)g;
      return;
    }
    g -= d[i].len - 200000;
  }
  *ref = (int32_t)d.size() - 1;
  *pos = d.back().len - 200000;
}

// Generate the uncompressed records [r0, r1) of the global sequence into `u`.
void gen_records(const Gen& g, int64_t r0, int64_t r1, std::vector<uint8_t>& u,
                 std::vector<Rec>* recs, std::vector<int64_t>* rec_uoff) {
  const dq_synth_opts& o = g.o;
  std::vector<uint8_t> seq4, qual, aux;
  std::vector<CigarOp> cig;
  int64_t mapped_total = g.total_records - g.n_unplaced;
  for (int64_t i = r0; i < r1; i++) {
    Rng r(o.seed * 0x2545F4914F6CDD1DULL ^ (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ULL);
    aux.clear();
    cig.clear();
    if (rec_uoff) rec_uoff->push_back((int64_t)u.size());
    if (o.shape == DQ_SYNTH_ANYSAM) {
      // T/AnySamTestUtil.java:37-64 shape: numPairs pairs at chr21 (index 20),
      // start1=(i+1)*1000, start2=start1+100, read length 36; pair 5 -> two placed-unmapped
      // fragments; two unplaced-unmapped fragments at the end.  Records are in coordinate order.
      int64_t np = o.n_records / 2;  // here n_records = 2*numPairs (+2 unplaced handled below)
      int L = 36;
      seq4.assign(18, 0x11);
      qual.assign(L, 30);
      char nm[64];
      if (i < 2 * np) {
        int64_t pi = i / 2;
        int second = (int)(i & 1);
        int32_t s1 = (int32_t)((pi + 1) * 1000), s2 = s1 + 100;
        int32_t p = second ? s2 : s1;
        if (pi == 5) {
          snprintf(nm, sizeof nm, "test-read-%03lld-%d", (long long)pi, second + 1);
          emit_record(u, nm, 20, p - 1, 0, 4, cig, L, seq4.data(), qual.data(), -1, -1, 0, aux);
          if (recs) recs->push_back({20, p - 1, p, false});
        } else {
          snprintf(nm, sizeof nm, "test-read-%03lld", (long long)pi);
          cig.push_back({(uint32_t)L, 'M'});
          uint16_t flag = 1 | 2 | (second ? (16 | 128) : (32 | 64));
          int32_t mp = second ? s1 : s2;
          int32_t tl = second ? -(s2 + L - s1) : (s2 + L - s1);
          Rec rr = emit_record(u, nm, 20, p - 1, 255, flag, cig, L, seq4.data(), qual.data(), 20,
                               mp - 1, tl, aux);
          if (recs) recs->push_back(rr);
        }
      } else {
        snprintf(nm, sizeof nm, "test-read-%03lld-unplaced-unmapped", (long long)(np + (i - 2 * np)));
        emit_record(u, nm, -1, -1, 0, 4, cig, L, seq4.data(), qual.data(), -1, -1, 0, aux);
        if (recs) recs->push_back({-1, -1, 0, false});
      }
      continue;
    }
    // WGS-like shapes.
    bool unplaced = i >= mapped_total;
    int L;
    if (o.shape == DQ_SYNTH_LONGREAD) {
      double u1 = r.unif();
      double lg = (r.unif() < 0.01) ? (5.7 + u1 * 0.6) : (4.0 + u1 * 1.0);  // 10^4..10^5 / 0.5-2Mb
      L = (int)std::min(2000000.0, std::pow(10.0, lg));
    } else {
      L = 150;
    }
    seq4.resize((size_t)(L + 1) / 2);
    qual.resize((size_t)L);
    gen_seq(r, seq4.data(), L);
    gen_qual(r, qual.data(), L);
    char nm[64];
    snprintf(nm, sizeof nm, "SYN:%u:%u:%u:%u", 1 + r.u32(8), 1101 + r.u32(2200), r.u32(30000),
             r.u32(30000));
    aux_z(aux, "RG", "grp1");
    if (unplaced) {
      uint16_t flag = 1 | 4 | 8 | (i & 1 ? 128 : 64);
      Rec rr = emit_record(u, nm, -1, -1, 0, flag, cig, L, seq4.data(), qual.data(), -1, -1, 0, aux);
      if (recs) recs->push_back(rr);
      continue;
    }
    // genome offset floor(i * s) + jitter < floor(s): non-decreasing in i; s = 5 bp for short
    // reads, or less when the records would run past the genome (30x-WGS-sized files)
    const double s = o.shape == DQ_SYNTH_LONGREAD ? 30000.0 : g.spacing;
    const int64_t js = std::max<int64_t>(1, (int64_t)s);
    int32_t ref, pos;
    locate(g.dict, (int64_t)((double)i * s) + (int64_t)r.u32((uint32_t)js), &ref, &pos);
    int nm_edits = 0;
    if (o.shape == DQ_SYNTH_LONGREAD) {
      int left = L;
      while (left > 0) {
        int m = std::min(left, 50 + (int)r.u32(400));
        cig.push_back({(uint32_t)m, 'M'});
        left -= m;
        if (left <= 0) break;
        if (r.unif() < 0.5) {
          int ins = std::min(left, 1 + (int)r.u32(6));
          cig.push_back({(uint32_t)ins, 'I'});
          left -= ins;
        } else {
          cig.push_back({1 + r.u32(6), 'D'});
        }
        nm_edits++;
      }
    } else {
      double c = r.unif();
      if (c < 0.90) {
        cig.push_back({150, 'M'});
      } else if (c < 0.94) {
        uint32_t s = 5 + r.u32(40);
        cig.push_back({s, 'S'});
        cig.push_back({150 - s, 'M'});
      } else if (c < 0.97) {
        uint32_t a = 20 + r.u32(100);
        cig.push_back({a, 'M'});
        cig.push_back({1, 'I'});
        cig.push_back({149 - a, 'M'});
        nm_edits = 1;
      } else {
        uint32_t a = 20 + r.u32(100), dl = 1 + r.u32(4);
        cig.push_back({a, 'M'});
        cig.push_back({dl, 'D'});
        cig.push_back({150 - a, 'M'});
        nm_edits = 1;
      }
    }
    nm_edits += (int)r.u32(3);
    uint8_t mapq = o.shape == DQ_SYNTH_LONGREAD ? (uint8_t)(r.unif() < 0.8 ? 60 : r.u32(60))
                                                : (uint8_t)(r.unif() < 0.95 ? 60 : r.u32(60));
    int second = (int)(i & 1);
    int32_t ins = (int32_t)(350 + 50 * (r.unif() + r.unif() + r.unif() - 1.5) * 2);
    uint16_t flag = o.shape == DQ_SYNTH_LONGREAD ? (uint16_t)(r.unif() < 0.5 ? 16 : 0)
                                                 : (uint16_t)(1 | 2 | (second ? 16 | 128 : 32 | 64));
    int32_t nref = o.shape == DQ_SYNTH_LONGREAD ? -1 : ref;
    int32_t npos = o.shape == DQ_SYNTH_LONGREAD ? -1 : (second ? std::max(0, pos - ins + L) : pos + ins - L);
    int32_t tlen = o.shape == DQ_SYNTH_LONGREAD ? 0 : (second ? -ins : ins);
    aux_i(aux, "NM", nm_edits);
    std::string md = std::to_string(ref_len_of(cig));
    if (nm_edits) md = std::to_string(40 + r.u32(60)) + "A" + std::to_string(std::max(1, ref_len_of(cig) - 101));
    aux_z(aux, "MD", md);
    aux_i(aux, "AS", std::max(0, L - 5 * nm_edits));
    aux_i(aux, "XS", (int)r.u32(100));
    if (o.shape != DQ_SYNTH_LONGREAD) aux_z(aux, "MC", cigar_str(cig));
    Rec rr = emit_record(u, nm, ref, pos, mapq, flag, cig, L, seq4.data(), qual.data(), nref, npos,
                         tlen, aux);
    if (recs) recs->push_back(rr);
  }
}

void make_chunk(const Gen& g, int64_t k, Chunk& c, bool index) {
  std::vector<uint8_t> u;
  if (k == 0) u = g.header;
  int64_t r0 = k * g.per_chunk, r1 = std::min(g.total_records, r0 + g.per_chunk);
  std::vector<int64_t> uoff;
  size_t hdr = u.size();
  gen_records(g, r0, r1, u, index ? &c.recs : nullptr, index ? &uoff : nullptr);
  c.n_records = r1 - r0;
  c.ubytes = (int64_t)(u.size() - hdr);
  z_stream zs;
  memset(&zs, 0, sizeof zs);
  deflateInit2(&zs, g.o.level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY);
  size_t n = u.size();
  for (size_t off = 0; off < n; off += kBlockU) {
    int len = (int)std::min((size_t)kBlockU, n - off);
    int bs = compress_block(&zs, u.data() + off, len, c.comp, g.o.level);
    c.blk_csize.push_back(bs);
    c.blk_usize.push_back(len);
  }
  deflateEnd(&zs);
  if (index) {
    for (int64_t x : uoff) {
      c.rec_blk.push_back((uint32_t)(x / kBlockU));
      c.rec_off.push_back((uint16_t)(x % kBlockU));
    }
    // end pointer: normalised position after the last byte
    uint64_t endb = n / kBlockU, endo = n % kBlockU;
    c.end_blk = (uint32_t)endb;
    c.end_off = (uint16_t)endo;
  }
}

struct BinChunks {
  std::map<uint32_t, std::vector<std::pair<uint64_t, uint64_t>>> bins;
  std::vector<uint64_t> linear;
  uint64_t beg = UINT64_MAX, end = 0;
  uint64_t n_mapped = 0, n_unmapped = 0;
};

void build_bai(const std::vector<Rec>& recs, const std::vector<uint64_t>& vstart,
               const std::vector<uint64_t>& vend, int32_t n_ref, std::vector<uint8_t>& out) {
  std::vector<BinChunks> per(n_ref);
  uint64_t no_coor = 0;
  for (size_t i = 0; i < recs.size(); i++) {
    const Rec& r = recs[i];
    if (r.ref < 0) {
      no_coor++;
      continue;
    }
    BinChunks& b = per[r.ref];
    int beg = r.beg < 0 ? 0 : r.beg, end = r.end <= beg ? beg + 1 : r.end;
    uint32_t bin = (uint32_t)reg2bin(beg, end);
    auto& v = b.bins[bin];
    if (!v.empty() && v.back().second == vstart[i]) v.back().second = vend[i];
    else v.push_back({vstart[i], vend[i]});
    for (int w = beg >> 14; w <= (end - 1) >> 14; w++) {
      if ((int)b.linear.size() <= w) b.linear.resize(w + 1, 0);
      if (b.linear[w] == 0) b.linear[w] = vstart[i];
    }
    b.beg = std::min(b.beg, vstart[i]);
    b.end = std::max(b.end, vend[i]);
    if (r.mapped) b.n_mapped++;
    else b.n_unmapped++;
  }
  out.insert(out.end(), {'B', 'A', 'I', 1});
  put32(out, n_ref);
  auto put64 = [&](uint64_t v) {
    for (int i = 0; i < 8; i++) out.push_back((uint8_t)(v >> (8 * i)));
  };
  for (auto& b : per) {
    bool any = !b.bins.empty();
    put32(out, (int32_t)b.bins.size() + (any ? 1 : 0));
    for (auto& kv : b.bins) {
      put32(out, (int32_t)kv.first);
      put32(out, (int32_t)kv.second.size());
      for (auto& c : kv.second) {
        put64(c.first);
        put64(c.second);
      }
    }
    if (any) {  // pseudo-bin 37450: ref span and mapped/unmapped counts
      put32(out, 37450);
      put32(out, 2);
      put64(b.beg);
      put64(b.end);
      put64(b.n_mapped);
      put64(b.n_unmapped);
    }
    // fill linear-index gaps with the following entry (as htsjdk/samtools do)
    for (int w = (int)b.linear.size() - 2; w >= 0; w--)
      if (b.linear[w] == 0) b.linear[w] = b.linear[w + 1];
    put32(out, (int32_t)b.linear.size());
    for (uint64_t x : b.linear) put64(x);
  }
  put64(no_coor);
}

void build_sbi(const std::vector<uint64_t>& vstart, uint64_t final_ptr, int64_t file_len,
               int64_t gran, std::vector<uint8_t>& out) {
  auto put64 = [&](uint64_t v) {
    for (int i = 0; i < 8; i++) out.push_back((uint8_t)(v >> (8 * i)));
  };
  std::vector<uint64_t> offs;
  for (size_t i = 0; i < vstart.size(); i++)
    if ((int64_t)i % gran == 0) offs.push_back(vstart[i]);
  offs.push_back(final_ptr);
  out.insert(out.end(), {'S', 'B', 'I', 1});
  put64((uint64_t)file_len);
  out.insert(out.end(), 32, 0);  // md5 + uuid
  put64(vstart.size());
  put64((uint64_t)gran);
  put64(offs.size());
  for (uint64_t x : offs) put64(x);
}

uint8_t* dup(const std::vector<uint8_t>& v) {
  uint8_t* p = (uint8_t*)malloc(v.size() ? v.size() : 1);
  if (p && !v.empty()) memcpy(p, v.data(), v.size());
  return p;
}

}  // namespace

extern "C" {

int dq_synth_bam(const dq_synth_opts* opts, dq_synth_result* res) {
  if (!opts || !res) return -3;
  memset(res, 0, sizeof *res);
  Gen g;
  g.o = *opts;
  if (g.o.level < 0 || g.o.level > 9) g.o.level = 5;
  if (g.o.nthreads < 1) g.o.nthreads = 1;
  bool index = opts->write_bai || opts->sbi_granularity > 0;
  if (g.o.shape == DQ_SYNTH_ANYSAM) {
    g.dict = anysam_dict();
    int64_t pairs = opts->n_records;  // number of pairs, like writeAnySamFile(numPairs, ...)
    g.o.n_records = 2 * pairs;
    g.total_records = pairs > 0 ? 2 * pairs + 2 : 0;
    g.n_unplaced = pairs > 0 ? 2 : 0;
  } else {
    g.dict = grch38_dict();
    g.total_records = opts->n_records;
    g.n_unplaced = (int64_t)(opts->unplaced_fraction * (double)opts->n_records);
    int64_t usable = 0;
    for (auto& r : g.dict) usable += r.len - 200000;
    const int64_t mapped = std::max<int64_t>(1, g.total_records - g.n_unplaced);
    g.spacing = std::min(5.0, (double)usable / (double)mapped);
  }
  build_header(g);
  g.per_chunk = opts->records_per_chunk > 0 ? opts->records_per_chunk : 20000;
  if (g.o.shape == DQ_SYNTH_LONGREAD && opts->records_per_chunk <= 0) g.per_chunk = 2000;
  g.n_chunks = std::max<int64_t>(1, (g.total_records + g.per_chunk - 1) / g.per_chunk);
  res->n_chunks = g.n_chunks;
  int64_t klo = 0, khi = g.n_chunks;
  if (opts->chunk_hi > 0) {
    if (index || opts->chunk_lo < 0 || opts->chunk_lo >= opts->chunk_hi || opts->chunk_hi > g.n_chunks)
      return -3;
    klo = opts->chunk_lo;
    khi = opts->chunk_hi;
  }
  const bool with_eof = khi == g.n_chunks;
  std::vector<Chunk> chunks((size_t)(khi - klo));
  std::atomic<int64_t> next{0}, finished{0};
  const bool progress = getenv("DQ_SYNTH_PROGRESS") != nullptr;
  const int64_t step = std::max<int64_t>(1, g.n_chunks / 20);
  auto work = [&]() {
    for (;;) {
      int64_t k = next++;
      if (k >= khi - klo) break;
      make_chunk(g, klo + k, chunks[(size_t)k], index);
      int64_t f = ++finished;
      if (progress && f % step == 0) {
        fprintf(stderr, "[synth] %lld/%lld chunks\n", (long long)f, (long long)(khi - klo));
        fflush(stderr);
      }
    }
  };
  std::vector<std::thread> th;
  for (int t = 0; t < g.o.nthreads; t++) th.emplace_back(work);
  for (auto& t : th) t.join();
  // concatenate
  int64_t total = with_eof ? 28 : 0;
  for (auto& c : chunks) total += (int64_t)c.comp.size();
  uint8_t* bam = (uint8_t*)malloc((size_t)std::max<int64_t>(1, total));
  if (!bam) return -5;
  int64_t off = 0;
  std::vector<int64_t> chunk_addr;
  std::vector<std::vector<int64_t>> blk_addr(chunks.size());
  for (size_t k = 0; k < chunks.size(); k++) {
    chunk_addr.push_back(off);
    int64_t a = off;
    for (int32_t cs : chunks[k].blk_csize) {
      blk_addr[k].push_back(a);
      a += cs;
    }
    blk_addr[k].push_back(a);
    memcpy(bam + off, chunks[k].comp.data(), chunks[k].comp.size());
    off += (int64_t)chunks[k].comp.size();
    res->n_blocks += (int64_t)chunks[k].blk_csize.size();
    res->n_records += chunks[k].n_records;
    res->record_bytes += chunks[k].ubytes;
    std::vector<uint8_t>().swap(chunks[k].comp);
  }
  static const uint8_t eof[28] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 0x42, 0x43,
                                  2,    0,    0x1b, 0, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  if (with_eof) {
    memcpy(bam + off, eof, 28);
    res->n_blocks += 1;
  }
  res->bam = bam;
  res->bam_len = total;
  if (index) {
    std::vector<Rec> recs;
    std::vector<uint64_t> vs;
    for (size_t k = 0; k < chunks.size(); k++) {
      const Chunk& c = chunks[k];
      for (size_t i = 0; i < c.recs.size(); i++) {
        recs.push_back(c.recs[i]);
        uint32_t b = c.rec_blk[i];
        uint16_t o2 = c.rec_off[i];
        // a record starting exactly at a block boundary reads as (that block, 0)
        vs.push_back((uint64_t)blk_addr[k][b] << 16 | o2);
      }
    }
    std::vector<uint64_t> ve(vs.size());
    for (size_t i = 0; i + 1 < vs.size(); i++) ve[i] = vs[i + 1];
    uint64_t final_ptr = (uint64_t)off << 16;  // EOF block address (normalised end pointer)
    if (!vs.empty()) ve.back() = final_ptr;
    if (opts->write_bai) {
      std::vector<uint8_t> bai;
      build_bai(recs, vs, ve, (int32_t)g.dict.size(), bai);
      res->bai = dup(bai);
      res->bai_len = (int64_t)bai.size();
    }
    if (opts->sbi_granularity > 0) {
      std::vector<uint8_t> sbi;
      build_sbi(vs, final_ptr, total, opts->sbi_granularity, sbi);
      res->sbi = dup(sbi);
      res->sbi_len = (int64_t)sbi.size();
    }
  }
  return 0;
}

void dq_synth_free(dq_synth_result* res) {
  if (!res) return;
  free(res->bam);
  free(res->bai);
  free(res->sbi);
  memset(res, 0, sizeof *res);
}

}  // extern "C"
