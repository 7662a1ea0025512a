// jpeg_decode.hip — baseline JPEG decode on the GPU, fused with the Pillow-exact nearest resize
// into the HBM image arena (the store-image path of parallel/rank_backend.py; gfx950).
//
// Why: the store-image pass is bound by the first decode of each distinct image — ~1.1 ms of
// Pillow / libjpeg-turbo per 300x250 JPEG, ~6.7k images/s from 12 decode worker processes on a
// 16-CPU share (DESIGN §1 "Store images") against ~75k images/s of model throughput.
//
// What: the host parses the headers and un-stuffs each entropy-coded segment (C++ below,
// dml_jpeg_prepare) into one pinned buffer: per image a fixed-size descriptor (geometry,
// natural-order quantisation tables, Huffman lookup tables, the output slot's nearest-index
// tables) and its entropy bytes. On the device:
//   1. jpeg_huff_par_kernel (r6): a 64-lane wave per image decodes the entropy stream in 64 bit
//      segments at once, self-synchronising (see "parallel entropy decoding" below), into
//      int16 coefficient blocks; the r5 serial one-wave decode (jpeg_huff_kernel) stays as the
//      A/B reference (DML_JPEG_SERIAL=1) and as the code the CPU tests compare against.
//   2. jpeg_idct_kernel: one thread per 8x8 block — libjpeg's "islow" integer IDCT
//      (jidctint.c arithmetic: CONST_BITS 13, PASS1_BITS 2, 64-bit products, its post-IDCT
//      range-limit table) into per-component sample planes.
//   3. jpeg_rgb_resize_kernel: per output pixel of the model's size, the source pixel of
//      Pillow's NEAREST tables; its chroma by libjpeg's h2v2 "fancy" triangle upsampling
//      (jdsample.c, with its edge and context-row rules) and the jdcolor.c YCbCr->RGB tables
//      (16-bit fixed point) — written straight into the arena slot. No full-resolution RGB
//      image is ever materialised.
// The same __host__ __device__ code decodes on the CPU (dml_jpeg_decode_host), which the CPU
// tests compare byte for byte with Pillow's decode (tests/test_jpeg_gpu.py).
//
// Supported: baseline / extended-sequential Huffman (SOF0 / SOF1), 8-bit, one interleaved
// scan, grayscale or YCbCr 4:2:0 / 4:4:4, no restart markers. Anything else (progressive,
// 4:2:2, restart intervals, Adobe RGB / CMYK, arithmetic coding, > 60 KiB of entropy data) is
// reported unsupported and takes the CPU decode workers.
//
// Acknowledgement: byte-exactness with Pillow requires the arithmetic of the Independent JPEG
// Group's libjpeg, which Pillow links. The islow IDCT below (jidctint.c), the h2v2 "fancy"
// upsampling and its edge rules (jdsample.c) and the YCbCr->RGB fixed-point tables (jdcolor.c)
// re-implement that arithmetic. This software is based in part on the work of the Independent
// JPEG Group (libjpeg, Copyright (C) 1991-1998, Thomas G. Lane; IJG license). The Huffman
// decoder, the lookup tables, the descriptor layout and the kernels are this project's own.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "common.h"
#include "dml.h"

#define DMLJ_MAXOUT 320
#define DMLJ_MAXSTREAM (60 * 1024)

struct DmljHuff {
  uint32_t look[512];   // 9-bit lookahead: (len << 8) | symbol; 0 = a longer code (32-bit: scalar loads)
  uint32_t fast[512];   // AC only: code + extra bits within the 9-bit lookahead, decoded in one step:
                        // (coefficient << 16) | (run << 4) | total bits; 0 = the general path
  int32_t maxcode[18];  // largest code of each length (-1: none); [17] = sentinel
  int32_t valoff[18];   // val index of a code of length l = valoff[l] + code
  uint8_t val[256];
};

struct DmljImage {
  int32_t ok, w, h, ncomp;
  int32_t hmax, vmax, mcux, mcuy;
  int32_t hs[3], vs[3], tq[3], td[3], ta[3];
  int32_t bw[3], bh[3];         // blocks per row / column of the padded MCU grid
  int32_t dw[3], dh[3];         // libjpeg's downsampled_width / downsampled_height
  int32_t nblk, slot;           // blocks over all components; arena slot (set at launch)
  int64_t coef_off[3];          // int16 index of the component's first coefficient (work buffer)
  int64_t plane_off[3];         // byte offset of the component's sample plane (work buffer)
  int64_t stream_off;           // byte offset of the entropy bytes (this buffer)
  int32_t stream_len, outH, outW, pad;
  int16_t rowtab[DMLJ_MAXOUT], coltab[DMLJ_MAXOUT];
  uint16_t q[4][64];            // natural order
  uint8_t izz[64];              // natural -> zigzag index (the IDCT's gather of a zigzag block)
  uint8_t pad2[16];
  DmljHuff dc[4], ac[4];
};
static_assert(sizeof(DmljImage) % 16 == 0 && offsetof(DmljImage, dc) % 16 == 0 && sizeof(DmljHuff) % 16 == 0 &&
                  offsetof(DmljImage, izz) % 4 == 0 && offsetof(DmljHuff, val) % 4 == 0,
              "aligned descriptors; 32-bit reads of the byte tables");

namespace dml {
namespace jpg {

// zigzag index -> natural (row-major) index, + 16 entries of 63 (libjpeg's safety pad); the
// device reads the copy each descriptor carries
static const uint8_t kNatural[80] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13,
    6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31,
    39, 46, 53, 60, 61, 54, 47, 55, 62, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

// ------------------------------------------------------------------ entropy decoding --
struct Bits {
  const uint32_t* w;   // the entropy bytes as aligned 32-bit words, byte-swapped by the host (a
                       // little-endian read gives the stream's big-endian bits); >= 8 zero bytes
                       // past the end
  int nw, pos, nb;
  uint64_t buf;
  uint32_t nextw;      // the next refill's word, loaded one refill ahead (its latency hidden)
  __host__ __device__ Bits(const uint32_t* words, int nwords) : w(words), nw(nwords), pos(0), nb(0), buf(0) {
    nextw = w[0];
  }
  // >= 33 bits after a fill: enough for one Huffman code AND its extra bits (<= 16 + 11). In
  // the GPU kernel every lane runs the decode with the same (wave-uniform) operands, so these
  // reads and the table lookups are scalar loads and the bit arithmetic scalar instructions;
  // past the end the reader keeps returning zeros, as libjpeg
  __host__ __device__ void fill() {
    if (nb <= 32) {
      buf |= (uint64_t)nextw << (32 - nb);
      pos = pos + 1 < nw ? pos + 1 : nw;
      nextw = w[pos];
      nb += 32;
    }
  }
  __host__ __device__ uint32_t peek(int n) const { return (uint32_t)(buf >> (64 - n)); }
  __host__ __device__ void skip(int n) {
    buf <<= n;
    nb -= n;
  }
  __host__ __device__ int get(int n) {  // n <= 16, after fill()
    if (n == 0) return 0;
    const int v = (int)peek(n);
    skip(n);
    return v;
  }
};

// the host side of the word reads above: swap each 4-byte group of the (zero-padded) stream
static void swap_words(uint8_t* p, long len) {
  for (long i = 0; i + 4 <= len; i += 4) {
    uint32_t w;
    memcpy(&w, p + i, 4);
    w = __builtin_bswap32(w);
    memcpy(p + i, &w, 4);
  }
}

// byte i of a 4-byte-aligned array through a 32-bit read (a scalar load in the uniform kernel;
// gfx950 has no scalar byte load)
__host__ __device__ static inline int byte_at(const uint8_t* p, int i) {
  return (int)((((const uint32_t*)p)[i >> 2] >> ((i & 3) * 8)) & 255);
}

// `look`: the 9-bit lookahead table to use (the parallel kernel's LDS copy; the descriptor's own
// otherwise). Always a valid pointer: a select between an LDS and a global table made the
// per-symbol lookup a FLAT load (counted with the global loads, waited for with them)
template <class BR>
__host__ __device__ static inline int huff_decode_lk(BR& b, const DmljHuff& t, const uint32_t* look) {
  b.fill();
  const uint32_t e = look[b.peek(9)];
  if (e) {
    b.skip(e >> 8);
    return e & 255;
  }
  int l = 10;
  int code = (int)b.peek(l);
  while (l <= 16 && code > t.maxcode[l]) {
    ++l;
    code = (int)b.peek(l);
  }
  if (l > 16) {  // corrupt data: libjpeg warns and returns 0
    b.skip(16);
    return 0;
  }
  b.skip(l);
  return byte_at(t.val, (t.valoff[l] + code) & 255);
}

template <class BR>
__host__ __device__ static inline int huff_decode(BR& b, const DmljHuff& t) {
  return huff_decode_lk(b, t, t.look);
}

__host__ __device__ static inline int extend(int v, int s) { return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v; }

// all MCUs of one image -> int16 coefficient blocks in ZIGZAG order (zero-filled by the caller;
// the IDCT reads them through the inverse table: no dependent table load per coefficient
// here). In the GPU kernel every lane runs this and stores the same value to the same address
// (no divergent branch around the stores)
__host__ __device__ static void decode_entropy(const DmljImage& d, const uint32_t* stream, int16_t* coef,
                                               bool writer) {
  const DmljHuff* dcs = d.dc;
  const DmljHuff* acs = d.ac;
  Bits b(stream, (d.stream_len + 3) / 4);
  int pred[3] = {0, 0, 0};
  const int nc = d.ncomp;
  for (int my = 0; my < d.mcuy; ++my)
    for (int mx = 0; mx < d.mcux; ++mx)
      for (int c = 0; c < nc; ++c) {
        const int hs = nc == 1 ? 1 : d.hs[c], vs = nc == 1 ? 1 : d.vs[c];
        const DmljHuff& dct = dcs[d.td[c]];
        const DmljHuff& act = acs[d.ta[c]];
        for (int v = 0; v < vs; ++v)
          for (int h = 0; h < hs; ++h) {
            const int bx = mx * hs + h, by = my * vs + v;
            int16_t* blk = coef + d.coef_off[c] + ((int64_t)by * d.bw[c] + bx) * 64;
            const int s = huff_decode(b, dct);
            const int diff = s ? extend(b.get(s), s) : 0;
            pred[c] += diff;
            if (writer) blk[0] = (int16_t)pred[c];
            for (int k = 1; k < 64; ++k) {
              b.fill();
              const uint32_t f = act.fast[b.peek(9)];
              if (f) {   // the common short code with a small coefficient: one lookup, one skip
                b.skip(f & 15);
                k += (f >> 4) & 15;
                if (writer) blk[k < 64 ? k : 63] = (int16_t)((int32_t)f >> 16);
                continue;
              }
              const int rs = huff_decode(b, act);
              const int r = rs >> 4, sz = rs & 15;
              if (sz) {
                k += r;
                const int v2 = extend(b.get(sz), sz);
                if (writer) blk[k < 64 ? k : 63] = (int16_t)v2;   // corrupt runs: libjpeg's pad maps to 63
              } else {
                if (r != 15) break;
                k += 15;
              }
            }
          }
      }
}

// --------------------------------------------------------- parallel entropy decoding --
// one wave decoding each image serially put ~one wave per CU to work for ~7 ms per
// 256-image window. Here a workgroup of PT threads decodes one image: thread t owns the
// symbols that START in bit segment t of the entropy stream. Huffman codes self-synchronise, so
//   1. every thread decodes its segment from a guessed state (MCU slot 0, coefficient 0) and
//      records its EXIT: the first symbol boundary at or past the segment end, with the decoder
//      state (MCU block slot u, next coefficient k) there, and the blocks it completed;
//   2. thread t re-decodes from thread t-1's exit until no exit changes (Jacobi rounds; the
//      chain from the exact thread 0 converges in a few rounds: a wrong start re-joins the true
//      symbol sequence within a few symbols, and from there its exit equals the true one);
//   3. a prefix sum over the block counts gives each thread the decode-order index of its first
//      block; every thread decodes its segment once more, now writing coefficients and DC
//      DIFFERENCES, and stops at the image's last block;
//   4. the DC predictions are rebuilt per component by a block-wide prefix sum in decode order.
// Per symbol: one 11-bit lookahead (code length + symbol) and the same run / size / extra-bits
// arithmetic for DC and AC; codes longer than 11 bits and corrupt codes take the serial
// decoder's general path, so the coefficients are identical to it (tests/test_jpeg_decode.py
// compares every block).
// Segments per image: a decoder started in the wrong state re-joins the true symbol AND
// block-slot sequence after ~5,000 bits (CPU replay, 40 bench images: 64 / 128 / 256 segments
// take 2.5 / 4.7 / 9.5 rounds), so a lane's bits (2 + rounds) x segment fall only 10.6k -> 7.0k
// from 64 to 256 segments. But the kernel is latency-bound with one image per workgroup and only
// 256 images a window: 64 threads leave three of a CU's four SIMDs idle. 256 threads (4 waves)
// won on the box (r6, profiles/r6_pt): window 2.96-3.00 -> 2.08-2.11 ms, 4 windows in flight
// 4.02-4.11 -> 2.97-2.99 ms, the 51,200-distinct pass 48.3k -> 52.5k images/s.
// 512 threads (replay: 18.7 rounds, 6.5k bits a lane) measured the same as 256 on the box
// (window 2.10-2.17 vs 2.14-2.45 ms, profiles/r6_p): 256 stays.
// DMLJ_PT stays the CPU replay's default; the GPU launch takes DMLJ_PT_GPU (DML_JPEG_PT: A/B)
#define DMLJ_PT 64
#define DMLJ_PT_GPU 256

struct PState {
  int pos, u, k;   // bit position of the next symbol; MCU block slot; next coefficient (0 = DC)
};

struct McuMap {
  int U, total;                  // block slots per MCU; blocks in the image
  // slot u -> component (2 bits at 2u) and its block offset inside the MCU (bit u): packed, so
  // the per-symbol lookups are shifts, not a runtime-indexed array (which goes to scratch)
  int comp, dv, dh;
  __host__ __device__ int comp_of(int u) const { return (comp >> (2 * u)) & 3; }
};

__host__ __device__ static inline McuMap mcu_map(const DmljImage& d) {
  McuMap m;
  m.U = m.comp = m.dv = m.dh = 0;
  const int nc = d.ncomp;
  for (int c = 0; c < nc; ++c) {
    const int hs = nc == 1 ? 1 : d.hs[c], vs = nc == 1 ? 1 : d.vs[c];
    for (int v = 0; v < vs; ++v)
      for (int h = 0; h < hs; ++h) {
        m.comp |= c << (2 * m.U);
        m.dv |= v << m.U;
        m.dh |= h << m.U;
        ++m.U;
      }
  }
  m.total = d.mcux * d.mcuy * m.U;
  return m;
}

// coefficient block of decode-order block gb
__host__ __device__ static inline int16_t* block_at(const DmljImage& d, const McuMap& m, int16_t* coef, int gb) {
  const int mcu = gb / m.U, u = gb - mcu * m.U;
  const int my = mcu / d.mcux, mx = mcu - my * d.mcux;
  const int c = m.comp_of(u);
  const int hs = d.ncomp == 1 ? 1 : d.hs[c], vs = d.ncomp == 1 ? 1 : d.vs[c];
  const int by = my * vs + ((m.dv >> u) & 1), bx = mx * hs + ((m.dh >> u) & 1);
  return coef + d.coef_off[c] + ((int64_t)by * d.bw[c] + bx) * 64;
}

// a bit reader that starts at any bit (the serial Bits starts at 0); same word layout. The next
// refill's word is loaded one refill ahead (`nextw`), so its global-memory latency is off the
// per-symbol dependency chain
struct BitsAt {
  const uint32_t* w;
  int nw, wpos, nb;
  uint64_t buf;
  uint32_t nextw;
  __host__ __device__ BitsAt(const uint32_t* words, int nwords, int bit) : w(words), nw(nwords) {
    wpos = bit >> 5;
    const uint32_t cur = wpos < nw ? w[wpos] : 0u;
    buf = ((uint64_t)cur << 32) << (bit & 31);
    nb = 32 - (bit & 31);
    ++wpos;
    nextw = wpos < nw ? w[wpos] : 0u;
  }
  __host__ __device__ int pos() const { return wpos * 32 - nb; }
  __host__ __device__ void fill() {
    if (nb <= 32) {
      buf |= (uint64_t)nextw << (32 - nb);
      ++wpos;
      nb += 32;
      nextw = wpos < nw ? w[wpos] : 0u;
    }
  }
  __host__ __device__ uint32_t peek(int n) const { return (uint32_t)(buf >> (64 - n)); }
  __host__ __device__ void skip(int n) {
    buf <<= n;
    nb -= n;
  }
  __host__ __device__ int get(int n) {
    if (n == 0) return 0;
    const int v = (int)peek(n);
    skip(n);
    return v;
  }
};

// the lookup tables one thread decodes with: an 11-bit lookahead per component and class,
// (code length << 8) | symbol, 0 = a longer code (LDS on the GPU; built per image by the kernel).
// Slot c: component c's DC table, slot 3 + c: its AC table.
#define DMLJ_LA 11
struct SegTabs {
  const uint16_t* t11;
};

// entry i of the 11-bit lookahead of table t (the 9-bit one extended by the canonical
// length-10 / 11 codes; huff_decode's search order)
__host__ __device__ static inline uint16_t t11_entry(const DmljHuff& t, int i) {
  const uint32_t e9 = t.look[i >> (DMLJ_LA - 9)];
  if (e9) return (uint16_t)e9;
  for (int l = 10; l <= DMLJ_LA; ++l) {
    const int code = i >> (DMLJ_LA - l);
    if (code <= t.maxcode[l]) return (uint16_t)((l << 8) | byte_at(t.val, (t.valoff[l] + code) & 255));
  }
  return 0;
}

// decode the symbols starting in [st.pos, end) from state st; returns the exit state and the
// blocks completed. WRITE: block gb onwards gets its AC coefficients and its DC DIFFERENCE, and
// decoding stops at the image's last block.
template <bool WRITE>
__host__ __device__ static PState seg_decode(const DmljImage& d, const McuMap& m, const SegTabs& tb,
                                             const uint32_t* stream, int nw, PState st, int end, int* nblocks,
                                             int gb, int16_t* coef) {
  BitsAt b(stream, nw, st.pos);
  int u = st.u, k = st.k, cnt = 0;
  // component -> Huffman table ids, packed once (2 bits each): `d.td[c]` with a per-lane c was a
  // vector load from the descriptor on every symbol (rocprofv3: ~4 VMEM per symbol, 5x the LDS
  // lookups; profiles/r6_pmc)
  const int tdp = d.td[0] | (d.ncomp > 1 ? (d.td[1] << 2) | (d.td[2] << 4) : 0);
  const int tap = d.ta[0] | (d.ncomp > 1 ? (d.ta[1] << 2) | (d.ta[2] << 4) : 0);
  int16_t* blk = WRITE && gb < m.total ? block_at(d, m, coef, gb) : nullptr;
  while (b.pos() < end) {
    if (WRITE && gb >= m.total) break;
    const int c = m.comp_of(u);
    // one path for every symbol (r6: with 64 lanes at different block positions the wave ran
    // the DC, the fast-AC and the general-AC branch on nearly every symbol; PMC profiles/r6_pmc):
    // an 11-bit lookahead gives code length + symbol for all but the rare longer codes, the
    // symbol's run / size / extra bits are then decoded the same way for DC and AC
    const bool dcs = k == 0;
    b.fill();
    const uint32_t e = tb.t11[(dcs ? c : 3 + c) * (1 << DMLJ_LA) + b.peek(DMLJ_LA)];
    int sym, len;
    if (e) {
      len = e >> 8;   // skipped together with the extra bits below (one shift of the buffer)
      sym = e & 255;
    } else {
      sym = dcs ? huff_decode(b, d.dc[(tdp >> (2 * c)) & 3]) : huff_decode(b, d.ac[(tap >> (2 * c)) & 3]);
      len = 0;        // the general path consumed the code
    }
    const int run = dcs ? 0 : sym >> 4, size = dcs ? sym : sym & 15;
    const int tot = len + size;   // <= 11 + 15 bits: the fill left >= 33
    const uint32_t bits = tot ? b.peek(tot) : 0u;
    b.skip(tot);
    const int v = size ? extend((int)(bits & ((1u << size) - 1u)), size) : 0;
    const int kk = dcs ? 0 : k + run;
    if (WRITE && (dcs || size)) blk[kk < 64 ? kk : 63] = (int16_t)v;   // corrupt runs: libjpeg's pad -> 63
    bool done;
    if (dcs) {
      k = 1;
      done = false;
    } else if (size) {
      k = kk + 1;
      done = k >= 64;
    } else if (run != 15) {
      done = true;   // EOB
    } else {
      k += 16;
      done = k >= 64;
    }
    if (done) {
      k = 0;
      u = u + 1 == m.U ? 0 : u + 1;
      ++cnt;
      if (WRITE) {
        ++gb;
        blk = gb < m.total ? block_at(d, m, coef, gb) : nullptr;
      }
    }
  }
  *nblocks = cnt;
  return PState{b.pos(), u, k};
}

__host__ __device__ static inline int seg_bits(const DmljImage& d, int nseg_max = DMLJ_PT) {
  const int nbits = d.stream_len * 8;
  int seg = (nbits + nseg_max - 1) / nseg_max;
  seg = (seg + 31) / 32 * 32;
  return seg < 64 ? 64 : seg;
}

// ----------------------------------------------------------------------------- IDCT --
// libjpeg jidctint.c (jpeg_idct_islow), 64-bit products as its JLONG
#define DJ_CONST_BITS 13
#define DJ_PASS1_BITS 2
#define DJ_DESCALE(x, n) (((x) + ((int64_t)1 << ((n)-1))) >> (n))

__host__ __device__ static inline uint8_t idct_range(int64_t x) {
  // the post-IDCT range_limit table, indexed by x & RANGE_MASK (1023)
  const int i = (int)(x & 1023);
  return (uint8_t)(i < 128 ? 128 + i : (i < 512 ? 255 : (i < 896 ? 0 : i - 896)));
}

__host__ __device__ static void idct_islow(const int16_t* in, const uint16_t* q, uint8_t* out, int stride) {
  int ws[64];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int16_t* ip = in + c;
    const uint16_t* qp = q + c;
    int* wp = ws + c;
    if (ip[8] == 0 && ip[16] == 0 && ip[24] == 0 && ip[32] == 0 && ip[40] == 0 && ip[48] == 0 && ip[56] == 0) {
      const int dc = (int)((int64_t)ip[0] * qp[0]) << DJ_PASS1_BITS;
#pragma unroll
      for (int r = 0; r < 8; ++r) wp[r * 8] = dc;
      continue;
    }
    int64_t z2 = (int64_t)ip[16] * qp[16], z3 = (int64_t)ip[48] * qp[48];
    int64_t z1 = (z2 + z3) * 4433;
    int64_t tmp2 = z1 + z3 * (-15137);
    int64_t tmp3 = z1 + z2 * 6270;
    z2 = (int64_t)ip[0] * qp[0];
    z3 = (int64_t)ip[32] * qp[32];
    int64_t tmp0 = (z2 + z3) << DJ_CONST_BITS;
    int64_t tmp1 = (z2 - z3) << DJ_CONST_BITS;
    const int64_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
    tmp0 = (int64_t)ip[56] * qp[56];
    tmp1 = (int64_t)ip[40] * qp[40];
    tmp2 = (int64_t)ip[24] * qp[24];
    tmp3 = (int64_t)ip[8] * qp[8];
    z1 = tmp0 + tmp3;
    z2 = tmp1 + tmp2;
    z3 = tmp0 + tmp2;
    int64_t z4 = tmp1 + tmp3;
    const int64_t z5 = (z3 + z4) * 9633;
    tmp0 *= 2446;
    tmp1 *= 16819;
    tmp2 *= 25172;
    tmp3 *= 12299;
    z1 *= -7373;
    z2 *= -20995;
    z3 *= -16069;
    z4 *= -3196;
    z3 += z5;
    z4 += z5;
    tmp0 += z1 + z3;
    tmp1 += z2 + z4;
    tmp2 += z2 + z3;
    tmp3 += z1 + z4;
    const int sh = DJ_CONST_BITS - DJ_PASS1_BITS;
    wp[0] = (int)DJ_DESCALE(tmp10 + tmp3, sh);
    wp[56] = (int)DJ_DESCALE(tmp10 - tmp3, sh);
    wp[8] = (int)DJ_DESCALE(tmp11 + tmp2, sh);
    wp[48] = (int)DJ_DESCALE(tmp11 - tmp2, sh);
    wp[16] = (int)DJ_DESCALE(tmp12 + tmp1, sh);
    wp[40] = (int)DJ_DESCALE(tmp12 - tmp1, sh);
    wp[24] = (int)DJ_DESCALE(tmp13 + tmp0, sh);
    wp[32] = (int)DJ_DESCALE(tmp13 - tmp0, sh);
  }
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const int* wp = ws + r * 8;
    uint8_t* op = out + r * stride;
    int64_t z2 = wp[2], z3 = wp[6];
    int64_t z1 = (z2 + z3) * 4433;
    int64_t tmp2 = z1 + z3 * (-15137);
    int64_t tmp3 = z1 + z2 * 6270;
    int64_t tmp0 = ((int64_t)wp[0] + wp[4]) << DJ_CONST_BITS;
    int64_t tmp1 = ((int64_t)wp[0] - wp[4]) << DJ_CONST_BITS;
    const int64_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
    tmp0 = wp[7];
    tmp1 = wp[5];
    tmp2 = wp[3];
    tmp3 = wp[1];
    z1 = tmp0 + tmp3;
    z2 = tmp1 + tmp2;
    z3 = tmp0 + tmp2;
    int64_t z4 = tmp1 + tmp3;
    const int64_t z5 = (z3 + z4) * 9633;
    tmp0 *= 2446;
    tmp1 *= 16819;
    tmp2 *= 25172;
    tmp3 *= 12299;
    z1 *= -7373;
    z2 *= -20995;
    z3 *= -16069;
    z4 *= -3196;
    z3 += z5;
    z4 += z5;
    tmp0 += z1 + z3;
    tmp1 += z2 + z4;
    tmp2 += z2 + z3;
    tmp3 += z1 + z4;
    const int sh = DJ_CONST_BITS + DJ_PASS1_BITS + 3;
    op[0] = idct_range(DJ_DESCALE(tmp10 + tmp3, sh));
    op[7] = idct_range(DJ_DESCALE(tmp10 - tmp3, sh));
    op[1] = idct_range(DJ_DESCALE(tmp11 + tmp2, sh));
    op[6] = idct_range(DJ_DESCALE(tmp11 - tmp2, sh));
    op[2] = idct_range(DJ_DESCALE(tmp12 + tmp1, sh));
    op[5] = idct_range(DJ_DESCALE(tmp12 - tmp1, sh));
    op[3] = idct_range(DJ_DESCALE(tmp13 + tmp0, sh));
    op[4] = idct_range(DJ_DESCALE(tmp13 - tmp0, sh));
  }
}

// ------------------------------------------------------- upsampling + colour conversion --
__host__ __device__ static inline uint8_t clamp255(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

// chroma sample c at full-resolution (sy, sx): libjpeg h2v2_fancy_upsample (4:2:0) or the
// sample itself (4:4:4)
__host__ __device__ static inline int chroma_at(const DmljImage& d, const uint8_t* work, int c, int sy, int sx) {
  const uint8_t* pl = work + d.plane_off[c];
  const int pw = d.bw[c] * 8;
  if (d.hs[c] == d.hmax) return pl[(int64_t)sy * pw + sx];
  const int r = sy >> 1, k = sx >> 1, dh = d.dh[c], dw = d.dw[c];
  // libjpeg-turbo (jdsample.c jinit_upsampler) uses the fancy filter only when the downsampled
  // width exceeds 2; narrower components are box-replicated
  if (dw <= 2) return pl[(int64_t)r * pw + k];
  // nearest row r; next nearest: above for the upper output row, below for the lower; the
  // row above the first and below the last real row are those rows themselves
  const int r1 = (sy & 1) ? (r + 1 < dh ? r + 1 : dh - 1) : (r > 0 ? r - 1 : 0);
  const uint8_t* in0 = pl + (int64_t)r * pw;
  const uint8_t* in1 = pl + (int64_t)r1 * pw;
  const int s = in0[k] * 3 + in1[k];
  if (!(sx & 1)) {
    if (k == 0) return (s * 4 + 8) >> 4;
    const int sl = in0[k - 1] * 3 + in1[k - 1];
    return (s * 3 + sl + 8) >> 4;
  }
  if (k == dw - 1) return (s * 4 + 7) >> 4;
  const int sr = in0[k + 1] * 3 + in1[k + 1];
  return (s * 3 + sr + 7) >> 4;
}

__host__ __device__ static inline void rgb_at(const DmljImage& d, const uint8_t* work, int sy, int sx, uint8_t* o) {
  const int y = work[d.plane_off[0] + (int64_t)sy * d.bw[0] * 8 + sx];
  if (d.ncomp == 1) {
    o[0] = o[1] = o[2] = (uint8_t)y;
    return;
  }
  const int x1 = chroma_at(d, work, 1, sy, sx) - 128, x2 = chroma_at(d, work, 2, sy, sx) - 128;
  // jdcolor.c build_ycc_rgb_table, SCALEBITS 16: FIX(1.40200) 91881, FIX(1.77200) 116130,
  // FIX(0.71414) 46802, FIX(0.34414) 22554, ONE_HALF 32768
  const int64_t crr = (91881 * (int64_t)x2 + 32768) >> 16;
  const int64_t cbb = (116130 * (int64_t)x1 + 32768) >> 16;
  const int64_t g = (-22554 * (int64_t)x1 + 32768 + (-46802) * (int64_t)x2) >> 16;
  o[0] = clamp255(y + (int)crr);
  o[1] = clamp255(y + (int)g);
  o[2] = clamp255(y + (int)cbb);
}

// ----------------------------------------------------------------------------- kernels --
// one wave per image; every lane runs the same decode (wave-uniform: scalar loads of the
// entropy words and the Huffman tables from the descriptor, scalar bit arithmetic)
__global__ __launch_bounds__(64) void jpeg_huff_kernel(const unsigned char* __restrict__ buf, int n,
                                                       int16_t* __restrict__ coef) {
  const int i = blockIdx.x;
  const DmljImage* ds = (const DmljImage*)(buf + 16);
  if (i >= n || !ds[i].ok) return;
  decode_entropy(ds[i], (const uint32_t*)(buf + ds[i].stream_off), coef, true);
}

// the parallel decode of one image per workgroup of PT threads = PT segments (see "parallel
// entropy decoding" above). r6 A/B: staging the image's entropy words in LDS first changed
// nothing (window 3.13-3.22 vs 3.21-3.28 ms, profiles/r6_lds): the per-symbol chain is not
// waiting on the stream reads
template <int PT>
struct ParLds {
  uint16_t t11[6][1 << DMLJ_LA];
  int ex_pos[2][PT], ex_u[2][PT], ex_k[2][PT], scan[2][PT];
  int chg[3];
};

template <int PT>
__global__ __launch_bounds__(PT) void jpeg_huff_par_kernel(const unsigned char* __restrict__ buf, int n,
                                                           int16_t* __restrict__ coef) {
  const int i = blockIdx.x;
  if (i >= n) return;
  const DmljImage& d = ((const DmljImage*)(buf + 16))[i];
  if (!d.ok) return;   // uniform over the workgroup
  __shared__ ParLds<PT> L;
  auto& ex_pos = L.ex_pos;
  auto& ex_u = L.ex_u;
  auto& ex_k = L.ex_k;
  auto& scan = L.scan;
  auto& chg = L.chg;
  const int t = threadIdx.x;
  const int nc = d.ncomp;
  for (int c = 0; c < nc; ++c) {
    const DmljHuff& hd = d.dc[d.td[c]];
    const DmljHuff& ha = d.ac[d.ta[c]];
#pragma unroll 4
    for (int j = t; j < (1 << DMLJ_LA); j += PT) {
      L.t11[c][j] = t11_entry(hd, j);
      L.t11[3 + c][j] = t11_entry(ha, j);
    }
  }
  if (t < 3) chg[t] = 0;
  const SegTabs tb = {&L.t11[0][0]};
  const McuMap m = mcu_map(d);
  const uint32_t* stream = (const uint32_t*)(buf + d.stream_off);
  const int nw = (d.stream_len + 3) / 4;
  const int SEG = seg_bits(d, PT), nbits = d.stream_len * 8;
  const int nseg = (nbits + SEG - 1) / SEG;
  const bool live = t < nseg;
  const int end = live ? min((t + 1) * SEG, nbits) : 0;
  __syncthreads();
  // 1. every segment from a guessed state
  PState start = {t * SEG, 0, 0}, ex = {0, 0, 0};
  int nb = 0;
  if (live) ex = seg_decode<false>(d, m, tb, stream, nw, start, end, &nb, 0, nullptr);
  ex_pos[0][t] = ex.pos;
  ex_u[0][t] = ex.u;
  ex_k[0][t] = ex.k;
  __syncthreads();
  // 2. Jacobi rounds: re-decode from the predecessor's exit until no exit changes. Flags rotate
  // over three slots: round r sets chg[r % 3]; thread 0 clears round r+1's slot before round r's
  // barrier, when every thread has read it for the last time (round r-2)
  int cur = 0;
  for (int r = 0; r < nseg; ++r) {
    if (t == 0) chg[(r + 1) % 3] = 0;
    if (live && t > 0) {
      const PState st = {ex_pos[cur][t - 1], ex_u[cur][t - 1], ex_k[cur][t - 1]};
      if (st.pos != start.pos || st.u != start.u || st.k != start.k) {
        start = st;
        const PState e2 = seg_decode<false>(d, m, tb, stream, nw, start, end, &nb, 0, nullptr);
        if (e2.pos != ex.pos || e2.u != ex.u || e2.k != ex.k) chg[r % 3] = 1;
        ex = e2;
      }
    }
    ex_pos[cur ^ 1][t] = ex.pos;
    ex_u[cur ^ 1][t] = ex.u;
    ex_k[cur ^ 1][t] = ex.k;
    __syncthreads();
    cur ^= 1;
    if (!chg[r % 3]) break;   // uniform: every thread reads the slot after the same barrier
  }
  // 3. exclusive prefix of the block counts -> each thread's first block; decode and write
  int sc = 0;
  scan[0][t] = live ? nb : 0;
  __syncthreads();
  for (int off = 1; off < PT; off <<= 1) {
    const int v = scan[sc][t] + (t >= off ? scan[sc][t - off] : 0);
    scan[sc ^ 1][t] = v;
    __syncthreads();
    sc ^= 1;
  }
  const int gb0 = t > 0 ? scan[sc][t - 1] : 0;
  if (live) seg_decode<true>(d, m, tb, stream, nw, start, end, &nb, gb0, coef);
  __syncthreads();
  // 4. DC predictions per component: block-wide prefix over the differences in decode order
  for (int c = 0; c < nc; ++c) {
    const int hs = nc == 1 ? 1 : d.hs[c], vs = nc == 1 ? 1 : d.vs[c];
    const int nbc = d.bw[c] * d.bh[c], per = (nbc + PT - 1) / PT;
    const int j0 = min(t * per, nbc), j1 = min(j0 + per, nbc);
    auto dcp = [&](int j) -> int16_t* {
      const int mcu = j / (hs * vs), w = j - mcu * (hs * vs);
      const int v = w / hs, h = w - v * hs;
      const int my = mcu / d.mcux, mx = mcu - my * d.mcux;
      return coef + d.coef_off[c] + ((int64_t)(my * vs + v) * d.bw[c] + (mx * hs + h)) * 64;
    };
    int sum = 0;
    for (int j = j0; j < j1; ++j) sum += *dcp(j);
    scan[0][t] = sum;
    __syncthreads();
    sc = 0;
    for (int off = 1; off < PT; off <<= 1) {
      const int v = scan[sc][t] + (t >= off ? scan[sc][t - off] : 0);
      scan[sc ^ 1][t] = v;
      __syncthreads();
      sc ^= 1;
    }
    int pred = t > 0 ? scan[sc][t - 1] : 0;
    for (int j = j0; j < j1; ++j) {
      int16_t* p = dcp(j);
      pred += *p;
      *p = (int16_t)pred;
    }
    __syncthreads();
  }
}


__global__ __launch_bounds__(256) void jpeg_idct_kernel(const unsigned char* __restrict__ buf, int n,
                                                        const int16_t* __restrict__ coef, uint8_t* __restrict__ work) {
  const int i = blockIdx.y;
  const DmljImage& d = ((const DmljImage*)(buf + 16))[i];
  int blk = blockIdx.x * 256 + threadIdx.x;
  if (!d.ok || blk >= d.nblk) return;
  int c = 0;
  while (c + 1 < d.ncomp && blk >= d.bw[c] * d.bh[c]) {
    blk -= d.bw[c] * d.bh[c];
    ++c;
  }
  const int by = blk / d.bw[c], bx = blk - by * d.bw[c];
  const int pw = d.bw[c] * 8;
  const int16_t* zz = coef + d.coef_off[c] + (int64_t)blk * 64;
  int16_t in[64];
#pragma unroll
  for (int j = 0; j < 64; ++j) in[j] = zz[d.izz[j]];   // zigzag -> natural
  idct_islow(in, d.q[d.tq[c]], work + d.plane_off[c] + (int64_t)by * 8 * pw + bx * 8, pw);
}

__global__ __launch_bounds__(256) void jpeg_rgb_resize_kernel(const unsigned char* __restrict__ buf, int n,
                                                              const uint8_t* __restrict__ work, int H, int W,
                                                              uint8_t* __restrict__ arena) {
  const int y = blockIdx.x, i = blockIdx.y;
  const DmljImage& d = ((const DmljImage*)(buf + 16))[i];
  if (!d.ok || y >= H) return;
  const int sy = d.rowtab[y];
  uint8_t* row = arena + ((int64_t)d.slot * H + y) * W * 3;
  for (int x = threadIdx.x; x < W; x += 256) {
    uint8_t o[3];
    rgb_at(d, work, sy, d.coltab[x], o);
    row[x * 3] = o[0];
    row[x * 3 + 1] = o[1];
    row[x * 3 + 2] = o[2];
  }
}

// ------------------------------------------------------------------------ host parser --
static int build_huff(const uint8_t* counts, const uint8_t* vals, int nvals, DmljHuff& t) {
  memset(&t, 0, sizeof t);
  int k = 0, code = 0;
  for (int l = 1; l <= 16; ++l) {
    const int cnt = counts[l - 1];
    if (cnt) {
      t.valoff[l] = k - code;
      for (int j = 0; j < cnt; ++j, ++k, ++code) {
        if (k >= nvals || k >= 256) return -1;
        if (l <= 9) {
          const int base = code << (9 - l);
          for (int e = 0; e < (1 << (9 - l)); ++e) t.look[base + e] = (uint32_t)((l << 8) | vals[k]);
        }
      }
      t.maxcode[l] = code - 1;
    } else {
      t.maxcode[l] = -1;
    }
    code <<= 1;
  }
  t.maxcode[17] = 0x7fffffff;
  memcpy(t.val, vals, nvals < 256 ? nvals : 256);
  for (int i = 0; i < 512; ++i) {   // fast AC entries (harmless, unused, for DC tables)
    const uint32_t e = t.look[i];
    const int len = (int)(e >> 8), sym = (int)(e & 255), run = sym >> 4, size = sym & 15;
    if (!e || size == 0 || len + size > 9) continue;
    const int extra = (i >> (9 - len - size)) & ((1 << size) - 1);
    const int v = extend(extra, size);
    t.fast[i] = (uint32_t)((int32_t)v * 65536) | (uint32_t)(run << 4) | (uint32_t)(len + size);
  }
  return 0;
}

// the same tables recur across a window (encoders write their standard or per-quality tables):
// a small per-thread cache keyed by the DHT bytes (counts + values) copies a built table instead
// of rebuilding its 512-entry lookups
static int build_huff_cached(const uint8_t* counts, const uint8_t* vals, int nvals, DmljHuff& t) {
  struct Ent {
    int n = -1;
    uint8_t key[16 + 256];
    DmljHuff tab;
  };
  static thread_local Ent cache[8];
  static thread_local int next = 0;
  for (Ent& e : cache)
    if (e.n == nvals && !memcmp(e.key, counts, 16) && !memcmp(e.key + 16, vals, nvals)) {
      memcpy(&t, &e.tab, sizeof t);
      return 0;
    }
  if (build_huff(counts, vals, nvals, t) != 0) return -1;
  Ent& e = cache[next];
  next = (next + 1) & 7;
  e.n = nvals;
  memcpy(e.key, counts, 16);
  memcpy(e.key + 16, vals, nvals);
  memcpy(&e.tab, &t, sizeof t);
  return 0;
}

static void nearest_tab(int n_in, int n_out, int16_t* tab) {
  // Pillow NEAREST: a float64 accumulator started at half a step, sequential adds, truncation
  // (rank_backend.nearest_index)
  const double a = (double)n_in / (double)n_out;
  volatile double acc = a * 0.5;
  for (int i = 0; i < n_out; ++i) {
    if (i) acc = acc + a;
    tab[i] = (int16_t)(int)acc;
  }
}

// parse one JPEG into d (+ un-stuffed entropy bytes at out); 0 = supported
static int parse_one(const uint8_t* p, int64_t len, DmljImage& d, uint8_t* out, int64_t cap, int outH, int outW) {
  memset(&d, 0, sizeof d);
  if (len < 4 || p[0] != 0xFF || p[1] != 0xD8) return -1;
  int64_t i = 2;
  bool have_sof = false, jfif = false, adobe = false;
  int adobe_transform = -1;
  int cid[3] = {0, 0, 0};
  bool qdef[4] = {false, false, false, false};
  while (i < len) {
    if (p[i] != 0xFF) return -1;
    while (i < len && p[i] == 0xFF) ++i;
    if (i >= len) return -1;
    const int m = p[i++];
    if (m == 0xD9) return -1;                    // EOI before the scan
    if (m >= 0xD0 && m <= 0xD7) continue;        // stray RST
    if (i + 2 > len) return -1;
    const int seglen = (p[i] << 8) | p[i + 1];
    if (seglen < 2 || i + seglen > len) return -1;
    const uint8_t* s = p + i + 2;
    const int sl = seglen - 2;
    if (m == 0xE0 && sl >= 5 && !memcmp(s, "JFIF", 5)) jfif = true;
    if (m == 0xEE && sl >= 12 && !memcmp(s, "Adobe", 5)) {
      adobe = true;
      adobe_transform = s[11];
    }
    if (m == 0xDB) {                             // DQT
      int o = 0;
      while (o < sl) {
        const int pq = s[o] >> 4, tqi = s[o] & 15;
        if (pq != 0 || tqi > 3 || o + 65 > sl) return -1;  // 16-bit tables: CPU path
        for (int k = 0; k < 64; ++k) d.q[tqi][kNatural[k]] = s[o + 1 + k];
        qdef[tqi] = true;
        o += 65;
      }
    } else if (m == 0xC4) {                      // DHT
      int o = 0;
      while (o < sl) {
        if (o + 17 > sl) return -1;
        const int tc = s[o] >> 4, th = s[o] & 15;
        if (tc > 1 || th > 3) return -1;
        int nv = 0;
        for (int k = 0; k < 16; ++k) nv += s[o + 1 + k];
        if (o + 17 + nv > sl || nv > 256) return -1;
        if (build_huff_cached(s + o + 1, s + o + 17, nv, tc ? d.ac[th] : d.dc[th]) != 0) return -1;
        o += 17 + nv;
      }
    } else if (m == 0xC0 || m == 0xC1) {         // baseline / extended sequential, Huffman
      if (sl < 6 || s[0] != 8) return -1;
      d.h = (s[1] << 8) | s[2];
      d.w = (s[3] << 8) | s[4];
      d.ncomp = s[5];
      if (d.h <= 0 || d.w <= 0 || (d.ncomp != 1 && d.ncomp != 3) || sl < 6 + 3 * d.ncomp) return -1;
      for (int c = 0; c < d.ncomp; ++c) {
        cid[c] = s[6 + 3 * c];
        d.hs[c] = s[7 + 3 * c] >> 4;
        d.vs[c] = s[7 + 3 * c] & 15;
        d.tq[c] = s[8 + 3 * c];
        if (d.tq[c] > 3 || d.hs[c] < 1 || d.vs[c] < 1) return -1;
      }
      have_sof = true;
    } else if ((m >= 0xC2 && m <= 0xCF) && m != 0xC4 && m != 0xC8 && m != 0xCC) {
      return -1;                                 // progressive / lossless / arithmetic: CPU path
    } else if (m == 0xDD) {                      // DRI
      if (sl < 2) return -1;
      if (((s[0] << 8) | s[1]) != 0) return -1;  // restart markers: CPU path
    } else if (m == 0xDA) {                      // SOS
      if (!have_sof || sl < 1) return -1;
      const int ns = s[0];
      if (ns != d.ncomp || sl < 1 + 2 * ns + 3) return -1;
      for (int j = 0; j < ns; ++j) {
        const int id = s[1 + 2 * j];
        int c = -1;
        for (int k = 0; k < d.ncomp; ++k)
          if (cid[k] == id) c = k;
        if (c != j) return -1;
        d.td[c] = s[2 + 2 * j] >> 4;
        d.ta[c] = s[2 + 2 * j] & 15;
        if (d.td[c] > 3 || d.ta[c] > 3) return -1;
      }
      const uint8_t* ss = s + 1 + 2 * ns;
      if (ss[0] != 0 || ss[1] != 63 || ss[2] != 0) return -1;
      // entropy-coded data: un-stuff FF00 until the next marker (data that just ends —
      // a truncated file — is left to the CPU path, which reports it failed as Pillow does)
      int64_t j = i + seglen, o = 0;
      bool ended = false;
      while (j < len) {
        // copy the run up to the next 0xFF at once (entropy bytes are mostly not 0xFF)
        const uint8_t* ff = (const uint8_t*)memchr(p + j, 0xFF, (size_t)(len - j));
        const int64_t run = ff ? ff - (p + j) : len - j;
        if (run > 0) {
          if (o + run > cap) return -1;
          memcpy(out + o, p + j, (size_t)run);
          o += run;
          j += run;
          if (j >= len) break;
        }
        const uint8_t b = p[j];
        if (b == 0xFF) {
          if (j + 1 >= len) break;
          const uint8_t nx = p[j + 1];
          if (nx == 0x00) {
            if (o >= cap) return -1;
            out[o++] = 0xFF;
            j += 2;
            continue;
          }
          if (nx == 0xFF) {  // fill byte
            ++j;
            continue;
          }
          if (nx >= 0xD0 && nx <= 0xD7) return -1;  // RST without DRI
          // any other marker ends the scan: a second SOS (multi-scan) is not supported
          int64_t k = j + 1;
          while (k < len && p[k] == 0xFF) ++k;
          if (k < len && p[k] == 0xDA) return -1;
          ended = true;
          break;
        }
        if (o >= cap) return -1;
        out[o++] = b;
        ++j;
      }
      if (!ended) return -1;
      d.stream_len = (int)o;
      break;
    }
    i += seglen;
  }
  if (!have_sof || d.stream_len <= 0) return -1;
  // colour space as libjpeg guesses it (jdapimin.c): 3 components are YCbCr unless an Adobe
  // marker says transform 0 or, with neither JFIF nor Adobe, the ids spell R G B
  if (d.ncomp == 3) {
    if (adobe && adobe_transform == 0) return -1;
    if (!jfif && !adobe && cid[0] == 'R' && cid[1] == 'G' && cid[2] == 'B') return -1;
  }
  (void)qdef;
  for (int c = 0; c < d.ncomp; ++c)
    if (!qdef[d.tq[c]]) return -1;
  // geometry (jdinput.c)
  if (d.ncomp == 1) {
    d.hs[0] = d.vs[0] = 1;
    d.hmax = d.vmax = 1;
    d.mcux = (d.w + 7) / 8;
    d.mcuy = (d.h + 7) / 8;
    d.bw[0] = d.mcux;
    d.bh[0] = d.mcuy;
    d.dw[0] = d.w;
    d.dh[0] = d.h;
  } else {
    const bool s420 = d.hs[0] == 2 && d.vs[0] == 2 && d.hs[1] == 1 && d.vs[1] == 1 && d.hs[2] == 1 && d.vs[2] == 1;
    const bool s444 = d.hs[0] == 1 && d.vs[0] == 1 && d.hs[1] == 1 && d.vs[1] == 1 && d.hs[2] == 1 && d.vs[2] == 1;
    if (!s420 && !s444) return -1;  // 4:2:2 / 4:4:0 / exotic: CPU path
    d.hmax = d.hs[0];
    d.vmax = d.vs[0];
    d.mcux = (d.w + 8 * d.hmax - 1) / (8 * d.hmax);
    d.mcuy = (d.h + 8 * d.vmax - 1) / (8 * d.vmax);
    for (int c = 0; c < 3; ++c) {
      d.bw[c] = d.mcux * d.hs[c];
      d.bh[c] = d.mcuy * d.vs[c];
      d.dw[c] = (d.w * d.hs[c] + d.hmax - 1) / d.hmax;
      d.dh[c] = (d.h * d.vs[c] + d.vmax - 1) / d.vmax;
    }
  }
  if (d.stream_len > DMLJ_MAXSTREAM) return -1;
  if (outH > 0) {
    if (outH > DMLJ_MAXOUT || outW > DMLJ_MAXOUT) return -1;
    nearest_tab(d.h, outH, d.rowtab);
    nearest_tab(d.w, outW, d.coltab);
  }
  d.outH = outH;
  d.outW = outW;
  for (int k = 0; k < 64; ++k) d.izz[kNatural[k]] = (uint8_t)k;
  d.ok = 1;
  return 0;
}

}  // namespace jpg
}  // namespace dml

using dml::jpg::parse_one;

// Layout of `buf` (pinned host memory, copied to the device as is): int64 n, int64 work bytes,
// n x DmljImage, then each image's entropy bytes (16-aligned). status[i] = 1: decoded on the
// GPU; 0: unsupported / corrupt (the caller decodes it on the CPU). Returns the bytes used, or
// -1 if `cap` is too small. info[0] = bytes of the device work buffer the decode needs
// (coefficients, then sample planes), info[1] = bytes of its coefficient part (zeroed before the
// launch), info[2] = the most 8x8 blocks of one image, info[3] = the longest entropy segment.
extern "C" long dml_jpeg_prepare(int n, const unsigned char* const* datas, const long* lens, int outH, int outW,
                                 void* buf, long cap, int* status, long* info) {
  unsigned char* b = (unsigned char*)buf;
  const long hdr = 16 + (long)n * (long)sizeof(DmljImage);
  if (cap < hdr) return -1;
  DmljImage* d = (DmljImage*)(b + 16);
  long off = (hdr + 15) / 16 * 16;
  int64_t ncoef = 0;
  long maxblk = 0, maxstream = 0;
  for (int i = 0; i < n; ++i) {
    const long room = cap - off;
    status[i] = 0;
    if (room <= 0 || parse_one(datas[i], lens[i], d[i], b + off, room, outH, outW) != 0) {
      memset(&d[i], 0, sizeof(DmljImage));
      continue;
    }
    d[i].stream_off = off;
    const long padded = (d[i].stream_len + 8 + 15) / 16 * 16;   // >= 8 zero bytes for the bit reader
    if (off + padded > cap) {
      memset(&d[i], 0, sizeof(DmljImage));
      continue;
    }
    memset(b + off + d[i].stream_len, 0, (size_t)(padded - d[i].stream_len));
    dml::jpg::swap_words(b + off, padded);
    off += padded;
    int nb = 0;
    for (int c = 0; c < d[i].ncomp; ++c) {
      d[i].coef_off[c] = ncoef;
      ncoef += (int64_t)d[i].bw[c] * d[i].bh[c] * 64;
      nb += d[i].bw[c] * d[i].bh[c];
    }
    d[i].nblk = nb;
    maxblk = nb > maxblk ? nb : maxblk;
    maxstream = d[i].stream_len > maxstream ? d[i].stream_len : maxstream;
    status[i] = 1;
  }
  int64_t pl = (ncoef * 2 + 255) / 256 * 256;
  info[1] = (long)pl;
  info[2] = maxblk;
  info[3] = maxstream;
  for (int i = 0; i < n; ++i) {
    if (!d[i].ok) continue;
    for (int c = 0; c < d[i].ncomp; ++c) {
      d[i].plane_off[c] = pl;
      pl += ((int64_t)d[i].bw[c] * 8 * d[i].bh[c] * 8 + 255) / 256 * 256;
    }
  }
  info[0] = (long)pl;
  ((int64_t*)b)[0] = n;
  ((int64_t*)b)[1] = pl;
  return off;
}

// set the arena slot of image i (host side, before the H2D copy)
extern "C" void dml_jpeg_set_slot(void* buf, int i, int slot) { ((DmljImage*)((unsigned char*)buf + 16))[i].slot = slot; }

// the same for n images in one call (idx == null: images 0..n-1): the serve loop issued one ctypes
// call per image, holding the GIL between them (256 per window)
extern "C" void dml_jpeg_set_slots(void* buf, const int* idx, const int* slots, int n) {
  DmljImage* d = (DmljImage*)((unsigned char*)buf + 16);
  for (int j = 0; j < n; ++j) d[idx ? idx[j] : j].slot = slots[j];
}

extern "C" int dml_jpeg_decode_resize(const void* dbuf, int n, int maxblk, long maxstream, void* dwork, int H, int W,
                                      void* arena, hipStream_t s) {
  if (n <= 0) return 0;
  if (H <= 0 || W <= 0 || H > DMLJ_MAXOUT || W > DMLJ_MAXOUT || maxstream > DMLJ_MAXSTREAM) {
    dml_set_error("dml_jpeg_decode_resize: bad output size or stream");
    return -1;
  }
  const unsigned char* b = (const unsigned char*)dbuf;
  int16_t* coef = (int16_t*)dwork;
  // the parallel segment decode (a workgroup per image); DML_JPEG_SERIAL=1: the r5 one-wave serial
  // decode (A/B)
  static const bool serial = getenv("DML_JPEG_SERIAL") && getenv("DML_JPEG_SERIAL")[0] == '1';
  // DML_JPEG_PT=64/128/256: segments (threads) per image (A/B; default DMLJ_PT_GPU)
  static const int pt = getenv("DML_JPEG_PT") ? atoi(getenv("DML_JPEG_PT")) : DMLJ_PT_GPU;
  if (serial)
    hipLaunchKernelGGL(dml::jpg::jpeg_huff_kernel, dim3(n), dim3(64), 0, s, b, n, coef);
  else if (pt == 512)
    hipLaunchKernelGGL(dml::jpg::jpeg_huff_par_kernel<512>, dim3(n), dim3(512), 0, s, b, n, coef);
  else if (pt == 256)
    hipLaunchKernelGGL(dml::jpg::jpeg_huff_par_kernel<256>, dim3(n), dim3(256), 0, s, b, n, coef);
  else if (pt == 128)
    hipLaunchKernelGGL(dml::jpg::jpeg_huff_par_kernel<128>, dim3(n), dim3(128), 0, s, b, n, coef);
  else
    hipLaunchKernelGGL(dml::jpg::jpeg_huff_par_kernel<64>, dim3(n), dim3(64), 0, s, b, n, coef);
  DML_CHECK_LAUNCH();
  hipLaunchKernelGGL(dml::jpg::jpeg_idct_kernel, dim3((maxblk + 255) / 256, n), dim3(256), 0, s, b, n, coef,
                     (uint8_t*)dwork);
  DML_CHECK_LAUNCH();
  hipLaunchKernelGGL(dml::jpg::jpeg_rgb_resize_kernel, dim3(H, n), dim3(256), 0, s, b, n, (const uint8_t*)dwork, H, W,
                     (uint8_t*)arena);
  DML_CHECK_LAUNCH();
  return 0;
}

// the whole GPU decode of a window in one call (GpuRankBackend's serve loop issued the H2D copy,
// the coefficient zeroing and the launch as three Python calls): pinned pack -> device copy,
// zeroed coefficient region, then the decode kernels, all on stream s
extern "C" int dml_jpeg_launch(const void* host, void* dev, long used, void* dwork, long coef_bytes, int n, int maxblk,
                               long maxstream, int H, int W, void* arena, hipStream_t s) {
  if (used <= 0 || coef_bytes < 0) {
    dml_set_error("dml_jpeg_launch: bad sizes");
    return -1;
  }
  if (hipMemcpyAsync(dev, host, (size_t)used, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemsetAsync(dwork, 0, (size_t)coef_bytes, s) != hipSuccess) {
    dml_set_error("dml_jpeg_launch: copy / memset failed");
    return -1;
  }
  return dml_jpeg_decode_resize(dev, n, maxblk, maxstream, dwork, H, W, arena, s);
}

// a decoded image's descriptor re-targeted to another output size (the other model's window):
// dst <- src with that size's NEAREST tables and ABSOLUTE plane addresses (base + plane_off), for
// dml_jpeg_resize_only — the image is decoded once for both models
extern "C" void dml_jpeg_retarget(void* dst, const void* src, int outH, int outW, long base) {
  DmljImage* d = (DmljImage*)dst;
  memcpy(d, src, offsetof(DmljImage, q));   // the colour + resize kernel reads nothing past it
  if (!d->ok || outH <= 0 || outW <= 0 || outH > DMLJ_MAXOUT || outW > DMLJ_MAXOUT) {
    d->ok = 0;
    return;
  }
  dml::jpg::nearest_tab(d->h, outH, d->rowtab);
  dml::jpg::nearest_tab(d->w, outW, d->coltab);
  d->outH = outH;
  d->outW = outW;
  for (int c = 0; c < d->ncomp; ++c) d->plane_off[c] += base;
}

// n re-targets in one call: dst + 16 + j * desc <- srcs[j] with base bases[j] (the other model's
// window: one native call instead of one per image from the decode pool)
extern "C" void dml_jpeg_retarget_many(void* dst, const void* const* srcs, const long* bases, int n, int outH,
                                       int outW) {
  unsigned char* b = (unsigned char*)dst + 16;
  for (int j = 0; j < n; ++j) dml_jpeg_retarget(b + (long)j * (long)sizeof(DmljImage), srcs[j], outH, outW, bases[j]);
}

// colour + resize only, from planes a dml_jpeg_decode_resize launch left (descriptors from
// dml_jpeg_retarget, in a buffer laid out as dml_jpeg_prepare's: int64 n, int64 0, records)
extern "C" int dml_jpeg_resize_only(const void* dbuf, int n, int H, int W, void* arena, hipStream_t s) {
  if (n <= 0) return 0;
  if (H <= 0 || W <= 0 || H > DMLJ_MAXOUT || W > DMLJ_MAXOUT) {
    dml_set_error("dml_jpeg_resize_only: bad output size");
    return -1;
  }
  hipLaunchKernelGGL(dml::jpg::jpeg_rgb_resize_kernel, dim3(H, n), dim3(256), 0, s, (const unsigned char*)dbuf, n,
                     (const uint8_t*)nullptr, H, W, (uint8_t*)arena);
  DML_CHECK_LAUNCH();
  return 0;
}

extern "C" int dml_jpeg_init(void) { return 0; }   // nothing to set up (kept for the backend's init order)

extern "C" long dml_jpeg_desc_size(void) { return (long)sizeof(DmljImage); }

// the descriptor's leading part a re-target needs (geometry, plane offsets, NEAREST tables): the
// plane cache keeps only this much per image
extern "C" long dml_jpeg_head_size(void) { return (long)offsetof(DmljImage, q); }

// CPU replay of jpeg_huff_par_kernel's algorithm (tests): the coefficient blocks of the parallel
// decode (coef_par) and of the serial one (coef_ser), each ncoef int16; info = {ncoef, Jacobi
// rounds, segments}; info[1] on entry: at most this many segments (0 = DMLJ_PT). 0 = ok,
// -1 = unsupported, -2 = the buffers are too small.
extern "C" int dml_jpeg_parallel_host(const unsigned char* data, long len, short* coef_par, short* coef_ser,
                                      long cap, long* info) {
  using namespace dml::jpg;
  DmljImage d;
  static thread_local uint8_t* stream = nullptr;
  if (!stream) stream = (uint8_t*)malloc(1 << 24);
  if (parse_one(data, len, d, stream, (1 << 24) - 16, 0, 0) != 0) return -1;
  memset(stream + d.stream_len, 0, 16);
  swap_words(stream, (d.stream_len + 8 + 15) / 16 * 16);
  int64_t ncoef = 0;
  for (int c = 0; c < d.ncomp; ++c) {
    d.coef_off[c] = ncoef;
    ncoef += (int64_t)d.bw[c] * d.bh[c] * 64;
  }
  info[0] = (long)ncoef;
  if (ncoef > cap) return -2;
  memset(coef_par, 0, (size_t)ncoef * 2);
  memset(coef_ser, 0, (size_t)ncoef * 2);
  decode_entropy(d, (const uint32_t*)stream, coef_ser, true);
  const McuMap m = mcu_map(d);
  static thread_local uint16_t t11[6][1 << DMLJ_LA];
  for (int c = 0; c < d.ncomp; ++c)
    for (int j = 0; j < (1 << DMLJ_LA); ++j) {
      t11[c][j] = t11_entry(d.dc[d.td[c]], j);
      t11[3 + c][j] = t11_entry(d.ac[d.ta[c]], j);
    }
  const SegTabs tb = {&t11[0][0]};
  const uint32_t* w = (const uint32_t*)stream;
  const int nw = (d.stream_len + 3) / 4;
  const int want = info[1] > 0 && info[1] <= 512 ? (int)info[1] : DMLJ_PT;   // segments (A/B: up to 512)
  const int SEG = seg_bits(d, want), nbits = d.stream_len * 8, nseg = (nbits + SEG - 1) / SEG;
  PState start[512], ex[512], nex[512];
  int nb[512] = {0};
  for (int t = 0; t < nseg; ++t) {
    start[t] = PState{t * SEG, 0, 0};
    ex[t] = seg_decode<false>(d, m, tb, w, nw, start[t], std::min((t + 1) * SEG, nbits), &nb[t], 0, nullptr);
  }
  int rounds = 0;
  for (int r = 0; r < nseg; ++r) {
    bool changed = false;
    for (int t = 0; t < nseg; ++t) {
      nex[t] = ex[t];
      if (t == 0) continue;
      const PState st = ex[t - 1];
      if (st.pos == start[t].pos && st.u == start[t].u && st.k == start[t].k) continue;
      start[t] = st;
      nex[t] = seg_decode<false>(d, m, tb, w, nw, st, std::min((t + 1) * SEG, nbits), &nb[t], 0, nullptr);
      changed |= nex[t].pos != ex[t].pos || nex[t].u != ex[t].u || nex[t].k != ex[t].k;
    }
    for (int t = 0; t < nseg; ++t) ex[t] = nex[t];
    ++rounds;
    if (!changed) break;
  }
  int gb = 0;
  for (int t = 0; t < nseg; ++t) {
    int dummy;
    seg_decode<true>(d, m, tb, w, nw, start[t], std::min((t + 1) * SEG, nbits), &dummy, gb, coef_par);
    gb += nb[t];
  }
  for (int c = 0; c < d.ncomp; ++c) {
    const int hs = d.ncomp == 1 ? 1 : d.hs[c], vs = d.ncomp == 1 ? 1 : d.vs[c];
    int pred = 0;
    for (int j = 0; j < d.bw[c] * d.bh[c]; ++j) {
      const int mcu = j / (hs * vs), ww = j - mcu * (hs * vs);
      const int v = ww / hs, h = ww - v * hs;
      const int my = mcu / d.mcux, mx = mcu - my * d.mcux;
      int16_t* p = coef_par + d.coef_off[c] + ((int64_t)(my * vs + v) * d.bw[c] + (mx * hs + h)) * 64;
      pred += *p;
      *p = (int16_t)pred;
    }
  }
  info[1] = rounds;
  info[2] = nseg;
  return 0;
}

// CPU decode with the same code (tests): full-resolution RGB into out (h*w*3); 0 = ok,
// -1 = unsupported (the CPU workers' path)
extern "C" int dml_jpeg_decode_host(const unsigned char* data, long len, unsigned char* out, int* hw) {
  DmljImage d;
  static thread_local uint8_t* stream = nullptr;
  if (!stream) stream = (uint8_t*)malloc(1 << 24);
  if (parse_one(data, len, d, stream, (1 << 24) - 16, 0, 0) != 0) return -1;
  memset(stream + d.stream_len, 0, 16);   // the bit reader's zero padding
  dml::jpg::swap_words(stream, (d.stream_len + 8 + 15) / 16 * 16);
  hw[0] = d.h;
  hw[1] = d.w;
  int64_t ncoef = 0;
  for (int c = 0; c < d.ncomp; ++c) {
    d.coef_off[c] = ncoef;
    ncoef += (int64_t)d.bw[c] * d.bh[c] * 64;
  }
  int64_t pl = ncoef * 2;
  for (int c = 0; c < d.ncomp; ++c) {
    d.plane_off[c] = pl;
    pl += (int64_t)d.bw[c] * 8 * d.bh[c] * 8;
  }
  uint8_t* work = (uint8_t*)calloc((size_t)pl, 1);
  if (!work) return -1;
  int16_t* coef = (int16_t*)work;
  dml::jpg::decode_entropy(d, (const uint32_t*)stream, coef, true);
  for (int c = 0; c < d.ncomp; ++c) {
    const int pw = d.bw[c] * 8;
    for (int by = 0; by < d.bh[c]; ++by)
      for (int bx = 0; bx < d.bw[c]; ++bx)
      {
        const int16_t* zz = coef + d.coef_off[c] + ((int64_t)by * d.bw[c] + bx) * 64;
        int16_t in[64];
        for (int j = 0; j < 64; ++j) in[j] = zz[d.izz[j]];
        dml::jpg::idct_islow(in, d.q[d.tq[c]], work + d.plane_off[c] + (int64_t)by * 8 * pw + bx * 8, pw);
      }
  }
  for (int y = 0; y < d.h; ++y)
    for (int x = 0; x < d.w; ++x) dml::jpg::rgb_at(d, work, y, x, out + ((int64_t)y * d.w + x) * 3);
  free(work);
  return 0;
}
