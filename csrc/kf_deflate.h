// kf_deflate.h — GeoTIFF tile encoding on the device: the TIFF floating-point
// predictor (predictor 3) and a zlib stream per 256 x 256 float32 tile, for
// reference-cadence output (every parameter's mean and uncertainty raster at
// every timestep, observations.py:354-394 / linear_kf.py:211-212).
//
// One tile = 256 rows of 1024 predicted bytes = one zlib stream (TIFF
// compression 8): the 2-byte header 78 01, ONE final DEFLATE block with the
// fixed Huffman codes (RFC 1951 §3.2.6), the Adler-32 of the predicted bytes.
// The LZ77 part is run-length only (distance 1, lengths 3..258), the same
// match family as zlib's Z_RLE strategy that ``--out-fast`` selects on the
// host, and every row starts with a literal: each row's symbols depend on
// that row alone, so one thread encodes one row.  The row encoder below is
// the source both the gfx950 kernel (kf_deflate.hip: one workgroup per tile,
// bit offsets by a workgroup scan) and the host runner (tests, CPU builds)
// execute, so their streams are bit-identical.
//
// Predictor 3 (TIFF Technical Note 3): each row's samples are split into byte
// planes, most significant byte first, and the 4 x 256 bytes are differenced
// (d[0] = r[0], d[i] = r[i] - r[i - 1] mod 256).
#pragma once
#include <stdint.h>
#include "kf_core.h"

namespace kf {

constexpr int DFL_TILE = 256;                                   // tile edge (pixels)
constexpr int DFL_ROW = DFL_TILE * 4;                           // predicted bytes per row
constexpr int64_t DFL_RAW = (int64_t)DFL_TILE * DFL_ROW;        // 262144 bytes per tile
// worst case: header 2 + (19 + 9 bits per byte + 7 EOB + 7 pad) / 8 + Adler 4, rounded to 16
constexpr int64_t DFL_BOUND = ((2 + (19 + 9 * DFL_RAW + 14) / 8 + 4) + 15) / 16 * 16;
constexpr int DFL_HEAD_BITS = 19;   // zlib header (16) + BFINAL/BTYPE (3)
// scratch words of one encoded row (9 bits per byte at most, plus a partial word)
constexpr int DFL_ROW_WORDS = (9 * DFL_ROW + 31) / 32 + 1;
constexpr uint32_t DFL_ADLER_MOD = 65521u;

KF_HD uint32_t dfl_rev(uint32_t code, int len) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_bitreverse32(code) >> (32 - len);
#else
  uint32_t r = 0;
  for (int i = 0; i < len; ++i) r |= ((code >> i) & 1u) << (len - 1 - i);
  return r;
#endif
}

// fixed-Huffman literal: (bits LSB-first, length)
KF_HD void dfl_lit(uint32_t v, uint32_t& bits, int& len) {
  if (v < 144u) {
    len = 8;
    bits = dfl_rev(0x30u + v, 8);
  } else {
    len = 9;
    bits = dfl_rev(0x190u + (v - 144u), 9);
  }
}

// run-length match of length L (3..258) at distance 1: length code + extra
// bits + the 5-bit distance code 0, as one LSB-first bit string
KF_HD void dfl_match(int L, uint32_t& bits, int& len) {
  int code, e = 0, ev = 0;
  if (L == 258) {
    code = 285;
  } else if (L <= 10) {
    code = 254 + L;
  } else {
    const int n = L - 3;
    int lg = 0;
    while ((n >> (lg + 1)) != 0) ++lg;        // floor(log2 n), n in [8, 254]
    e = lg - 2;
    code = 261 + 4 * e + (n >> e) - 4;
    ev = n & ((1 << e) - 1);
  }
  uint32_t c;
  int cl;
  if (code < 280) {
    c = dfl_rev((uint32_t)(code - 256), 7);
    cl = 7;
  } else {
    c = dfl_rev(0xC0u + (uint32_t)(code - 280), 8);
    cl = 8;
  }
  bits = c | ((uint32_t)ev << cl);   // distance code 0 (5 zero bits) follows
  len = cl + e + 5;
}

// byte i of a predicted row (before differencing) from the row's samples
// (float bits; samples past the raster are 0): plane i / 256 is the sample's
// byte 3 - i / 256 (most significant first)
template <typename ROW>
KF_HD uint32_t dfl_row_byte(const ROW& row, int i) {
  const int k = i >> 8, c = i & 255;
  return (row(c) >> (8 * (3 - k))) & 0xFFu;
}

// Encodes one tile row: SINK(bits, len) receives the LSB-first bit strings in
// order.  Also returns the row's Adler-32 partial sums over its predicted bytes
// d: s1 = sum d, s2 = sum (rest - i) d with rest = bytes from the row's start
// to the end of the tile.
template <typename ROW, typename SINK>
KF_HD void dfl_encode_row(const ROW& row, int64_t rest, SINK&& sink, uint64_t& s1, uint64_t& s2) {
  uint32_t prev = dfl_row_byte(row, 0);
  uint32_t last = prev;           // the last byte of the output so far (d)
  uint32_t b;
  int l;
  dfl_lit(last, b, l);
  sink(b, l);
  s1 = last;
  s2 = (uint64_t)rest * last;
  int run = 0;                    // bytes equal to `last` not yet emitted
  auto flush = [&]() {
    if (run >= 3) {
      dfl_match(run, b, l);
      sink(b, l);
    } else {
      for (int j = 0; j < run; ++j) {
        dfl_lit(last, b, l);
        sink(b, l);
      }
    }
    run = 0;
  };
  for (int i = 1; i < DFL_ROW; ++i) {
    const uint32_t r = dfl_row_byte(row, i);
    const uint32_t d = (r - prev) & 0xFFu;
    prev = r;
    s1 += d;
    s2 += (uint64_t)(rest - i) * d;
    if (d == last && run < 258) {
      ++run;
      continue;
    }
    flush();
    if (d == last) {              // a full 258 run ended: the next run repeats it
      run = 1;
      continue;
    }
    dfl_lit(d, b, l);
    sink(b, l);
    last = d;
  }
  flush();
}

// Adler-32 from the tile's summed partials (n bytes)
KF_HD uint32_t dfl_adler(uint64_t s1, uint64_t s2, int64_t n) {
  const uint32_t a = (uint32_t)((1u + s1) % DFL_ADLER_MOD);
  const uint32_t b = (uint32_t)(((uint64_t)n + s2) % DFL_ADLER_MOD);
  return (b << 16) | a;
}

}  // namespace kf
