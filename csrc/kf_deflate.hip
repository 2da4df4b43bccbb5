// kf_deflate.hip — device GeoTIFF tile encoder (kf_deflate.h): predictor 3 +
// one fixed-Huffman zlib stream per 256 x 256 float32 tile, then the tiles
// packed back to back.  Reference-cadence output (observations.py:354-394)
// then ships compressed tiles to the host instead of raw planes, and the host
// writer only writes files.
//
// Launch: one workgroup of 256 threads per tile (thread = tile row), grid =
// planes x tiles (a 10980^2 x 7 date: 12,943 workgroups, 50 per CU).
//   pass 1: each thread encodes its row once, into a word-aligned scratch
//           slot of its own, with the Adler-32 partials; a workgroup scan
//           gives every row its bit offset in the stream;
//   pass 2: each thread moves its row's words to that offset (a shift).
//           Words wholly inside a row's range are stored directly; the one
//           word a row shares with the next (its tail) goes through LDS and is
//           OR-ed into the next row's head word, so no atomics and no zeroed
//           buffer are needed (every row emits >= 65 bits, so a word never
//           spans three rows).
// Thread 0 prepends the zlib header and the block header, thread 255 appends
// the end-of-block code, the byte padding and the Adler-32 (big-endian).
#include <hip/hip_runtime.h>

#include "kf_deflate.h"
#include "kf_launch.h"

namespace kf {

__global__ __launch_bounds__(DFL_TILE) void dfl_tile_kernel(DflArgs a) {
  const int tile = blockIdx.x;
  const int per = a.tiles_x * a.tiles_y;
  const int plane = tile / per, tt = tile - plane * per;
  const int ty = tt / a.tiles_x, tx = tt - ty * a.tiles_x;
  const int r = threadIdx.x;
  const int64_t y = (int64_t)ty * DFL_TILE + r;
  const int x0 = tx * DFL_TILE;
  const bool rin = y < a.H;
  const int ncol = a.W - x0 < DFL_TILE ? a.W - x0 : DFL_TILE;
  const float* rowp = a.src + (int64_t)plane * a.plane_ld + (rin ? y : 0) * a.W + x0;
  // the row's samples in groups of 16: one burst of independent loads into this
  // thread's LDS line per group (the encoder reads columns in order, 4 passes
  // over the row, one per byte plane), instead of one dependent load per byte
  __shared__ uint32_t line[DFL_TILE][17];
  auto row = [&](int c) -> uint32_t {
    if ((c & 15) == 0) {
      uint32_t v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = (rin && c + j < ncol) ? __float_as_uint(rowp[c + j]) : 0u;
#pragma unroll
      for (int j = 0; j < 16; ++j) line[r][j] = v[j];
    }
    return line[r][c & 15];
  };
  const int64_t rest = DFL_RAW - (int64_t)r * DFL_ROW;

  // pass 1: the row's bit string into its own word-aligned scratch slot (one
  // encode of the row), its length and Adler partials
  uint32_t* rs = reinterpret_cast<uint32_t*>(a.scratch) + ((int64_t)tile * DFL_TILE + r) * DFL_ROW_WORDS;
  uint64_t nbits = 0, s1 = 0, s2 = 0;
  {
    uint64_t acc = 0;
    int nacc = 0, wi = 0;
    dfl_encode_row(row, rest, [&](uint32_t bits, int len) {
      acc |= (uint64_t)bits << nacc;
      nacc += len;
      nbits += (uint64_t)len;
      if (nacc >= 32) {
        rs[wi++] = (uint32_t)acc;
        acc >>= 32;
        nacc -= 32;
      }
    }, s1, s2);
    if (nacc > 0) rs[wi] = (uint32_t)acc;
  }
  KF_DCHECK(nbits >= 64 && nbits <= 32u * DFL_ROW_WORDS);

  __shared__ uint64_t scan[DFL_TILE];
  __shared__ uint64_t red1[DFL_TILE / 64], red2[DFL_TILE / 64];
  __shared__ uint32_t tail[DFL_TILE];
  scan[r] = nbits;
  uint64_t w1 = s1, w2 = s2;
  for (int o = 32; o > 0; o >>= 1) {
    w1 += __shfl_down(w1, o, 64);
    w2 += __shfl_down(w2, o, 64);
  }
  if ((r & 63) == 0) {
    red1[r >> 6] = w1;
    red2[r >> 6] = w2;
  }
  __syncthreads();
  // inclusive Hillis-Steele scan of the row bit counts
  for (int o = 1; o < DFL_TILE; o <<= 1) {
    const uint64_t v = r >= o ? scan[r - o] : 0;
    __syncthreads();
    scan[r] += v;
    __syncthreads();
  }
  const uint64_t start = DFL_HEAD_BITS + scan[r] - nbits;
  uint64_t t1 = 0, t2 = 0;
#pragma unroll
  for (int w = 0; w < DFL_TILE / 64; ++w) {
    t1 += red1[w];
    t2 += red2[w];
  }
  const uint32_t adler = dfl_adler(t1, t2, DFL_RAW);

  // pass 2: the row's words shifted to its bit offset in the stream.  Words
  // wholly inside the row's range are stored; the word shared with the next
  // row goes through LDS (every row emits >= 65 bits: no word spans 3 rows)
  uint32_t* out = reinterpret_cast<uint32_t*>(a.out + (int64_t)tile * DFL_BOUND);
  const bool shared_left = r > 0 && (start & 31u) != 0;
  uint64_t wi = start >> 5;
  uint64_t acc = 0;
  int nacc = (int)(start & 31u);
  if (r == 0) {
    acc = 0x0178u | (1u << 16) | (1u << 17);   // 78 01, BFINAL = 1, BTYPE = 01 (fixed Huffman)
    nacc = DFL_HEAD_BITS;
  }
  uint32_t head = 0;
  bool first = true;
  auto put = [&](uint32_t v) {
    if (first && shared_left) head = v;
    else out[wi] = v;
    first = false;
    ++wi;
  };
  auto sink = [&](uint32_t bits, int len) {
    acc |= (uint64_t)bits << nacc;
    nacc += len;
    while (nacc >= 32) {
      put((uint32_t)acc);
      acc >>= 32;
      nacc -= 32;
    }
  };
  const int full = (int)(nbits >> 5), part = (int)(nbits & 31u);
  for (int k = 0; k < full; ++k) sink(rs[k], 32);
  if (part) sink(rs[full] & ((1u << part) - 1u), part);
  if (r == DFL_TILE - 1) {
    sink(0u, 7);                                       // end of block (code 256: 7 zero bits)
    const int pad = (8 - (int)(((wi << 5) + nacc) & 7u)) & 7;
    if (pad) sink(0u, pad);
    for (int k = 3; k >= 0; --k) sink((adler >> (8 * k)) & 0xFFu, 8);   // Adler-32, big-endian bytes
    const uint64_t end_bits = (wi << 5) + nacc;
    if (nacc > 0) out[wi] = (uint32_t)acc;             // the stream's last word: nobody shares it
    a.sizes[tile] = (uint32_t)(end_bits >> 3);
  } else if (nacc > 0) {
    tail[r] = (uint32_t)acc;                           // shared with row r + 1's head word
  }
  __syncthreads();
  if (shared_left) out[start >> 5] = head | tail[r - 1];
}

// tile t's stream (sizes[t] bytes at t * DFL_BOUND) -> packed + offs[t]
__global__ __launch_bounds__(256) void dfl_pack_kernel(const uint8_t* scratch, const uint32_t* sizes,
                                                       const int64_t* offs, uint8_t* packed) {
  const int t = blockIdx.x;
  const uint32_t n = sizes[t];
  const uint8_t* src = scratch + (int64_t)t * DFL_BOUND;
  uint8_t* dst = packed + offs[t];
  for (uint32_t i = threadIdx.x; i < n; i += 256) dst[i] = src[i];
}

hipError_t dev_deflate_tiles(const DflArgs& a, hipStream_t s) {
  const int n = a.nplanes * a.tiles_x * a.tiles_y;
  if (n <= 0 || a.W <= 0 || a.H <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(dfl_tile_kernel, dim3(n), dim3(DFL_TILE), 0, s, a);
  return hipGetLastError();
}

hipError_t dev_deflate_pack(const uint8_t* scratch, const uint32_t* sizes, const int64_t* offs, uint8_t* packed,
                            int ntiles, hipStream_t s) {
  if (ntiles <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(dfl_pack_kernel, dim3(ntiles), dim3(256), 0, s, scratch, sizes, offs, packed);
  return hipGetLastError();
}

}  // namespace kf
