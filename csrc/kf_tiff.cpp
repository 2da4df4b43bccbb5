// kf_tiff.cpp — native (Geo)TIFF I/O for granule-scale rasters.
//
// The reference reads and writes every raster through GDAL
// (Sentinel2_Observations.py:148-185, observations.py:354-394: DEFLATE,
// TILED, BIGTIFF, SetProjection).  GDAL is not in this stack, and a 10980^2
// granule pushed through Python zlib one strip at a time costs seconds per
// band, so this file decodes and encodes strips / tiles on a thread pool,
// straight from / into caller memory (pinned host buffers that feed the
// device by hipMemcpyAsync on the side stream, input_output/streaming.py).
//
//   read : classic + BigTIFF, little-endian, strips or tiles, uncompressed or
//          DEFLATE (8 / 32946), predictor 1 / 2 (integer) / 3 (float), one
//          sample per pixel or planar multi-band; a row/column window of one
//          band is decoded into a dense row-major buffer.
//   write: tiled (default 256 x 256) DEFLATE planar rasters, BigTIFF when the
//          file can exceed 4 GiB, GeoTIFF georeferencing: ModelPixelScale,
//          ModelTiepoint and a GeoKeyDirectory with GTModelType, GTRasterType,
//          ProjectedCSType / GeographicType (EPSG) and the WKT as citation;
//          GDAL_NODATA; optional horizontal predictor 2 / 3 and zlib strategy
//          (RLE / Huffman-only for fast float output).  Tiles are compressed in
//          parallel and written with parallel pwrite; uncompressed rasters are
//          written as whole-row strips straight from the caller's planes.
//          The zlib streams come from libdeflate when the system has it
//          (libdeflate.so.0, dlopen'ed: 3-4x zlib's speed for the same
//          standard stream, so TIFF compression 8 and every reader are
//          unchanged), else from zlib with the requested strategy.
#include <dlfcn.h>
#include <fcntl.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include "kf_tiff.h"

#include <algorithm>
#include <atomic>
#include <functional>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace py = pybind11;

namespace kf {
namespace tiff {

struct Info {
  uint64_t W = 0, H = 0;
  int spp = 1, bits = 8, fmt = 1, comp = 1, pred = 1, planar = 1;
  bool big = false, tiled = false;
  uint64_t tw = 0, th = 0, rps = 0;
  std::vector<uint64_t> off, cnt;
  std::vector<double> scale, tie;
  std::vector<uint16_t> geokeys;
  std::string ascii, nodata;
};

struct File {
  int fd = -1;
  explicit File(const std::string& p, int flags = O_RDONLY, int mode = 0644) {
    fd = ::open(p.c_str(), flags, mode);
    if (fd < 0) throw std::runtime_error("cannot open " + p);
  }
  ~File() {
    if (fd >= 0) ::close(fd);
  }
  void read_at(void* dst, size_t n, uint64_t off) const {
    char* d = static_cast<char*>(dst);
    while (n) {
      const ssize_t r = ::pread(fd, d, n, (off_t)off);
      if (r <= 0) throw std::runtime_error("short read");
      d += r;
      n -= (size_t)r;
      off += (uint64_t)r;
    }
  }
  void write_at(const void* src, size_t n, uint64_t off) const {
    const char* s = static_cast<const char*>(src);
    while (n) {
      const ssize_t r = ::pwrite(fd, s, n, (off_t)off);
      if (r <= 0) throw std::runtime_error("short write");
      s += r;
      n -= (size_t)r;
      off += (uint64_t)r;
    }
  }
};

static size_t type_size(int t) {
  switch (t) {
    case 1: case 2: case 6: case 7: return 1;
    case 3: case 8: return 2;
    case 4: case 9: case 11: return 4;
    case 5: case 10: case 12: case 16: case 17: return 8;
    default: return 1;
  }
}

template <typename T>
static T rd(const uint8_t* p) {
  T v;
  std::memcpy(&v, p, sizeof(T));
  return v;
}

static std::vector<uint64_t> as_u64(const std::vector<uint8_t>& b, int typ, uint64_t n) {
  std::vector<uint64_t> v(n);
  for (uint64_t i = 0; i < n; ++i) {
    switch (typ) {
      case 1: v[i] = b[i]; break;
      case 3: v[i] = rd<uint16_t>(&b[2 * i]); break;
      case 4: v[i] = rd<uint32_t>(&b[4 * i]); break;
      case 16: v[i] = rd<uint64_t>(&b[8 * i]); break;
      default: throw std::runtime_error("unexpected integer TIFF field type");
    }
  }
  return v;
}

Info parse(const File& f) {
  uint8_t hdr[16];
  f.read_at(hdr, 16, 0);
  if (hdr[0] != 'I' || hdr[1] != 'I') throw std::runtime_error("big-endian TIFF not supported natively");
  Info in;
  const uint16_t magic = rd<uint16_t>(hdr + 2);
  in.big = magic == 43;
  if (magic != 42 && magic != 43) throw std::runtime_error("not a TIFF file");
  const uint64_t ifd = in.big ? rd<uint64_t>(hdr + 8) : rd<uint32_t>(hdr + 4);
  uint8_t nb[8];
  f.read_at(nb, in.big ? 8 : 2, ifd);
  const uint64_t n = in.big ? rd<uint64_t>(nb) : rd<uint16_t>(nb);
  const size_t ent = in.big ? 20 : 12, inl = in.big ? 8 : 4;
  std::vector<uint8_t> e(n * ent);
  f.read_at(e.data(), e.size(), ifd + (in.big ? 8 : 2));
  for (uint64_t i = 0; i < n; ++i) {
    const uint8_t* p = &e[i * ent];
    const uint16_t tag = rd<uint16_t>(p), typ = rd<uint16_t>(p + 2);
    const uint64_t cnt = in.big ? rd<uint64_t>(p + 4) : rd<uint32_t>(p + 4);
    const uint8_t* val = p + (in.big ? 12 : 8);
    const size_t sz = type_size(typ) * cnt;
    std::vector<uint8_t> data(sz);
    if (sz <= inl) {
      std::memcpy(data.data(), val, sz);
    } else {
      const uint64_t o = in.big ? rd<uint64_t>(val) : rd<uint32_t>(val);
      f.read_at(data.data(), sz, o);
    }
    auto u = [&]() { return as_u64(data, typ, cnt); };
    // first value of a scalar tag; a count of 0 is a malformed IFD, not UB
    auto u0 = [&]() -> uint64_t {
      if (cnt < 1) throw std::runtime_error("TIFF tag " + std::to_string(tag) + " has no value");
      return as_u64(data, typ, 1)[0];
    };
    switch (tag) {
      case 256: in.W = u0(); break;
      case 257: in.H = u0(); break;
      case 258: in.bits = (int)u0(); break;
      case 259: in.comp = (int)u0(); break;
      case 277: in.spp = (int)u0(); break;
      case 278: in.rps = u0(); break;
      case 284: in.planar = (int)u0(); break;
      case 317: in.pred = (int)u0(); break;
      case 322: in.tw = u0(); in.tiled = true; break;
      case 323: in.th = u0(); break;
      case 273: case 324: in.off = u(); break;
      case 279: case 325: in.cnt = u(); break;
      case 339: in.fmt = (int)u0(); break;
      case 33550: in.scale.resize(cnt); std::memcpy(in.scale.data(), data.data(), sz); break;
      case 33922: in.tie.resize(cnt); std::memcpy(in.tie.data(), data.data(), sz); break;
      case 34735: in.geokeys.resize(cnt); std::memcpy(in.geokeys.data(), data.data(), sz); break;
      case 34737: in.ascii.assign((const char*)data.data(), strnlen((const char*)data.data(), sz)); break;
      case 42113: in.nodata.assign((const char*)data.data(), strnlen((const char*)data.data(), sz)); break;
      default: break;
    }
  }
  if (!in.W || !in.H || in.off.empty() || in.off.size() != in.cnt.size()) throw std::runtime_error("bad TIFF IFD");
  if (in.bits <= 0 || in.bits % 8 != 0 || in.bits > 64)
    throw std::runtime_error("unsupported TIFF sample size: " + std::to_string(in.bits) + " bits");
  if (in.tiled && (!in.tw || !in.th)) throw std::runtime_error("bad TIFF tile size");
  if (!in.rps) in.rps = in.H;
  // every chunk must lie inside the file (a hostile or truncated table would
  // otherwise read past EOF or allocate an arbitrary buffer)
  struct stat sb;
  if (::fstat(f.fd, &sb) != 0) throw std::runtime_error("fstat failed");
  const uint64_t fsz = (uint64_t)sb.st_size;
  for (size_t i = 0; i < in.off.size(); ++i)
    if (in.off[i] > fsz || in.cnt[i] > fsz - in.off[i])
      throw std::runtime_error("TIFF chunk " + std::to_string(i) + " lies outside the file");
  return in;
}

// Undo the horizontal predictor of one decoded chunk row (w samples of `bps` bytes).
static void undo_predictor(uint8_t* row, uint64_t w, int bps, int pred) {
  if (pred == 2) {
    switch (bps) {
      case 1: for (uint64_t i = 1; i < w; ++i) row[i] = (uint8_t)(row[i] + row[i - 1]); break;
      case 2: {
        uint16_t* r = reinterpret_cast<uint16_t*>(row);
        for (uint64_t i = 1; i < w; ++i) r[i] = (uint16_t)(r[i] + r[i - 1]);
      } break;
      case 4: {
        uint32_t* r = reinterpret_cast<uint32_t*>(row);
        for (uint64_t i = 1; i < w; ++i) r[i] += r[i - 1];
      } break;
      default: {
        uint64_t* r = reinterpret_cast<uint64_t*>(row);
        for (uint64_t i = 1; i < w; ++i) r[i] += r[i - 1];
      }
    }
  } else if (pred == 3) {
    // floating-point predictor: bytes differenced, then stored most
    // significant byte plane first (TIFF Technical Note 3)
    const uint64_t nbytes = w * (uint64_t)bps;
    for (uint64_t i = 1; i < nbytes; ++i) row[i] = (uint8_t)(row[i] + row[i - 1]);
    std::vector<uint8_t> tmp(row, row + nbytes);
    for (uint64_t i = 0; i < w; ++i)
      for (int b = 0; b < bps; ++b) row[i * bps + b] = tmp[(uint64_t)(bps - 1 - b) * w + i];
  }
}

// Apply the horizontal predictor to one chunk row before compression (inverse of undo_predictor).
static void apply_predictor(uint8_t* row, uint64_t w, int bps, int pred, std::vector<uint8_t>& tmp) {
  if (pred == 2) {
    switch (bps) {
      case 1: for (uint64_t i = w - 1; i > 0; --i) row[i] = (uint8_t)(row[i] - row[i - 1]); break;
      case 2: {
        uint16_t* r = reinterpret_cast<uint16_t*>(row);
        for (uint64_t i = w - 1; i > 0; --i) r[i] = (uint16_t)(r[i] - r[i - 1]);
      } break;
      case 4: {
        uint32_t* r = reinterpret_cast<uint32_t*>(row);
        for (uint64_t i = w - 1; i > 0; --i) r[i] -= r[i - 1];
      } break;
      default: {
        uint64_t* r = reinterpret_cast<uint64_t*>(row);
        for (uint64_t i = w - 1; i > 0; --i) r[i] -= r[i - 1];
      }
    }
  } else if (pred == 3) {
    const uint64_t nbytes = w * (uint64_t)bps;
    tmp.assign(row, row + nbytes);
    for (uint64_t i = 0; i < w; ++i)
      for (int b = 0; b < bps; ++b) row[(uint64_t)(bps - 1 - b) * w + i] = tmp[i * bps + b];
    for (uint64_t i = nbytes - 1; i > 0; --i) row[i] = (uint8_t)(row[i] - row[i - 1]);
  }
}

// libdeflate's stable C API, resolved at run time (no headers in this image)
struct FastDeflate {
  void* (*alloc)(int) = nullptr;
  size_t (*compress)(void*, const void*, size_t, void*, size_t) = nullptr;
  size_t (*bound)(void*, size_t) = nullptr;
  void (*release)(void*) = nullptr;
  bool ok = false;
  FastDeflate() {
    void* h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    alloc = reinterpret_cast<void* (*)(int)>(dlsym(h, "libdeflate_alloc_compressor"));
    compress = reinterpret_cast<size_t (*)(void*, const void*, size_t, void*, size_t)>(
        dlsym(h, "libdeflate_zlib_compress"));
    bound = reinterpret_cast<size_t (*)(void*, size_t)>(dlsym(h, "libdeflate_zlib_compress_bound"));
    release = reinterpret_cast<void (*)(void*)>(dlsym(h, "libdeflate_free_compressor"));
    ok = alloc && compress && bound && release;
  }
  static const FastDeflate& get() {
    static const FastDeflate f;
    return f;
  }
};

// one compressor per thread and level (libdeflate's are not thread safe)
struct ThreadCompressor {
  void* c = nullptr;
  int level = -1;
  ~ThreadCompressor() {
    if (c) FastDeflate::get().release(c);
  }
  void* at(int lv) {
    if (lv != level) {
      if (c) FastDeflate::get().release(c);
      c = FastDeflate::get().alloc(lv);
      level = lv;
    }
    return c;
  }
};

// zlib even where libdeflate is present (A/B of the two encoders: tiff_deflate_backend)
static std::atomic<bool> g_force_zlib{false};

static bool use_fast_deflate() { return FastDeflate::get().ok && !g_force_zlib.load(std::memory_order_relaxed); }

bool fast_deflate_available() { return use_fast_deflate(); }

static void parallel_for(int64_t n, int nthreads, const std::function<void(int64_t)>& fn) {
  nthreads = std::max(1, std::min<int>(nthreads, (int)std::max<int64_t>(1, n)));
  std::atomic<int64_t> next{0};
  std::exception_ptr err;
  std::atomic<bool> failed{false};
  auto work = [&]() {
    for (int64_t i = next++; i < n && !failed; i = next++) {
      try {
        fn(i);
      } catch (...) {
        if (!failed.exchange(true)) err = std::current_exception();
      }
    }
  };
  std::vector<std::thread> ts;
  for (int t = 1; t < nthreads; ++t) ts.emplace_back(work);
  work();
  for (auto& t : ts) t.join();
  if (err) std::rethrow_exception(err);
}

// Decode rows [r0, r1) x columns [c0, c1) of sample `band` into dst (dense, row-major).
void read_window(const std::string& path, int band, void* dst, uint64_t r0, uint64_t r1, uint64_t c0, uint64_t c1,
                 int nthreads, int elem_bytes) {
  File f(path);
  const Info in = parse(f);
  // the destination was sized by the caller for elem_bytes per sample: a file
  // of another sample size would overflow (or half-fill) it
  if (elem_bytes > 0 && in.bits / 8 != elem_bytes)
    throw std::runtime_error("TIFF samples are " + std::to_string(in.bits) + "-bit, the destination expects " +
                             std::to_string(8 * elem_bytes) + "-bit");
  if (in.spp > 1 && in.planar != 2) throw std::runtime_error("pixel-interleaved multi-band TIFF not supported natively");
  if (band < 0 || band >= in.spp) throw std::runtime_error("band out of range");
  if (r1 > in.H || c1 > in.W || r0 >= r1 || c0 >= c1) throw std::runtime_error("window outside the raster");
  if (in.comp != 1 && in.comp != 8 && in.comp != 32946) throw std::runtime_error("unsupported TIFF compression");
  const int bps = in.bits / 8;
  const uint64_t cw = in.tiled ? in.tw : in.W, ch = in.tiled ? in.th : in.rps;
  const uint64_t across = in.tiled ? (in.W + cw - 1) / cw : 1, down = (in.H + ch - 1) / ch;
  const uint64_t per_band = across * down;
  if (in.off.size() < per_band * (uint64_t)(band + 1)) throw std::runtime_error("truncated chunk table");
  // chunks overlapping the window
  std::vector<uint64_t> chunks;
  for (uint64_t ty = r0 / ch; ty <= (r1 - 1) / ch; ++ty)
    for (uint64_t tx = c0 / cw; tx <= (c1 - 1) / cw; ++tx) chunks.push_back(ty * across + tx);
  uint8_t* out = static_cast<uint8_t*>(dst);
  const uint64_t ow = c1 - c0;
  parallel_for((int64_t)chunks.size(), nthreads, [&](int64_t k) {
    const uint64_t id = chunks[k], ty = id / across, tx = id % across;
    const uint64_t cid = per_band * (uint64_t)band + id;
    const uint64_t rows = in.tiled ? ch : std::min<uint64_t>(ch, in.H - ty * ch);
    const uint64_t raw = rows * cw * (uint64_t)bps;
    // some writers pad a compressed last strip to the full RowsPerStrip: room
    // for a whole strip, of which the rows inside the raster are used
    const uint64_t room = ch * cw * (uint64_t)bps;
    std::vector<uint8_t> comp(in.cnt[cid]), buf(room);
    f.read_at(comp.data(), comp.size(), in.off[cid]);
    if (in.comp == 1) {
      if (comp.size() < raw) throw std::runtime_error("truncated TIFF chunk " + std::to_string(cid) + " in " + path);
      std::memcpy(buf.data(), comp.data(), raw);
    } else {
      // a good chunk is a complete stream that fills at least the rows inside
      // the raster and at most a whole strip / tile (Z_BUF_ERROR = truncated or
      // corrupt input, or more data than a chunk holds)
      uLongf dl = (uLongf)room;
      const int rc = uncompress(buf.data(), &dl, comp.data(), (uLong)comp.size());
      if (rc != Z_OK || dl < (uLongf)raw)
        throw std::runtime_error("inflate failed (zlib " + std::to_string(rc) + ", " + std::to_string(dl) + " of " +
                                 std::to_string(raw) + " bytes) for chunk " + std::to_string(cid) + " in " + path);
    }
    if (in.pred != 1)
      for (uint64_t r = 0; r < rows; ++r) undo_predictor(buf.data() + r * cw * bps, cw, bps, in.pred);
    const uint64_t gy0 = ty * ch, gx0 = tx * cw;
    const uint64_t ya = std::max(gy0, r0), yb = std::min(gy0 + rows, r1);
    const uint64_t xa = std::max(gx0, c0), xb = std::min(gx0 + cw, std::min(c1, in.W));
    for (uint64_t y = ya; y < yb; ++y)
      std::memcpy(out + ((y - r0) * ow + (xa - c0)) * bps, buf.data() + ((y - gy0) * cw + (xa - gx0)) * bps,
                  (xb - xa) * bps);
  });
}

// ---------------------------------------------------------------- writer
struct Tag {
  uint16_t tag, typ;
  uint64_t count;
  std::vector<uint8_t> bytes;
};

template <typename T>
static Tag mk(uint16_t tag, uint16_t typ, const std::vector<T>& v) {
  Tag t{tag, typ, v.size(), {}};
  t.bytes.resize(v.size() * sizeof(T));
  if (!v.empty()) std::memcpy(t.bytes.data(), v.data(), t.bytes.size());
  return t;
}
static Tag mk_ascii(uint16_t tag, const std::string& s) {
  Tag t{tag, 2, s.size() + 1, {}};
  t.bytes.assign(s.begin(), s.end());
  t.bytes.push_back(0);
  return t;
}

// Raw file of n bytes written by parallel pwrite of 64 MiB pieces (checkpoint
// payloads: a 10980^2 PROSAIL state is ~31 GB); optional fsync before return.
void write_raw(const std::string& path, const void* data, uint64_t n, int nthreads, bool sync) {
  File f(path, O_WRONLY | O_CREAT | O_TRUNC);
  if (n && ::ftruncate(f.fd, (off_t)n) != 0) throw std::runtime_error("ftruncate failed: " + path);
  const uint64_t piece = 64ull << 20, np = (n + piece - 1) / piece;
  const uint8_t* src = static_cast<const uint8_t*>(data);
  parallel_for((int64_t)np, nthreads, [&](int64_t i) {
    const uint64_t off = (uint64_t)i * piece;
    f.write_at(src + off, std::min(piece, n - off), off);
  });
  if (sync && ::fsync(f.fd) != 0) throw std::runtime_error("fsync failed: " + path);
}

void write_chunks(const std::string& path, int nb, uint64_t H, uint64_t W, int bits, int fmt, uint32_t tile,
                  uint64_t rps, int comp, int predictor, const std::vector<uint64_t>& cnts,
                  const std::function<const uint8_t*(uint64_t)>& chunk, int nthreads, const std::vector<double>& gt,
                  int epsg, const std::string& citation, const std::string& nodata, int force_big);

void write(const std::string& path, const void* data, int nb, uint64_t H, uint64_t W, int bits, int fmt,
           uint32_t tile, int level, int nthreads, const std::vector<double>& gt, int epsg,
           const std::string& citation, const std::string& nodata, int force_big, int predictor, int strategy) {
  if (predictor == 3 && fmt != 3) throw std::runtime_error("predictor 3 needs floating-point samples");
  if (level <= 0) predictor = 1;
  const int bps = bits / 8;
  // uncompressed: strips of whole rows written straight from the caller's
  // planes (zero copy, parallel pwrite); compressed: tiles deflated on the pool
  const bool striped = level <= 0;
  const uint64_t row_bytes = W * (uint64_t)bps;
  const uint64_t rps = striped ? std::max<uint64_t>(1, std::min<uint64_t>(H, (4ull << 20) / std::max<uint64_t>(1, row_bytes))) : 0;
  const uint64_t nstrip = striped ? (H + rps - 1) / rps : 0;
  const uint64_t across = (W + tile - 1) / tile, down = (H + tile - 1) / tile;
  const uint64_t nchunk = striped ? nstrip * (uint64_t)nb : across * down * (uint64_t)nb;
  const uint64_t traw = (uint64_t)tile * tile * bps;
  std::vector<std::vector<uint8_t>> enc(striped ? 0 : nchunk);
  const uint8_t* src = static_cast<const uint8_t*>(data);
  auto strip_ptr = [&](uint64_t i) {
    const uint64_t b = i / nstrip, st = i % nstrip;
    return src + (b * H + st * rps) * row_bytes;
  };
  auto strip_bytes = [&](uint64_t i) { return std::min<uint64_t>(rps, H - (i % nstrip) * rps) * row_bytes; };
  if (!striped) {
    parallel_for((int64_t)nchunk, nthreads, [&](int64_t i) {
      const uint64_t b = (uint64_t)i / (across * down), id = (uint64_t)i % (across * down);
      const uint64_t ty = id / across, tx = id % across;
      // per-thread scratch reused across tiles (no page faults per tile)
      thread_local std::vector<uint8_t> t, c, tmp;
      const uint64_t y0 = ty * tile, x0 = tx * tile;
      const uint64_t rows = std::min<uint64_t>(tile, H - y0), cols = std::min<uint64_t>(tile, W - x0);
      t.resize(traw);
      if (rows < tile || cols < tile) std::fill(t.begin(), t.end(), 0);   // edge tiles zero padded (TIFF 6.0 §15)
      const uint8_t* plane = src + b * H * W * bps;
      for (uint64_t r = 0; r < rows; ++r)
        std::memcpy(&t[r * tile * bps], plane + ((y0 + r) * W + x0) * bps, cols * bps);
      if (predictor > 1)
        for (uint64_t r = 0; r < tile; ++r) apply_predictor(&t[r * tile * bps], tile, bps, predictor, tmp);
      const FastDeflate& fd = FastDeflate::get();
      // libdeflate has no zlib strategies: a requested Z_RLE / Z_HUFFMAN_ONLY
      // (--out-fast) always runs zlib, so its speed and ratio do not depend on
      // which libraries the host has
      if (use_fast_deflate() && strategy == Z_DEFAULT_STRATEGY) {
        thread_local ThreadCompressor tc;
        void* comp = tc.at(std::min(level, 12));
        if (!comp) throw std::runtime_error("libdeflate_alloc_compressor failed");
        c.resize(fd.bound(comp, traw));
        const size_t n = fd.compress(comp, t.data(), traw, c.data(), c.size());
        if (n == 0) throw std::runtime_error("libdeflate_zlib_compress failed");
        enc[i].assign(c.begin(), c.begin() + n);
        return;
      }
      // zlib stream (TIFF compression 8); strategy Z_RLE / Z_HUFFMAN_ONLY trade a
      // little ratio for ~3x encode speed on float rasters
      z_stream zs{};
      if (deflateInit2(&zs, level, Z_DEFLATED, 15, 8, strategy) != Z_OK) throw std::runtime_error("deflateInit2 failed");
      c.resize(deflateBound(&zs, (uLong)traw));
      zs.next_in = t.data();
      zs.avail_in = (uInt)traw;
      zs.next_out = c.data();
      zs.avail_out = (uInt)c.size();
      const int rc = deflate(&zs, Z_FINISH);
      deflateEnd(&zs);
      if (rc != Z_STREAM_END) throw std::runtime_error("deflate failed");
      enc[i].assign(c.begin(), c.begin() + zs.total_out);
    });
  }
  std::vector<uint64_t> cnts(nchunk);
  for (uint64_t i = 0; i < nchunk; ++i) cnts[i] = striped ? strip_bytes(i) : enc[i].size();
  write_chunks(path, nb, H, W, bits, fmt, striped ? 0u : tile, rps, level > 0 ? 8 : 1, predictor, cnts,
               [&](uint64_t i) { return striped ? strip_ptr(i) : enc[i].data(); }, nthreads, gt, epsg, citation,
               nodata, force_big);
}

// The file of a raster whose chunks (tiles, or strips when tile == 0) are
// already encoded: header, chunk payloads (parallel pwrite), IFD with the
// GeoTIFF tags.  comp: TIFF compression tag (1 / 8).
void write_chunks(const std::string& path, int nb, uint64_t H, uint64_t W, int bits, int fmt, uint32_t tile,
                  uint64_t rps, int comp, int predictor, const std::vector<uint64_t>& cnts,
                  const std::function<const uint8_t*(uint64_t)>& chunk, int nthreads, const std::vector<double>& gt,
                  int epsg, const std::string& citation, const std::string& nodata, int force_big) {
  const bool striped = tile == 0;
  const uint64_t nchunk = cnts.size();
  std::vector<uint64_t> offs(nchunk);
  uint64_t payload = 0;
  for (auto c : cnts) payload += c + (c & 1);
  const bool big = force_big > 0 || (force_big < 0 && payload > 3500000000ull);
  const uint64_t hdr = big ? 16 : 8;
  uint64_t pos = hdr;
  for (uint64_t i = 0; i < nchunk; ++i) {
    offs[i] = pos;
    pos += cnts[i] + (cnts[i] & 1);
  }
  std::vector<Tag> tags;
  const uint16_t L = big ? 16 : 4;   // LONG8 / LONG for offsets and counts
  tags.push_back(mk<uint32_t>(256, 4, {(uint32_t)W}));
  tags.push_back(mk<uint32_t>(257, 4, {(uint32_t)H}));
  tags.push_back(mk<uint16_t>(258, 3, std::vector<uint16_t>(nb, (uint16_t)bits)));
  tags.push_back(mk<uint16_t>(259, 3, {(uint16_t)comp}));
  tags.push_back(mk<uint16_t>(262, 3, {1}));
  tags.push_back(mk<uint16_t>(277, 3, {(uint16_t)nb}));
  tags.push_back(mk<uint16_t>(284, 3, {(uint16_t)(nb > 1 ? 2 : 1)}));
  tags.push_back(mk<uint16_t>(317, 3, {(uint16_t)predictor}));
  // tiles: TileWidth/Length + TileOffsets/ByteCounts; strips: RowsPerStrip +
  // StripOffsets/ByteCounts
  const uint16_t t_off = striped ? 273 : 324, t_cnt = striped ? 279 : 325;
  if (striped) {
    tags.push_back(mk<uint32_t>(278, 4, {(uint32_t)rps}));
  } else {
    tags.push_back(mk<uint32_t>(322, 4, {tile}));
    tags.push_back(mk<uint32_t>(323, 4, {tile}));
  }
  if (big) {
    tags.push_back(mk<uint64_t>(t_off, L, offs));
    tags.push_back(mk<uint64_t>(t_cnt, L, cnts));
  } else {
    std::vector<uint32_t> o32(offs.begin(), offs.end()), c32(cnts.begin(), cnts.end());
    tags.push_back(mk<uint32_t>(t_off, L, o32));
    tags.push_back(mk<uint32_t>(t_cnt, L, c32));
  }
  tags.push_back(mk<uint16_t>(339, 3, std::vector<uint16_t>(nb, (uint16_t)fmt)));
  if (gt.size() == 6) {
    tags.push_back(mk<double>(33550, 12, {gt[1], -gt[5], 0.0}));
    tags.push_back(mk<double>(33922, 12, {0.0, 0.0, 0.0, gt[0], gt[3], 0.0}));
    // GeoKeyDirectory: header, then (key, location, count, value) sorted by key
    const bool geographic = epsg >= 4000 && epsg < 5000;
    const std::string cit = (citation.empty() ? std::string("unknown") : citation) + "|";
    std::vector<uint16_t> keys = {1, 1, 0, 0};
    auto key = [&](uint16_t k, uint16_t loc, uint16_t cnt, uint16_t v) {
      keys.insert(keys.end(), {k, loc, cnt, v});
      keys[3]++;
    };
    key(1024, 0, 1, epsg > 0 ? (geographic ? 2 : 1) : 32767);   // GTModelType
    key(1025, 0, 1, 1);                                          // GTRasterType: PixelIsArea
    key(1026, 34737, (uint16_t)std::min<size_t>(cit.size(), 65535), 0);   // GTCitation
    if (epsg > 0 && geographic) key(2048, 0, 1, (uint16_t)epsg);           // GeographicType
    if (epsg > 0 && !geographic) key(3072, 0, 1, (uint16_t)epsg);          // ProjectedCSType
    tags.push_back(mk<uint16_t>(34735, 3, keys));
    tags.push_back(mk_ascii(34737, cit));
  }
  if (!nodata.empty()) tags.push_back(mk_ascii(42113, nodata));
  std::sort(tags.begin(), tags.end(), [](const Tag& a, const Tag& b) { return a.tag < b.tag; });
  // IFD after the data; out-of-line values after the IFD
  const uint64_t ifd = pos;
  const size_t ent = big ? 20 : 12, inl = big ? 8 : 4;
  const uint64_t ifd_bytes = (big ? 8 : 2) + ent * tags.size() + (big ? 8 : 4);
  std::vector<uint8_t> ifdb(ifd_bytes, 0), extra;
  uint8_t* p = ifdb.data();
  if (big) {
    const uint64_t n = tags.size();
    std::memcpy(p, &n, 8);
    p += 8;
  } else {
    const uint16_t n = (uint16_t)tags.size();
    std::memcpy(p, &n, 2);
    p += 2;
  }
  for (auto& t : tags) {
    std::memcpy(p, &t.tag, 2);
    std::memcpy(p + 2, &t.typ, 2);
    if (big) {
      std::memcpy(p + 4, &t.count, 8);
    } else {
      const uint32_t c = (uint32_t)t.count;
      std::memcpy(p + 4, &c, 4);
    }
    uint8_t* val = p + (big ? 12 : 8);
    if (t.bytes.size() <= inl) {
      std::memcpy(val, t.bytes.data(), t.bytes.size());
    } else {
      const uint64_t o = ifd + ifd_bytes + extra.size();
      if (big) std::memcpy(val, &o, 8);
      else {
        const uint32_t o32 = (uint32_t)o;
        std::memcpy(val, &o32, 4);
      }
      extra.insert(extra.end(), t.bytes.begin(), t.bytes.end());
      if (extra.size() & 1) extra.push_back(0);
    }
    p += ent;
  }
  if (!big && ifd + ifd_bytes + extra.size() > 0xFFFFFFFFull) throw std::runtime_error("classic TIFF overflow");
  File f(path, O_WRONLY | O_CREAT | O_TRUNC);
  uint8_t h[16] = {'I', 'I'};
  if (big) {
    const uint16_t m = 43, b8 = 8, z = 0;
    std::memcpy(h + 2, &m, 2);
    std::memcpy(h + 4, &b8, 2);
    std::memcpy(h + 6, &z, 2);
    std::memcpy(h + 8, &ifd, 8);
  } else {
    const uint16_t m = 42;
    const uint32_t o = (uint32_t)ifd;
    std::memcpy(h + 2, &m, 2);
    std::memcpy(h + 4, &o, 4);
  }
  f.write_at(h, hdr, 0);
  // chunk payloads in parallel pwrite (disjoint ranges)
  parallel_for((int64_t)nchunk, std::max(1, std::min(nthreads, 8)), [&](int64_t i) {
    if (cnts[i]) f.write_at(chunk((uint64_t)i), cnts[i], offs[i]);
  });
  f.write_at(ifdb.data(), ifdb.size(), ifd);
  if (!extra.empty()) f.write_at(extra.data(), extra.size(), ifd + ifd_bytes);
}

}  // namespace tiff

void bind_tiff(py::module_& m) {
  m.def("tiff_info", [](const std::string& path) {
    tiff::File f(path);
    const tiff::Info in = tiff::parse(f);
    py::dict d;
    d["width"] = in.W;
    d["height"] = in.H;
    d["bands"] = in.spp;
    d["bits"] = in.bits;
    d["sample_format"] = in.fmt;
    d["compression"] = in.comp;
    d["predictor"] = in.pred;
    d["planar"] = in.planar;
    d["tiled"] = in.tiled;
    d["tile"] = py::make_tuple(in.tw, in.th);
    d["rows_per_strip"] = in.rps;
    d["bigtiff"] = in.big;
    d["pixel_scale"] = in.scale;
    d["tiepoint"] = in.tie;
    d["geokeys"] = in.geokeys;
    d["geo_ascii"] = in.ascii;
    d["nodata"] = in.nodata;
    d["n_chunks"] = in.off.size();
    return d;
  });
  m.def("tiff_read", [](const std::string& path, int band, uintptr_t dst, uint64_t r0, uint64_t r1, uint64_t c0,
                        uint64_t c1, int nthreads, int elem_bytes) {
    py::gil_scoped_release nogil;
    tiff::read_window(path, band, reinterpret_cast<void*>(dst), r0, r1, c0, c1, nthreads, elem_bytes);
  }, py::arg("path"), py::arg("band"), py::arg("dst"), py::arg("r0"), py::arg("r1"), py::arg("c0"), py::arg("c1"),
     py::arg("nthreads"), py::arg("elem_bytes") = 0);
  m.def("tiff_fast_deflate", &tiff::fast_deflate_available,
        "True when tile DEFLATE uses libdeflate (else zlib)");
  m.def("tiff_deflate_backend", [](const std::string& b) {
    if (b != "auto" && b != "zlib") throw std::invalid_argument("deflate backend: 'auto' or 'zlib'");
    tiff::g_force_zlib.store(b == "zlib");
    return tiff::fast_deflate_available();
  }, "DEFLATE encoder of the TIFF writer: 'auto' (libdeflate when present) or 'zlib'; returns tiff_fast_deflate()");
  m.def("write_raw", [](const std::string& path, uintptr_t src, uint64_t n, int nthreads, bool sync) {
    py::gil_scoped_release nogil;
    tiff::write_raw(path, reinterpret_cast<const void*>(src), n, nthreads, sync);
  });
  m.def("tiff_write", [](const std::string& path, uintptr_t src, int nb, uint64_t H, uint64_t W, int bits, int fmt,
                         uint32_t tile, int level, int nthreads, const std::vector<double>& gt, int epsg,
                         const std::string& citation, const std::string& nodata, int force_big, int predictor,
                         int strategy) {
    py::gil_scoped_release nogil;
    tiff::write(path, reinterpret_cast<const void*>(src), nb, H, W, bits, fmt, tile, level, nthreads, gt, epsg,
                citation, nodata, force_big, predictor, strategy);
  }, py::arg("path"), py::arg("src"), py::arg("nb"), py::arg("H"), py::arg("W"), py::arg("bits"), py::arg("fmt"),
     py::arg("tile"), py::arg("level"), py::arg("nthreads"), py::arg("gt"), py::arg("epsg"), py::arg("citation"),
     py::arg("nodata"), py::arg("force_big"), py::arg("predictor") = 1, py::arg("strategy") = 0);
  // tiles already encoded (the device encoder, kf_deflate.hip): data + offsets[i]
  // holds sizes[i] bytes of tile i (row-major tiles of one band)
  m.def("tiff_write_tiles", [](const std::string& path, uintptr_t data, uint64_t H, uint64_t W, int bits, int fmt,
                               uint32_t tile, int comp, int predictor, const std::vector<uint64_t>& offsets,
                               const std::vector<uint64_t>& sizes, int nthreads, const std::vector<double>& gt,
                               int epsg, const std::string& citation, const std::string& nodata, int force_big) {
    const uint64_t n = ((W + tile - 1) / tile) * ((H + tile - 1) / tile);
    if (offsets.size() != n || sizes.size() != n) throw std::runtime_error("tiff_write_tiles: one offset and size per tile");
    if (tile == 0 || tile % 16) throw std::runtime_error("tiff_write_tiles: tile edge must be a multiple of 16");
    py::gil_scoped_release nogil;
    const uint8_t* base = reinterpret_cast<const uint8_t*>(data);
    tiff::write_chunks(path, 1, H, W, bits, fmt, tile, 0, comp, predictor, sizes,
                       [&](uint64_t i) { return base + offsets[i]; }, nthreads, gt, epsg, citation, nodata, force_big);
  });
}

}  // namespace kf
