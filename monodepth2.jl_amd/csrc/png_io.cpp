// Native host data pipeline: PNG decode of the Depth10k / KITTI triplets
// straight into the library's uint8 batch layout, on host threads.
//
// The reference loads with FileIO/PNGFiles (libpng) and slices / resizes in Julia
// (src/dtk.jl:29-46, src/kitty.jl:45-61); the Python mirror decodes with PIL, whose decoder holds
// the GIL between IDAT blocks, so worker THREADS scale poorly (2.2x on 8 threads, measured).  Here
// every sample is decoded on a std::thread: zlib inflate of the IDAT stream, PNG row unfiltering
// (None / Sub / Up / Average / Paeth), then one pass that writes the frames in [n][3][C][H][W]
// order (the Depth10k split at width*j, dtk.jl:36; the HWC -> CHW transpose; FlipX's mirror) or,
// for KITTI, ImageTransformations' imresize to the target size kept N0f8 (kitty.jl:52; restated in
// md2hip/data.py and pinned there).  PNG decoding is lossless: the bytes equal PIL's / libpng's.
// Supported: 8-bit, non-interlaced, colour types 0 (gray), 2 (RGB), 4 (gray+alpha, alpha dropped),
// 6 (RGBA, alpha dropped) -- what both datasets ship.  This file is host code only.
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <string>
#include <thread>
#include <vector>

#include "../../include/md2.h"
#include "common.h"

namespace md2 {
namespace {

struct Png {
  int w = 0, h = 0, ch = 0;             // channels in the decoded buffer (1, 2, 3 or 4)
  std::vector<unsigned char> px;        // h * w * ch, row-major, interleaved
};

inline unsigned be32(const unsigned char* p) {
  return ((unsigned)p[0] << 24) | ((unsigned)p[1] << 16) | ((unsigned)p[2] << 8) | p[3];
}

inline unsigned char paeth(int a, int b, int c) {
  const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
  return (unsigned char)((pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c));
}

bool read_file(const char* path, std::vector<unsigned char>& buf, std::string& err) {
  FILE* f = std::fopen(path, "rb");
  if (!f) {
    err = std::string("cannot open ") + path;
    return false;
  }
  std::fseek(f, 0, SEEK_END);
  const long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  buf.resize(n > 0 ? (size_t)n : 0);
  const size_t got = n > 0 ? std::fread(buf.data(), 1, (size_t)n, f) : 0;
  std::fclose(f);
  if ((long)got != n) {
    err = std::string("short read ") + path;
    return false;
  }
  return true;
}

// Largest image side accepted (KITTI is 1241x376, a Depth10k triplet 1248x128): a corrupt or
// hostile header must not size an allocation.
constexpr unsigned kMaxSide = 1u << 14;

// exp_w / exp_h > 0: the caller's expected size, checked against IHDR before anything is
// allocated.
bool decode_png(const char* path, Png& out, std::string& err, int exp_w = 0, int exp_h = 0) {
  std::vector<unsigned char> f;
  if (!read_file(path, f, err)) return false;
  static const unsigned char sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  if (f.size() < 33 || std::memcmp(f.data(), sig, 8) != 0) {
    err = std::string("not a PNG file: ") + path;
    return false;
  }
  size_t pos = 8;
  int depth = 0, ctype = -1, interlace = 0;
  z_stream zs{};
  std::vector<unsigned char> raw;
  bool zinit = false, done = false;
  while (pos + 12 <= f.size() && !done) {
    const unsigned len = be32(&f[pos]);
    const unsigned char* type = &f[pos + 4];
    const unsigned char* data = &f[pos + 8];
    if (pos + 12 + (size_t)len > f.size()) {
      err = std::string("truncated chunk in ") + path;
      break;
    }
    if (!std::memcmp(type, "IHDR", 4)) {
      if (zinit || len != 13) {
        err = std::string(zinit ? "repeated IHDR in " : "bad IHDR length in ") + path;
        break;
      }
      const unsigned w = be32(data), h = be32(data + 4);
      if (w == 0 || h == 0 || w > kMaxSide || h > kMaxSide) {
        err = std::string("PNG size out of range (") + std::to_string(w) + "x" + std::to_string(h) + "): " + path;
        return false;
      }
      out.w = (int)w;
      out.h = (int)h;
      if ((exp_w > 0 && out.w != exp_w) || (exp_h > 0 && out.h != exp_h)) {
        err = std::string(path) + ": expected " + std::to_string(exp_w) + "x" + std::to_string(exp_h) + ", got " +
              std::to_string(out.w) + "x" + std::to_string(out.h);
        return false;
      }
      depth = data[8];
      ctype = data[9];
      interlace = data[12];
      if (depth != 8 || interlace != 0 || (ctype != 0 && ctype != 2 && ctype != 4 && ctype != 6)) {
        err = std::string("unsupported PNG (8-bit non-interlaced gray/RGB(A) only): ") + path;
        return false;
      }
      out.ch = ctype == 0 ? 1 : ctype == 2 ? 3 : ctype == 4 ? 2 : 4;
      raw.resize((size_t)out.h * (1 + (size_t)out.w * out.ch));
      if (inflateInit(&zs) != Z_OK) {
        err = "inflateInit failed";
        return false;
      }
      zinit = true;
      zs.next_out = raw.data();
      zs.avail_out = (uInt)raw.size();
    } else if (!std::memcmp(type, "IDAT", 4)) {
      if (!zinit) {
        err = std::string("IDAT before IHDR in ") + path;
        return false;
      }
      zs.next_in = const_cast<unsigned char*>(data);
      zs.avail_in = len;
      const int rc = inflate(&zs, Z_NO_FLUSH);
      if (rc != Z_OK && rc != Z_STREAM_END && rc != Z_BUF_ERROR) {
        err = std::string("zlib error in ") + path;
        inflateEnd(&zs);
        return false;
      }
    } else if (!std::memcmp(type, "IEND", 4)) {
      done = true;
    }
    pos += 12 + (size_t)len;
  }
  if (zinit) inflateEnd(&zs);
  if (!zinit || !err.empty()) {
    if (err.empty()) err = std::string("no image data in ") + path;
    return false;
  }
  if (zs.total_out != raw.size()) {
    err = std::string("truncated image data in ") + path;
    return false;
  }
  // unfilter (PNG spec 9.2-9.4), bpp = channels for 8-bit samples
  const int bpp = out.ch;
  const size_t stride = (size_t)out.w * bpp;
  out.px.resize((size_t)out.h * stride);
  const unsigned char* prev = nullptr;
  for (int y = 0; y < out.h; ++y) {
    const unsigned char* in = &raw[(size_t)y * (stride + 1)];
    const int ft = in[0];
    ++in;
    unsigned char* row = &out.px[(size_t)y * stride];
    switch (ft) {
      case 0: std::memcpy(row, in, stride); break;
      case 1:
        for (size_t i = 0; i < stride; ++i) row[i] = (unsigned char)(in[i] + (i >= (size_t)bpp ? row[i - bpp] : 0));
        break;
      case 2:
        for (size_t i = 0; i < stride; ++i) row[i] = (unsigned char)(in[i] + (prev ? prev[i] : 0));
        break;
      case 3:
        for (size_t i = 0; i < stride; ++i) {
          const int a = i >= (size_t)bpp ? row[i - bpp] : 0, b = prev ? prev[i] : 0;
          row[i] = (unsigned char)(in[i] + ((a + b) >> 1));
        }
        break;
      case 4:
        for (size_t i = 0; i < stride; ++i) {
          const int a = i >= (size_t)bpp ? row[i - bpp] : 0, b = prev ? prev[i] : 0;
          const int c = (prev && i >= (size_t)bpp) ? prev[i - bpp] : 0;
          row[i] = (unsigned char)(in[i] + paeth(a, b, c));
        }
        break;
      default:
        err = std::string("bad PNG row filter in ") + path;
        return false;
    }
    prev = row;
  }
  return true;
}

// ImageTransformations' imresize (md2hip/data.py imresize): per output index the 0-based cell
// (i0, i1) and fraction at sf*(i - 1/2) + 1/2 (1-based), clamped to the image when upsampling
void imresize_axis(int n_in, int n_out, std::vector<int>& i0, std::vector<int>& i1,
                   std::vector<double>& f) {
  const double sf = (double)n_in / (double)n_out;
  i0.resize(n_out);
  i1.resize(n_out);
  f.resize(n_out);
  for (int i = 0; i < n_out; ++i) {
    double p = sf * ((double)(i + 1) - 0.5) + 0.5;
    if (sf < 1) p = std::min(std::max(p, 1.0), (double)n_in);
    p -= 1.0;
    const int a = std::min((int)std::floor(p), n_in - 1);
    i0[i] = a;
    f[i] = p - (double)a;
    i1[i] = std::min(a + 1, n_in - 1);
  }
}

// run fn(i) for i in [0, n) on up to `threads` host threads; first error wins
template <class F>
int parallel_for(int n, int threads, F fn) {
  threads = std::max(1, std::min(threads, n));
  std::atomic<int> next{0};
  std::atomic<int> failed{0};
  std::vector<std::string> errs(threads);
  auto work = [&](int t) {
    for (int i; (i = next.fetch_add(1)) < n && !failed.load();) {
      std::string e;
      bool ok;
      try {                            // nothing may escape a worker thread or the C ABI
        ok = fn(i, e);
      } catch (const std::exception& x) {
        e = std::string("loader: ") + x.what();
        ok = false;
      } catch (...) {
        e = "loader: unknown exception";
        ok = false;
      }
      if (!ok) {
        errs[t] = e;
        failed.store(1);
      }
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; ++t) pool.emplace_back(work, t);
  work(0);
  for (auto& th : pool) th.join();
  if (failed.load()) {
    for (auto& e : errs)
      if (!e.empty()) {
        set_error(e);
        break;
      }
    return MD2_EINVAL;
  }
  return MD2_OK;
}

}  // namespace
}  // namespace md2

using namespace md2;

extern "C" {

int md2_png_info(const char* path, int* width, int* height, int* channels) {
  MD2_CHECK_ARG(path && width && height && channels, "png_info args");
  std::vector<unsigned char> f;
  std::string err;
  if (!read_file(path, f, err)) {
    set_error(err);
    return MD2_EINVAL;
  }
  if (f.size() < 33 || std::memcmp(&f[12], "IHDR", 4) != 0) {
    set_error(std::string("not a PNG file: ") + path);
    return MD2_EINVAL;
  }
  *width = (int)be32(&f[16]);
  *height = (int)be32(&f[20]);
  const int ct = f[25];
  *channels = ct == 0 ? 1 : ct == 2 ? 3 : ct == 4 ? 2 : ct == 6 ? 4 : 0;
  return MD2_OK;
}

int md2_load_triplets_u8(const char* const* paths, int n, int width, int height,
                         const unsigned char* flip, unsigned char* out, int threads) {
  MD2_CHECK_ARG(paths && out && n >= 0 && width > 0 && height > 0, "load_triplets args");
  const size_t plane = (size_t)width * height, sample = 3 * 3 * plane;
  return parallel_for(n, threads, [&](int i, std::string& err) {
    Png p;
    if (!decode_png(paths[i], p, err, 3 * width, height)) return false;
    if (p.w != 3 * width || p.h != height || p.ch < 3) {
      err = std::string(paths[i]) + ": expected a " + std::to_string(3 * width) + "x" + std::to_string(height) +
            " RGB triplet, got " + std::to_string(p.w) + "x" + std::to_string(p.h) + "x" + std::to_string(p.ch);
      return false;
    }
    const bool fl = flip && flip[i];
    unsigned char* dst = out + (size_t)i * sample;
    for (int y = 0; y < height; ++y) {
      const unsigned char* row = &p.px[(size_t)y * p.w * p.ch];
      for (int j = 0; j < 3; ++j)
        for (int x = 0; x < width; ++x) {
          const unsigned char* s = row + ((size_t)j * width + (fl ? width - 1 - x : x)) * p.ch;
          unsigned char* d = dst + (size_t)j * 3 * plane + (size_t)y * width + x;
          d[0] = s[0];
          d[plane] = s[1];
          d[2 * plane] = s[2];
        }
    }
    return true;
  });
}

int md2_load_kitti_u8(const char* const* paths, int n, int height, int width,
                      const unsigned char* flip, unsigned char* out, int threads) {
  MD2_CHECK_ARG(paths && out && n >= 0 && width > 0 && height > 0, "load_kitti args");
  const size_t plane = (size_t)width * height;
  return parallel_for(3 * n, threads, [&](int k, std::string& err) {
    Png p;
    if (!decode_png(paths[k], p, err)) return false;
    if (p.ch != 1) {
      err = std::string(paths[k]) + ": KITTI image_0 frames are 8-bit grayscale";
      return false;
    }
    std::vector<int> y0, y1, x0, x1;
    std::vector<double> fy, fx;
    unsigned char* dst = out + (size_t)k * plane;   // [n][3][1][h][w]: frame k of the flat list
    const bool fl = flip && flip[k / 3];
    if (p.w == width && p.h == height) {
      for (int y = 0; y < height; ++y)
        for (int x = 0; x < width; ++x) dst[(size_t)y * width + x] = p.px[(size_t)y * width + (fl ? width - 1 - x : x)];
      return true;
    }
    imresize_axis(p.h, height, y0, y1, fy);
    imresize_axis(p.w, width, x0, x1, fx);
    const auto v = [&](int y, int x) { return (double)p.px[(size_t)y * p.w + x] / 255.0; };
    for (int y = 0; y < height; ++y)
      for (int xo = 0; xo < width; ++xo) {
        const int x = fl ? width - 1 - xo : xo;        // FlipX after the resize
        const double top = v(y0[y], x0[x]) * (1 - fx[x]) + v(y0[y], x1[x]) * fx[x];
        const double bot = v(y1[y], x0[x]) * (1 - fx[x]) + v(y1[y], x1[x]) * fx[x];
        const double r = top * (1 - fy[y]) + bot * fy[y];
        dst[(size_t)y * width + xo] = (unsigned char)std::nearbyint(r * 255.0);
      }
    return true;
  });
}

}  // extern "C"
