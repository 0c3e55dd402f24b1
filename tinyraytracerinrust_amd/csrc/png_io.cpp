// png_io.cpp -- PNG decode (textures) and encode (frames) on top of zlib.
//
// Decode matches what the reference gets from lodepng::decode32_file (sceneparser/texture.rs:22):
// RGBA8 output for every colour type; 16-bit samples keep the high byte; sub-byte greys are
// scaled by 255/(2^bits-1); palette + tRNS alpha; grey/RGB tRNS colour keys; Adam7 supported;
// ancillary chunks (gAMA, sRGB, iCCP ...) are ignored -- no colour management, as lodepng.
// Encode is new plumbing (the reference has no PNG writer): 8-bit RGB/RGBA, filter 0, zlib.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include <string>
#include <vector>

#include "scene.h"

namespace rt {

bool read_file(const std::string& path, std::vector<uint8_t>* out) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return false;
  out->clear();
  uint8_t buf[1 << 16];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) out->insert(out->end(), buf, buf + n);
  fclose(f);
  return true;
}

static uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

static int paeth(int a, int b, int c) {
  int p = a + b - c, pa = p > a ? p - a : a - p, pb = p > b ? p - b : b - p, pc = p > c ? p - c : c - p;
  if (pa <= pb && pa <= pc) return a;
  return pb <= pc ? b : c;
}

// Unfilter one (sub)image of w x h in place; data = h rows of (1 + stride) bytes.
static bool unfilter(uint8_t* data, uint32_t h, size_t stride, size_t bpp, std::vector<uint8_t>* out) {
  out->assign((size_t)h * stride, 0);
  std::vector<uint8_t> zero(stride, 0);
  for (uint32_t y = 0; y < h; ++y) {
    const uint8_t* in = data + (size_t)y * (stride + 1);
    uint8_t ft = in[0];
    ++in;
    uint8_t* cur = out->data() + (size_t)y * stride;
    const uint8_t* prev = y ? out->data() + (size_t)(y - 1) * stride : zero.data();
    for (size_t i = 0; i < stride; ++i) {
      int a = i >= bpp ? cur[i - bpp] : 0, b = prev[i], c = i >= bpp ? prev[i - bpp] : 0;
      int v = in[i];
      switch (ft) {
        case 0: break;
        case 1: v += a; break;
        case 2: v += b; break;
        case 3: v += (a + b) >> 1; break;
        case 4: v += paeth(a, b, c); break;
        default: return false;
      }
      cur[i] = (uint8_t)v;
    }
  }
  return true;
}

int png_decode_rgba8(const std::vector<uint8_t>& f, std::vector<uint8_t>* rgba, uint32_t* W, uint32_t* H) {
  static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  if (f.size() < 33 || memcmp(f.data(), sig, 8) != 0) return fail(RT_ERR_IO, "not a PNG file");
  size_t p = 8;
  uint32_t w = 0, h = 0;
  int depth = 0, ctype = -1, interlace = 0;
  std::vector<uint8_t> idat, palette, trns;
  bool have_ihdr = false;
  while (p + 12 <= f.size()) {
    uint32_t len = be32(&f[p]);
    if (p + 12 + (size_t)len > f.size()) return fail(RT_ERR_IO, "truncated PNG chunk");
    const uint8_t* type = &f[p + 4];
    const uint8_t* d = &f[p + 8];
    if (!memcmp(type, "IHDR", 4)) {
      if (len < 13) return fail(RT_ERR_IO, "bad IHDR");
      w = be32(d); h = be32(d + 4); depth = d[8]; ctype = d[9]; interlace = d[12];
      if (d[10] != 0 || d[11] != 0) return fail(RT_ERR_IO, "unsupported PNG compression/filter method");
      have_ihdr = true;
    } else if (!memcmp(type, "PLTE", 4)) {
      palette.assign(d, d + len);
    } else if (!memcmp(type, "tRNS", 4)) {
      trns.assign(d, d + len);
    } else if (!memcmp(type, "IDAT", 4)) {
      idat.insert(idat.end(), d, d + len);
    } else if (!memcmp(type, "IEND", 4)) {
      break;
    }
    p += 12 + (size_t)len;
  }
  if (!have_ihdr || w == 0 || h == 0 || (uint64_t)w * h > (1ull << 28)) return fail(RT_ERR_IO, "bad PNG header");
  int channels;
  switch (ctype) {
    case 0: channels = 1; break;
    case 2: channels = 3; break;
    case 3: channels = 1; break;
    case 4: channels = 2; break;
    case 6: channels = 4; break;
    default: return fail(RT_ERR_IO, "bad PNG colour type %d", ctype);
  }
  bool depth_ok = depth == 8 || depth == 16 || ((ctype == 0 || ctype == 3) && (depth == 1 || depth == 2 || depth == 4));
  if (!depth_ok || (ctype == 3 && depth == 16)) return fail(RT_ERR_IO, "bad PNG bit depth %d", depth);
  if (ctype == 3 && palette.empty()) return fail(RT_ERR_IO, "palette PNG without PLTE");
  size_t bits_pp = (size_t)channels * depth;
  size_t bpp = (bits_pp + 7) / 8;

  // Adam7 passes (or one pass for non-interlaced images)
  static const int ax0[7] = {0, 4, 0, 2, 0, 1, 0}, ay0[7] = {0, 0, 4, 0, 2, 0, 1};
  static const int adx[7] = {8, 8, 4, 4, 2, 2, 1}, ady[7] = {8, 8, 8, 4, 4, 2, 2};
  int npass = interlace ? 7 : 1;
  size_t expect = 0;
  uint32_t pw[7], ph[7];
  for (int k = 0; k < npass; ++k) {
    pw[k] = interlace ? (w + adx[k] - 1 - ax0[k]) / adx[k] : w;
    ph[k] = interlace ? (h + ady[k] - 1 - ay0[k]) / ady[k] : h;
    if (w <= (uint32_t)ax0[k]) pw[k] = 0;
    if (h <= (uint32_t)ay0[k]) ph[k] = 0;
    if (pw[k] && ph[k]) expect += (size_t)ph[k] * (1 + (pw[k] * bits_pp + 7) / 8);
  }
  std::vector<uint8_t> raw(expect);
  z_stream zs;
  memset(&zs, 0, sizeof zs);
  if (inflateInit(&zs) != Z_OK) return fail(RT_ERR_IO, "zlib init failed");
  zs.next_in = idat.data();
  zs.avail_in = (uInt)idat.size();
  zs.next_out = raw.data();
  zs.avail_out = (uInt)raw.size();
  int zr = inflate(&zs, Z_FINISH);
  inflateEnd(&zs);
  if ((zr != Z_STREAM_END && zr != Z_OK && zr != Z_BUF_ERROR) || zs.total_out != expect)
    return fail(RT_ERR_IO, "PNG image data corrupt (zlib %d, %lu of %zu bytes)", zr, zs.total_out, expect);

  rgba->assign((size_t)w * h * 4, 0);
  size_t off = 0;
  for (int k = 0; k < npass; ++k) {
    if (!pw[k] || !ph[k]) continue;
    size_t stride = (pw[k] * bits_pp + 7) / 8;
    std::vector<uint8_t> img;
    if (!unfilter(raw.data() + off, ph[k], stride, bpp, &img)) return fail(RT_ERR_IO, "bad PNG filter");
    off += (size_t)ph[k] * (stride + 1);
    for (uint32_t y = 0; y < ph[k]; ++y) {
      const uint8_t* row = img.data() + (size_t)y * stride;
      for (uint32_t x = 0; x < pw[k]; ++x) {
        uint32_t X = interlace ? ax0[k] + x * adx[k] : x, Y = interlace ? ay0[k] + y * ady[k] : y;
        uint8_t* o = rgba->data() + ((size_t)Y * w + X) * 4;
        auto sample = [&](int ch) -> unsigned {   // raw sample value of channel ch
          if (depth == 8) return row[(size_t)x * channels + ch];
          if (depth == 16) return (unsigned)row[((size_t)x * channels + ch) * 2] << 8 | row[((size_t)x * channels + ch) * 2 + 1];
          size_t bit = (size_t)x * depth;
          return (row[bit / 8] >> (8 - depth - bit % 8)) & ((1u << depth) - 1);
        };
        auto to8 = [&](unsigned v) -> uint8_t {
          if (depth == 16) return (uint8_t)(v >> 8);
          if (depth == 8) return (uint8_t)v;
          return (uint8_t)(v * 255 / ((1u << depth) - 1));
        };
        switch (ctype) {
          case 0: {
            unsigned g = sample(0);
            o[0] = o[1] = o[2] = to8(g);
            o[3] = (trns.size() >= 2 && g == ((unsigned)trns[0] << 8 | trns[1])) ? 0 : 255;
            break;
          }
          case 2: {
            unsigned r = sample(0), g = sample(1), b = sample(2);
            o[0] = to8(r); o[1] = to8(g); o[2] = to8(b);
            o[3] = (trns.size() >= 6 && r == ((unsigned)trns[0] << 8 | trns[1]) &&
                    g == ((unsigned)trns[2] << 8 | trns[3]) && b == ((unsigned)trns[4] << 8 | trns[5])) ? 0 : 255;
            break;
          }
          case 3: {
            unsigned i = sample(0);
            if ((size_t)i * 3 + 2 >= palette.size()) return fail(RT_ERR_IO, "palette index out of range");
            o[0] = palette[i * 3]; o[1] = palette[i * 3 + 1]; o[2] = palette[i * 3 + 2];
            o[3] = i < trns.size() ? trns[i] : 255;
            break;
          }
          case 4:
            o[0] = o[1] = o[2] = to8(sample(0));
            o[3] = to8(sample(1));
            break;
          default:
            o[0] = to8(sample(0)); o[1] = to8(sample(1)); o[2] = to8(sample(2)); o[3] = to8(sample(3));
        }
      }
    }
  }
  *W = w;
  *H = h;
  return RT_OK;
}

static void put32(std::vector<uint8_t>* o, uint32_t v) {
  uint8_t b[4] = {(uint8_t)(v >> 24), (uint8_t)(v >> 16), (uint8_t)(v >> 8), (uint8_t)v};
  o->insert(o->end(), b, b + 4);
}
static void chunk(std::vector<uint8_t>* o, const char* type, const uint8_t* d, size_t n) {
  put32(o, (uint32_t)n);
  size_t start = o->size();
  o->insert(o->end(), type, type + 4);
  if (n) o->insert(o->end(), d, d + n);
  uLong crc = crc32(0L, o->data() + start, (uInt)(n + 4));
  put32(o, (uint32_t)crc);
}

int png_encode(const uint8_t* rgba8, uint32_t w, uint32_t h, size_t stride, int channels, std::vector<uint8_t>* out) {
  if (channels != 3 && channels != 4) return fail(RT_ERR_INVALID, "channels must be 3 or 4");
  std::vector<uint8_t> raw((size_t)h * (1 + (size_t)w * channels));
  for (uint32_t y = 0; y < h; ++y) {
    uint8_t* r = raw.data() + (size_t)y * (1 + (size_t)w * channels);
    r[0] = 0;
    const uint8_t* src = rgba8 + (size_t)y * stride;
    for (uint32_t x = 0; x < w; ++x)
      for (int c = 0; c < channels; ++c) r[1 + (size_t)x * channels + c] = src[(size_t)x * 4 + c];
  }
  uLongf zlen = compressBound((uLong)raw.size());
  std::vector<uint8_t> z(zlen);
  if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 6) != Z_OK) return fail(RT_ERR_NOMEM, "zlib compress failed");
  out->clear();
  static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  out->insert(out->end(), sig, sig + 8);
  uint8_t ihdr[13];
  for (int i = 0; i < 4; ++i) { ihdr[i] = (uint8_t)(w >> (24 - 8 * i)); ihdr[4 + i] = (uint8_t)(h >> (24 - 8 * i)); }
  ihdr[8] = 8; ihdr[9] = channels == 4 ? 6 : 2; ihdr[10] = ihdr[11] = ihdr[12] = 0;
  chunk(out, "IHDR", ihdr, 13);
  chunk(out, "IDAT", z.data(), zlen);
  chunk(out, "IEND", nullptr, 0);
  return RT_OK;
}

}  // namespace rt

using namespace rt;

extern "C" {

int rt_write_png(const char* path, const uint8_t* rgba8, uint32_t width, uint32_t height,
                 size_t row_stride_bytes, int channels) {
  if (!path || !rgba8 || !width || !height) return fail(RT_ERR_INVALID, "bad argument");
  if (row_stride_bytes < (size_t)width * 4) return fail(RT_ERR_INVALID, "row stride too small");
  std::vector<uint8_t> png;
  int rc = png_encode(rgba8, width, height, row_stride_bytes, channels, &png);
  if (rc) return rc;
  FILE* f = fopen(path, "wb");
  if (!f) return fail(RT_ERR_IO, "cannot open %s for writing", path);
  size_t n = fwrite(png.data(), 1, png.size(), f);
  fclose(f);
  return n == png.size() ? RT_OK : fail(RT_ERR_IO, "short write to %s", path);
}

int rt_read_png_rgba8(const char* path, uint8_t** pixels, uint32_t* width, uint32_t* height) {
  if (!path || !pixels || !width || !height) return fail(RT_ERR_INVALID, "bad argument");
  *pixels = nullptr;
  std::vector<uint8_t> file, rgba;
  if (!read_file(path, &file)) return fail(RT_ERR_IO, "cannot read %s", path);
  int rc = png_decode_rgba8(file, &rgba, width, height);
  if (rc) return rc;
  *pixels = (uint8_t*)malloc(rgba.size());
  if (!*pixels) return fail(RT_ERR_NOMEM, "out of memory");
  memcpy(*pixels, rgba.data(), rgba.size());
  return RT_OK;
}

void rt_free_buffer(void* p) { free(p); }

}  // extern "C"
