// Output formats on the far side of the hot path:
// Scotty3D's tonemap to 8-bit colour and PNG / PFM writers.
//
//   HDRImageBuffer::toColor   src/image.h:168-185   -> pt_tonemap
//   ImageBuffer::update_pixel src/image.h:49-58     -> 8-bit quantisation
//   PathTracer::save_image    src/pathtracer.cpp:577-591 (lodepng) -> pt_write_png
//
// The PNG writer emits stored (uncompressed) deflate blocks: no zlib needed,
// any PNG reader accepts them.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "pt_api.h"

namespace {

uint32_t crc_table[256];
bool crc_ready = false;

void crc_init() {
  for (uint32_t n = 0; n < 256; ++n) {
    uint32_t c = n;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    crc_table[n] = c;
  }
  crc_ready = true;
}

uint32_t crc32(const uint8_t* p, size_t n, uint32_t c = 0xFFFFFFFFu) {
  if (!crc_ready) crc_init();
  for (size_t i = 0; i < n; ++i) c = crc_table[(c ^ p[i]) & 0xFF] ^ (c >> 8);
  return c;
}

void put32(std::vector<uint8_t>& v, uint32_t x) {
  v.push_back((uint8_t)(x >> 24));
  v.push_back((uint8_t)(x >> 16));
  v.push_back((uint8_t)(x >> 8));
  v.push_back((uint8_t)x);
}

void chunk(std::vector<uint8_t>& out, const char* type, const std::vector<uint8_t>& data) {
  put32(out, (uint32_t)data.size());
  std::vector<uint8_t> td(type, type + 4);
  td.insert(td.end(), data.begin(), data.end());
  out.insert(out.end(), td.begin(), td.end());
  put32(out, crc32(td.data(), td.size()) ^ 0xFFFFFFFFu);
}

}  // namespace

extern "C" {

int pt_tonemap(const float* rgba, int32_t width, int32_t height, float gamma, float level, uint8_t* rgba8) {
  if (!rgba || !rgba8 || width <= 0 || height <= 0 || !(gamma > 0.0f)) return PT_E_INVALID;
  const float one_over_gamma = 1.0f / gamma;
  const float exposure = std::sqrt(std::pow(2.0f, level));
  auto q = [](float c) {  // clamp(0, 1, c) * 255, truncated (image.h:53-56)
    c = c < 0.0f ? 0.0f : (c > 1.0f ? 1.0f : c);
    return (uint8_t)(uint32_t)(c * 255);
  };
  for (size_t i = 0; i < (size_t)width * height; ++i) {
    const float* s = rgba + i * 4;
    rgba8[i * 4 + 0] = q(std::pow(s[0] * exposure, one_over_gamma));
    rgba8[i * 4 + 1] = q(std::pow(s[1] * exposure, one_over_gamma));
    rgba8[i * 4 + 2] = q(std::pow(s[2] * exposure, one_over_gamma));
    rgba8[i * 4 + 3] = 255;
  }
  return PT_OK;
}

int pt_write_png(const char* path, const uint8_t* rgba8, int32_t width, int32_t height) {
  if (!path || !rgba8 || width <= 0 || height <= 0) return PT_E_INVALID;
  // raw scanlines, top row first (the buffer's rows are bottom-up), filter 0
  const size_t row = (size_t)width * 4;
  std::vector<uint8_t> raw;
  raw.reserve((row + 1) * height);
  for (int32_t y = height - 1; y >= 0; --y) {
    raw.push_back(0);
    raw.insert(raw.end(), rgba8 + (size_t)y * row, rgba8 + (size_t)(y + 1) * row);
  }
  // zlib stream of stored deflate blocks
  std::vector<uint8_t> z = {0x78, 0x01};
  size_t pos = 0;
  do {
    const size_t n = std::min<size_t>(65535, raw.size() - pos);
    const bool last = pos + n == raw.size();
    z.push_back(last ? 1 : 0);
    z.push_back((uint8_t)n);
    z.push_back((uint8_t)(n >> 8));
    z.push_back((uint8_t)~n);
    z.push_back((uint8_t)(~n >> 8));
    z.insert(z.end(), raw.begin() + pos, raw.begin() + pos + n);
    pos += n;
  } while (pos < raw.size());
  uint32_t a = 1, b = 0;  // Adler-32
  for (uint8_t c : raw) {
    a = (a + c) % 65521u;
    b = (b + a) % 65521u;
  }
  put32(z, (b << 16) | a);

  std::vector<uint8_t> out = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
  std::vector<uint8_t> ihdr;
  put32(ihdr, (uint32_t)width);
  put32(ihdr, (uint32_t)height);
  ihdr.insert(ihdr.end(), {8, 6, 0, 0, 0});  // 8-bit RGBA, deflate, no filter set, no interlace
  chunk(out, "IHDR", ihdr);
  chunk(out, "IDAT", z);
  chunk(out, "IEND", {});
  FILE* f = fopen(path, "wb");
  if (!f) return PT_E_IO;
  const bool ok = fwrite(out.data(), 1, out.size(), f) == out.size();
  return (fclose(f) == 0 && ok) ? PT_OK : PT_E_IO;
}

int pt_write_pfm(const char* path, const float* rgba, int32_t width, int32_t height) {
  if (!path || !rgba || width <= 0 || height <= 0) return PT_E_INVALID;
  FILE* f = fopen(path, "wb");
  if (!f) return PT_E_IO;
  // PFM scanlines run bottom-to-top, like this ABI's frames; -1.0 = little endian
  fprintf(f, "PF\n%d %d\n-1.0\n", width, height);
  bool ok = true;
  for (size_t i = 0; i < (size_t)width * height && ok; ++i) ok = fwrite(rgba + i * 4, 4, 3, f) == 3;
  return (fclose(f) == 0 && ok) ? PT_OK : PT_E_IO;
}

}  // extern "C"
