// Encode a synthetic RGBA frame and decode it back through the C++ mirror
// (include/nice.hpp).  Build: make -C examples ;
// run: examples/roundtrip [w h [stream_out_path]]
#include <cstdio>
#include <cstdlib>

#include "nice.hpp"

int main(int argc, char** argv) {
  uint32_t w = argc > 2 ? atoi(argv[1]) : 640, h = argc > 2 ? atoi(argv[2]) : 480;
  // NICE-SYN-v1 photo-like frame, seed 1
  std::vector<uint8_t> px((size_t)w * h * 4);
  static const int amp_tab[8] = {0, 1, 2, 3, 8, 24, 64, 256};
  uint32_t s = 1;
  for (uint32_t y = 0; y < h; ++y)
    for (uint32_t x = 0; x < w; ++x) {
      uint8_t* p = &px[((size_t)y * w + x) * 4];
      const int bx = w > 1 ? 200 * x / (w - 1) : 0, by = h > 1 ? 200 * y / (h - 1) : 0;
      const int base[3] = {bx, by, (bx + by) / 2};
      p[3] = 255;
      if (((x / 16) + (y / 16)) % 7 == 0) { p[0] = 40; p[1] = 80; p[2] = 120; continue; }
      const int amp = amp_tab[8 * y / h];
      for (int c = 0; c < 3; ++c) {
        s ^= s << 13; s ^= s >> 17; s ^= s << 5;
        const int n = amp == 0 ? 0 : amp < 256 ? (int)(s % amp) - amp / 2 : (int)(s & 255);
        p[c] = (uint8_t)((base[c] + n) & 255);
      }
    }
  try {
    std::vector<uint8_t> stream, back;
    nice::encode(px, nice::Image::make(w, h, 4), 4, stream);
    if (argc > 3) {
      FILE* fo = std::fopen(argv[3], "wb");
      if (!fo || std::fwrite(stream.data(), 1, stream.size(), fo) != stream.size()) return 3;
      std::fclose(fo);
    }
    nice::Image img = nice::decode(stream, 3, back);
    if (img.width != w || img.height != h || back != px) {
      std::printf("MISMATCH\n");
      return 1;
    }
    std::printf("ok %ux%u RGBA -> %zu bytes (%.3f bpp) -> identical\n", w, h, stream.size(),
                stream.size() * 8.0 / ((double)w * h));
  } catch (const nice::Error& e) {
    std::printf("error: %s\n", e.what());
    return 2;
  }
  return 0;
}
