// Encode a synthetic RGBA frame and decode it back through the C++ mirror
// (include/nice.hpp).  Build: make -C examples ; run: examples/roundtrip [w h]
#include <cstdio>
#include <cstdlib>

#include "nice.hpp"

int main(int argc, char** argv) {
  uint32_t w = argc > 2 ? atoi(argv[1]) : 640, h = argc > 2 ? atoi(argv[2]) : 480;
  std::vector<uint8_t> px((size_t)w * h * 4);
  uint32_t s = 1;
  for (uint32_t y = 0; y < h; ++y)
    for (uint32_t x = 0; x < w; ++x) {
      uint8_t* p = &px[((size_t)y * w + x) * 4];
      s ^= s << 13; s ^= s >> 17; s ^= s << 5;
      p[0] = (uint8_t)(x + (s & 3)); p[1] = (uint8_t)(y + ((s >> 2) & 3));
      p[2] = (uint8_t)((x + y) / 2); p[3] = 255;
    }
  try {
    std::vector<uint8_t> stream, back;
    nice::encode(px, nice::Image::make(w, h, 4), 4, stream);
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
