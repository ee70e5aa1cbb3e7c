// nice_png.cpp -- host helper for the command-line front end (cli.py):
// reverses the five PNG scanline filters in place (ISO 15948 §9), the one
// part of PNG decoding that is a serial per-byte recurrence.  The reference
// CLI gets this from the png crate (main.rs:33-40); inflate is zlib's.
#include <stdint.h>
#include <stdlib.h>

#include "../../include/nice.h"

extern "C" int nice_png_unfilter(const uint8_t* raw, uint32_t w, uint32_t h, uint32_t bpp, uint8_t* out) {
  if (!raw || !out || bpp == 0 || bpp > 8) return NICE_E_ARG;
  const size_t stride = (size_t)w * bpp;
  const uint8_t* prev = nullptr;
  for (uint32_t y = 0; y < h; ++y) {
    const uint8_t ft = raw[y * (stride + 1)];
    const uint8_t* in = raw + y * (stride + 1) + 1;
    uint8_t* cur = out + y * stride;
    for (size_t x = 0; x < stride; ++x) {
      const int a = x >= bpp ? cur[x - bpp] : 0;
      const int b = prev ? prev[x] : 0;
      const int c = (prev && x >= bpp) ? prev[x - bpp] : 0;
      int pred;
      switch (ft) {
        case 0: pred = 0; break;
        case 1: pred = a; break;
        case 2: pred = b; break;
        case 3: pred = (a + b) >> 1; break;
        case 4: {
          const int p = a + b - c, pa = abs(p - a), pb = abs(p - b), pc = abs(p - c);
          pred = (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
          break;
        }
        default: return NICE_E_FORMAT;
      }
      cur[x] = (uint8_t)(in[x] + pred);
    }
    prev = cur;
  }
  return NICE_OK;
}
