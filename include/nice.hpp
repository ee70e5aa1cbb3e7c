// nice.hpp -- header-only C++ mirror of the reference codec API over nice.h.
//
//   nice::Image                 image.rs:5-43   (width, height, channels)
//   nice::encode(in, img, channels_out, out)   code.rs:59-64
//   nice::decode(in, channels_out, out) -> Image   code.rs:464-468
//
// Errors: the reference returns io::Error from its writer/reader and panics on
// malformed input; here every failure is a nice::Error carrying the nice.h
// status code.
#ifndef NICE_HPP
#define NICE_HPP
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "nice.h"

namespace nice {

struct Image {
  uint32_t width = 0, height = 0;
  uint8_t channels = 0;
  static Image make(uint32_t w, uint32_t h, uint8_t c) { return Image{w, h, c}; }
};

class Error : public std::runtime_error {
 public:
  Error(int code, const std::string& what)
      : std::runtime_error(what + " failed (status " + std::to_string(code) + ")"), code_(code) {}
  int code() const { return code_; }

 private:
  int code_;
};

inline void check(int rc, const char* what) {
  if (rc != NICE_OK) throw Error(rc, what);
}

// code::encode: appends the stream to `out`.
inline void encode(const std::vector<uint8_t>& in, const Image& img, uint8_t channels_out,
                   std::vector<uint8_t>& out) {
  const size_t base = out.size();
  out.resize(base + nice_encode_bound(img.width, img.height));
  size_t n = 0;
  int rc = nice_encode(in.data(), in.size(), img.width, img.height, img.channels, channels_out,
                       out.data() + base, out.size() - base, &n);
  if (rc != NICE_OK) out.resize(base);
  check(rc, "nice_encode");
  out.resize(base + n);
}

// code::decode: replaces `out` with the pixels (stride = header channels).
// channels_out is accepted and ignored, as in the reference (code.rs never reads it).
inline Image decode(const std::vector<uint8_t>& in, uint8_t /*channels_out*/,
                    std::vector<uint8_t>& out, uint32_t flags = NICE_DEC_ALPHA_FILL_FF) {
  Image img;
  check(nice_peek_header(in.data(), in.size(), &img.width, &img.height, &img.channels),
        "nice_peek_header");
  out.assign((size_t)img.width * img.height * img.channels, 0);
  size_t n = 0;
  check(nice_decode(in.data(), in.size(), out.data(), out.size(), flags, &n), "nice_decode");
  out.resize(n);
  return img;
}

// Owns a device context (scratch arena) for device-resident batches.
class Context {
 public:
  explicit Context(int device = 0) { check(nice_ctx_create(device, &ctx_), "nice_ctx_create"); }
  ~Context() { nice_ctx_destroy(ctx_); }
  Context(const Context&) = delete;
  Context& operator=(const Context&) = delete;
  nice_ctx* get() const { return ctx_; }

 private:
  nice_ctx* ctx_ = nullptr;
};

}  // namespace nice
#endif  // NICE_HPP
