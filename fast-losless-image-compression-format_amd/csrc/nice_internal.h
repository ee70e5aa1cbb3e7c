// nice_internal.h -- host entry points shared between translation units of
// libnice_hip.so (not part of the C ABI in include/nice.h).
#pragma once
#include <stdint.h>

#include "../../include/nice.h"

namespace nice {

// nice_decode_batch_dev with the stream lengths optionally already on the host
// (h_stream_len non-null): no device round trip before the first launch.  The
// parse reaches its fixpoint on the device, so with host lengths the call only
// enqueues work.
int decode_batch_impl(nice_ctx* ctx, void* stream, const uint8_t* d_streams, uint64_t stream_stride,
                      const uint64_t* d_stream_len, const uint64_t* h_stream_len, uint32_t n_frames,
                      uint32_t w, uint32_t h, uint8_t out_channels, uint8_t* d_px, uint64_t px_stride,
                      uint32_t flags, int32_t* d_status);

}  // namespace nice
