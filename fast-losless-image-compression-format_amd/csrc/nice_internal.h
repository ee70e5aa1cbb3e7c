// nice_internal.h -- host entry points shared between translation units of
// libnice_hip.so (not part of the C ABI in include/nice.h).
#pragma once
#include <stdint.h>

#include "../../include/nice.h"

namespace nice {

// nice_decode_batch_dev with the stream lengths optionally already on the host
// (h_stream_len non-null): no device round trip before the first launch.
// h_unsettled (pinned host word, optional): the call does not wait for the
// queued sync iterations to reach their fixpoint; it enqueues everything and
// copies the last queued iteration's change flag there -- nonzero after the
// stream completes means the parse had not settled and the call must be
// repeated without it (the streamed pipeline checks when it reuses the slot).
int decode_batch_impl(nice_ctx* ctx, void* stream, const uint8_t* d_streams, uint64_t stream_stride,
                      const uint64_t* d_stream_len, const uint64_t* h_stream_len, uint32_t n_frames,
                      uint32_t w, uint32_t h, uint8_t out_channels, uint8_t* d_px, uint64_t px_stride,
                      uint32_t flags, int32_t* d_status, uint32_t* h_unsettled = nullptr);

}  // namespace nice
