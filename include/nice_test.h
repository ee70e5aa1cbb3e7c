/* nice_test.h -- test / A/B options of libnice_hip.so (NOT part of the codec API).
 *
 * The product reads no environment variables.  Tests and the diagnostic tools
 * force internal routes (slice size, row kernel, strip split, queued Jacobi
 * iterations, ...) through this process-wide table instead; every option is
 * off until set.  tests/conftest.py (`opts` fixture) and tools/phase_time.py
 * mirror the ids below.
 */
#ifndef NICE_TEST_H
#define NICE_TEST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum nice_test_opt {
  NICE_OPT_DEC_SLICE_BITS = 0,  /* parse slice size in bits (power of two in [1K, 16K]) */
  NICE_OPT_DEC_SINGLE_WAVE = 1, /* != 0: the one-wave row kernel (dec_reconstruct) */
  NICE_OPT_DEC_SEG = 2,         /* 8: dec_rows8 (8-pixel row segments) */
  NICE_OPT_DEC_SPLIT = 3,       /* strips of the split row kernel (0: never split) */
  NICE_OPT_DEC_FLOW = 4,        /* 0: no dataflow row kernel; k >= 1: k row groups */
  NICE_OPT_DEC_NO_EVENTS = 5,   /* != 0: do not keep the first pass's pixel events */
  NICE_OPT_DEC_EV_CAP = 6,      /* events kept per slice (forces overflow) */
  NICE_OPT_DEC_SLOW_PARSE = 7,  /* != 0: the general symbol-by-symbol parse only */
  NICE_OPT_DEC_STATS = 8,       /* != 0: print the decoder's statistics to stderr */
  NICE_OPT_DEC_SYNC_QUEUED = 9, /* queued Jacobi iterations before the settle (1..16) */
  NICE_OPT_DEC_REC_CLEAR = 10,  /* != 0: clear the record buffer on every call */
  NICE_OPT_ENC_NO_RING = 11,    /* != 0: the round-1 window classify kernel */
  NICE_OPT_ENC_NO_PAIR = 12,    /* != 0: no two-tile classify iterations */
  NICE_OPT_ENC_NO_SLIDE = 13,   /* != 0: no per-lane sliding-window classify */
  NICE_OPT_TEST_FLOW_ABSENT = 14, /* != 0: dec_rows_flow's last wave never starts (fallback test) */
  NICE_OPT_COUNT = 16
};

/* value < 0 unsets the option; returns 0, or NICE_E_ARG for an unknown id */
int nice_test_set_option(int id, int64_t value);
/* every option back to unset */
void nice_test_reset_options(void);

#ifdef __cplusplus
}
#endif
#endif /* NICE_TEST_H */
