/* asan_driver.c -- TEST INFRASTRUCTURE: host code under AddressSanitizer and
 * UndefinedBehaviorSanitizer.  Built by tests/test_asan.py with
 * gcc -fsanitize=address,undefined from oracle/nice_oracle.c and
 * csrc/nice_png.cpp; exercises the reference KATs, encode/decode of SYN-v1,
 * gradient, long-code, empty, 1-pixel and random frames in every decode mode,
 * decodes of truncated and bit-flipped streams, and the PNG scanline
 * unfilter on random rows of every filter type. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../oracle/nice_oracle.h"
#include "../include/nice.h"

static uint32_t rs = 12345u;
static uint32_t rnd(void) { rs ^= rs << 13; rs ^= rs >> 17; rs ^= rs << 5; return rs; }

static int roundtrip(const uint8_t *px, uint32_t w, uint32_t h, uint32_t c) {
    uint8_t *s = NULL; size_t n = 0;
    nice_oracle_stats st;
    memset(&st, 0, sizeof st);
    if (nice_oracle_encode(px, (size_t)w * h * c, w, h, (uint8_t)c, (uint8_t)c, &s, &n, &st)) return 1;
    int bad = 0;
    for (int mode = 0; mode < 3; ++mode) {
        uint8_t *o = NULL; size_t on = 0; uint32_t ow, oh; uint8_t oc;
        int rc = nice_oracle_decode(s, n, mode, &o, &on, &ow, &oh, &oc);
        /* W <= 3: back_ref W-1 (W = 1) or rel_ref W-3 (W = 3) is offset 0, a
         * pixel referencing itself (code.rs:141-145): no decoder can rebuild it */
        if (rc == 0 && mode >= 1 && w >= 4) {
            for (size_t i = 0; i < (size_t)w * h; ++i)
                if (memcmp(o + i * c, px + i * c, 3)) { fprintf(stderr, "mismatch mode %d %ux%ux%u px %zu\n", mode, w, h, c, i); bad = 1; break; }
        }
        nice_oracle_free(o);
    }
    /* truncated and corrupted streams must fail cleanly or decode something */
    for (int k = 0; k < 8 && n > 20; ++k) {
        size_t cut = 13 + rnd() % (n - 13);
        uint8_t *t = (uint8_t *)malloc(n);
        memcpy(t, s, n);
        t[13 + rnd() % (n - 13)] ^= (uint8_t)(1u << (rnd() & 7));
        for (int mode = 0; mode < 3; ++mode) {
            uint8_t *o = NULL; size_t on = 0; uint32_t ow, oh; uint8_t oc;
            (void)nice_oracle_decode(t, (k & 1) ? cut : n, mode, &o, &on, &ow, &oh, &oc);
            nice_oracle_free(o);
        }
        free(t);
    }
    nice_oracle_free(s);
    return bad;
}

int main(void) {
    int bad = 0;
    uint8_t kat[16];
    bad |= nice_oracle_kat_writer(kat, 16) < 1 || kat[0] != 0xFC;
    size_t hl; uint8_t mx;
    bad |= nice_oracle_kat_hfe(&hl, &mx) != 0;
    const uint32_t shapes[][3] = {{64, 48, 3}, {37, 23, 4}, {1, 50, 3}, {2, 30, 3}, {3, 20, 4}, {1, 1, 3},
                                  {256, 128, 4}, {5, 5, 3}};
    for (size_t k = 0; k < sizeof shapes / sizeof shapes[0]; ++k) {
        uint32_t w = shapes[k][0], h = shapes[k][1], c = shapes[k][2];
        uint8_t *px = (uint8_t *)malloc((size_t)w * h * c);
        nice_oracle_gen_syn_v1(px, w, h, c, 1 + (uint32_t)k);
        bad |= roundtrip(px, w, h, c);
        nice_oracle_gen_gradient(px, w, h, c);
        bad |= roundtrip(px, w, h, c);
        for (size_t i = 0; i < (size_t)w * h * c; ++i) px[i] = (uint8_t)rnd();
        bad |= roundtrip(px, w, h, c);
        free(px);
    }
    {   /* long codes (Fibonacci-skewed counts) */
        uint32_t w = 1536, h = 1024, c = 4;
        uint8_t *px = (uint8_t *)malloc((size_t)w * h * c);
        nice_oracle_gen_deep_codes(px, w, h, c, 1, 28);
        bad |= roundtrip(px, w, h, c);
        free(px);
    }
    {   /* empty image */
        uint8_t *s = NULL; size_t n = 0;
        bad |= nice_oracle_encode(NULL, 0, 0, 0, 4, 4, &s, &n, NULL) != 0;
        nice_oracle_free(s);
    }
    {   /* PNG unfilter, all five filter types, bpp 3 and 4 */
        for (uint32_t bpp = 3; bpp <= 4; ++bpp) {
            uint32_t w = 33, h = 10;
            uint8_t *raw = (uint8_t *)malloc((size_t)h * (w * bpp + 1));
            uint8_t *out = (uint8_t *)malloc((size_t)h * w * bpp);
            for (size_t i = 0; i < (size_t)h * (w * bpp + 1); ++i) raw[i] = (uint8_t)rnd();
            for (uint32_t y = 0; y < h; ++y) raw[y * (w * bpp + 1)] = (uint8_t)(y % 5);
            bad |= nice_png_unfilter(raw, w, h, bpp, out) != NICE_OK;
            raw[0] = 9;
            bad |= nice_png_unfilter(raw, w, h, bpp, out) != NICE_E_FORMAT;
            free(raw); free(out);
        }
    }
    printf(bad ? "FAIL\n" : "OK\n");
    return bad;
}
