/*
 * nice_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, single-threaded restatement of the reference NICE2 codec
 * (wouter-rombouts/fast-losless-image-compression-format, Rust, release profile)
 * used as the CHECKER for the MI355X HIP path and as the timed CPU baseline
 * ("kind": "port") in bench.py.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library.  The product library
 * (libnice_hip.so) never links, loads or calls it.
 *
 * Parity pinning: the reference is Rust and no Rust toolchain exists in this
 * image, so it cannot be built or run here.  This restatement is
 * pinned by (1) the reference's own known-answer tests (bitwriter.rs:86-97,
 * bitreader.rs:106-146, hfe.rs:300-348 round trip), ported in
 * tests/test_oracle_kat.py, and (2) byte sizes / max code lengths produced by a
 * second, independent restatement during the survey.
 * Full-stream byte parity against the Rust binary is therefore "unpinned" by
 * reference outputs; see DESIGN.md §Parity.
 *
 * Rust release semantics reproduced (Cargo.toml:12-16): wrapping +/- on
 * u8/u32/usize, shift amounts masked to the operand width, `u8::next_power_of_two`
 * wrapping to 0 above 128, `io::Read` on an exhausted slice returning Ok(0)
 * (stale buffer byte reused, bitreader.rs:90-96), std `BinaryHeap` push/pop
 * order (hfe.rs:63-84 with the reversed Ord of hfe.rs:246-251).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "nice_oracle.h"

/* ------------------------------------------------------------------------- */
/* Format constants: code.rs:16-45 (prefix ids, stream ids), code.rs:91-116   */
/* (alphabet sizes, in stream order).                                         */
/* ------------------------------------------------------------------------- */
enum {
    P_BACK_REF = 0, P_RGB = 1, P_LUMA = 2, P_SMALL_DIFF = 3, P_LUMA2 = 4, P_RUN1 = 5
};
enum {
    S_RGB = 0, S_PREFIX = 1, S_LUMA_BASE = 2, S_LUMA_OTHER = 3, S_LUMA_REF = 4,
    S_SMALL_DIFF = 5, S_LUMA2_BASE = 6, S_LUMA2_R = 7, S_LUMA2_B = 8, S_BACK_REF = 9,
    N_STREAMS = 10
};
static const int STREAM_N[N_STREAMS] = {256, 13, 64, 32, 11, 343, 64, 32, 32, 11};

/* ------------------------------------------------------------------------- */
/* Growable byte sink (stands in for the Vec<u8>/io::Write of main.rs:61).    */
/* ------------------------------------------------------------------------- */
typedef struct { uint8_t *p; size_t len, cap; int oom; } sink_t;

static void sink_put(sink_t *s, uint8_t b) {
    if (s->len == s->cap) {
        size_t nc = s->cap ? s->cap * 2 : 4096;
        uint8_t *np = (uint8_t *)realloc(s->p, nc);
        if (!np) { s->oom = 1; return; }
        s->p = np; s->cap = nc;
    }
    s->p[s->len++] = b;
}

/* ------------------------------------------------------------------------- */
/* Bitwriter: bitwriter.rs:3-73.  bit_offset is u8, cache is u32.             */
/* ------------------------------------------------------------------------- */
typedef struct { sink_t *w; uint8_t bit_offset; uint32_t cache; } bitwriter_t;

static inline uint32_t shl32(uint32_t v, unsigned s) { return v << (s & 31u); }
static inline uint32_t shr32(uint32_t v, unsigned s) { return v >> (s & 31u); }

/* bitwriter.rs:17-35 -- at most one byte flushed per call. */
static void bw_write_8bits(bitwriter_t *b, uint8_t amount, uint8_t value) {
    b->bit_offset = (uint8_t)(b->bit_offset + amount);
    b->cache += shl32((uint32_t)value, (uint8_t)(32 - b->bit_offset));
    if (b->bit_offset >= 8) {
        sink_put(b->w, (uint8_t)(b->cache >> 24));
        b->bit_offset = (uint8_t)(b->bit_offset - 8);
        b->cache <<= 8;
    }
}

/* bitwriter.rs:55-73 -- flushes while >= 8 bits are pending. */
static void bw_write_24bits(bitwriter_t *b, uint8_t amount, uint32_t value) {
    b->bit_offset = (uint8_t)(b->bit_offset + amount);
    b->cache += shl32(value, (uint8_t)(32 - b->bit_offset));
    while (b->bit_offset >= 8) {
        sink_put(b->w, (uint8_t)(b->cache >> 24));
        b->bit_offset = (uint8_t)(b->bit_offset - 8);
        b->cache <<= 8;
    }
}

/* ------------------------------------------------------------------------- */
/* Bitreader over a byte slice: bitreader.rs:3-100.                           */
/* ------------------------------------------------------------------------- */
typedef struct {
    const uint8_t *p; size_t len, pos;
    uint8_t bit_offset; uint32_t cache; uint8_t buffer;
    size_t stale;   /* bytes "read" past the end (stale buffer reuse) */
    int hung;       /* the reference refill loop would never terminate */
} bitreader_t;

static void br_init(bitreader_t *r, const uint8_t *p, size_t len, size_t pos) {
    r->p = p; r->len = len; r->pos = pos; r->bit_offset = 32; r->cache = 0; r->buffer = 0;
    r->stale = 0; r->hung = 0;
}

/* bitreader.rs:31-54: read_exact of one byte (EOF -> Err -> the caller's
 * unwrap panics), then extract. Returns -1 on EOF. */
static int br_read_bitsu8(bitreader_t *r, uint8_t amount, uint8_t *out) {
    if (amount > (uint8_t)(32 - r->bit_offset)) {
        if (r->pos >= r->len) return -1;
        uint8_t byte = r->p[r->pos++];
        r->cache = (uint32_t)byte + shl32(r->cache, 8);
        r->bit_offset = (uint8_t)(r->bit_offset - 8);
    }
    uint32_t ret = shr32(shl32(r->cache, r->bit_offset), (uint8_t)(32 - amount));
    if (ret > 255) return -2;               /* try_into::<u8>().unwrap() panics */
    r->bit_offset = (uint8_t)(r->bit_offset + amount);
    *out = (uint8_t)ret;
    return 0;
}

/* bitreader.rs:56-75 (test-only helper, ported for the KAT). */
static uint32_t br_read_24bits(bitreader_t *r, uint8_t amount) {
    uint8_t aob_rev = (uint8_t)(32 - amount);
    while (r->bit_offset > aob_rev) {
        if (r->pos < r->len) r->buffer = r->p[r->pos++];   /* read_exact().expect() */
        r->bit_offset = (uint8_t)(r->bit_offset - 8);
        r->cache = (uint32_t)r->buffer + shl32(r->cache, 8);
    }
    r->bit_offset = (uint8_t)(r->bit_offset + amount);
    return shr32(shl32(r->cache, (uint8_t)(r->bit_offset - amount)), aob_rev);
}

/* bitreader.rs:78-100: `Read::read` on an exhausted slice returns Ok(0) and
 * leaves `buffer` holding the previous byte, which is shifted in again. */
static uint32_t br_read_24bits_noclear(bitreader_t *r, uint8_t amount) {
    uint8_t aob_rev = (uint8_t)(32 - amount);
    while (r->bit_offset > aob_rev) {
        if (r->bit_offset < 8) {
            /* u8 `bit_offset -= 8` wraps (release build): the refill loop then
             * cycles through one residue class mod 8 and never terminates. */
            r->hung = 1;
            return 0;
        }
        if (r->pos < r->len) r->buffer = r->p[r->pos++];
        else r->stale++;
        r->bit_offset = (uint8_t)(r->bit_offset - 8);
        r->cache = shl32(r->cache, 8) + (uint32_t)r->buffer;
    }
    return shr32(shl32(r->cache, r->bit_offset), aob_rev);
}

/* ------------------------------------------------------------------------- */
/* Huffman code lengths: hfe.rs:58-87 with std BinaryHeap<TreeNode>.           */
/* TreeNode's Ord is reversed on occurrences_sum (hfe.rs:246-251), so the     */
/* max-heap behaves as a min-heap on counts.  Only counts are compared.        */
/* ------------------------------------------------------------------------- */
typedef struct { uint64_t cnt; int32_t node; } hn_t;

/* std BinaryHeap::sift_up(start, pos): move up while elem < parent in the
 * reversed order, i.e. while elem.cnt < parent.cnt. */
static size_t heap_sift_up(hn_t *d, size_t start, size_t pos) {
    hn_t e = d[pos];
    while (pos > start) {
        size_t parent = (pos - 1) / 2;
        if (d[parent].cnt <= e.cnt) break;            /* elem <= parent */
        d[pos] = d[parent];
        pos = parent;
    }
    d[pos] = e;
    return pos;
}

/* std BinaryHeap::sift_down_to_bottom(pos): walk to the bottom always taking
 * the "greater" child (right iff right.cnt <= left.cnt), then sift_up. */
static void heap_sift_down_to_bottom(hn_t *d, size_t len, size_t pos) {
    size_t end = len, start = pos;
    hn_t e = d[pos];
    size_t child = 2 * pos + 1;
    size_t lim = end >= 2 ? end - 2 : 0;
    while (child <= lim && end >= 2) {
        if (d[child + 1].cnt <= d[child].cnt) child += 1;
        d[pos] = d[child];
        pos = child;
        child = 2 * pos + 1;
    }
    if (child == end - 1) {
        d[pos] = d[child];
        pos = child;
    }
    d[pos] = e;
    heap_sift_up(d, start, pos);
}

static void heap_push(hn_t *d, size_t *len, hn_t x) {
    d[*len] = x;
    *len += 1;
    heap_sift_up(d, 0, *len - 1);
}

static hn_t heap_pop(hn_t *d, size_t *len) {
    *len -= 1;
    hn_t item = d[*len];
    if (*len > 0) {
        hn_t t = d[0]; d[0] = item; item = t;
        heap_sift_down_to_bottom(d, *len, 0);
    }
    return item;
}

/* Code lengths for one stream (hfe.rs:62-84).  aob starts at 1 and every merge
 * adds 1 (u8, wrapping) to each symbol under the merged node; the loop stops
 * with two nodes left.  We keep parent links instead of concatenated symbol
 * vectors: aob(sym) = 1 + (#merged ancestors of sym).  Exposed for tests. */
void nice_oracle_code_lengths(const uint64_t *counts, int n, uint8_t *aob) {
    hn_t *heap = (hn_t *)malloc(sizeof(hn_t) * (size_t)(n + 1));
    int32_t *parent = (int32_t *)malloc(sizeof(int32_t) * (size_t)(2 * n + 2));
    size_t len = 0;
    int next = n;
    for (int i = 0; i < 2 * n + 2; ++i) parent[i] = -1;
    for (int i = 0; i < n; ++i) {
        hn_t x = {counts[i], i};
        heap_push(heap, &len, x);
    }
    while (len > 2) {
        hn_t a = heap_pop(heap, &len);
        hn_t b = heap_pop(heap, &len);
        int id = next++;
        parent[a.node] = id;
        parent[b.node] = id;
        hn_t m = {a.cnt + b.cnt, id};
        heap_push(heap, &len, m);
    }
    for (int i = 0; i < n; ++i) {
        unsigned depth = 0;
        for (int p = parent[i]; p >= 0; p = parent[p]) depth++;
        aob[i] = (uint8_t)(1u + depth);
    }
    free(heap);
    free(parent);
}

/* amount_of_bits_to_bcodes: hfe.rs:255-296.  Sort by (aob desc, symbol desc),
 * walk with a usize running code.  Exposed for tests. */
typedef struct { int sym; uint8_t aob; } so_t;
static int so_cmp(const void *pa, const void *pb) {
    const so_t *a = (const so_t *)pa, *b = (const so_t *)pb;
    if (a->aob != b->aob) return a->aob > b->aob ? -1 : 1;
    return a->sym > b->sym ? -1 : (a->sym < b->sym ? 1 : 0);
}
void nice_oracle_canonical(const uint8_t *aob, int n, uint64_t *code) {
    so_t *s = (so_t *)malloc(sizeof(so_t) * (size_t)n);
    for (int i = 0; i < n; ++i) { s[i].sym = i; s[i].aob = aob[i]; }
    qsort(s, (size_t)n, sizeof(so_t), so_cmp);
    uint64_t cur = 0;
    uint8_t prev = 0;
    for (int k = 0; k < n; ++k) {
        uint8_t a = s[k].aob;
        if (a < prev) cur >>= ((uint8_t)(prev - a)) & 63u;
        if (prev > 0) cur += 1;
        code[s[k].sym] = (((uint64_t)1) << (a & 63u)) - cur - 1;
        prev = a;
    }
    free(s);
}

/* u8::next_power_of_two().count_zeros() in release mode (hfe.rs:102,178). */
static uint8_t field_bits(uint8_t max_aob) {
    unsigned np;
    if (max_aob <= 1) np = 1;
    else if (max_aob > 128) np = 0;               /* wraps to 0 */
    else { np = 1; while (np < max_aob) np <<= 1; }
    unsigned pop = 0;
    for (unsigned b = np; b; b >>= 1) pop += b & 1u;
    return (uint8_t)(8 - pop);
}

/* ------------------------------------------------------------------------- */
/* Encoder: code.rs:59-457 + hfe.rs:29-117.                                    */
/* ------------------------------------------------------------------------- */
typedef struct { uint16_t sym; uint8_t stream; } symrec_t;
typedef struct {
    symrec_t *v; size_t len, cap; int oom;
    uint64_t *occ[N_STREAMS];
} encout_t;

static void add_symbol(encout_t *e, unsigned sym, int stream) {
    if (e->len == e->cap) {
        size_t nc = e->cap ? e->cap * 2 : 4096;
        symrec_t *np = (symrec_t *)realloc(e->v, nc * sizeof(symrec_t));
        if (!np) { e->oom = 1; return; }
        e->v = np; e->cap = nc;
    }
    e->v[e->len].sym = (uint16_t)sym;
    e->v[e->len].stream = (uint8_t)stream;
    e->len++;
    e->occ[stream][sym] += 1;
}

/* Pixel RGB at byte position pos (channels bytes per pixel; only +0..+2 read). */
static inline int rgb_eq(const uint8_t *in, size_t a, size_t b) {
    return in[a] == in[b] && in[a + 1] == in[b + 1] && in[a + 2] == in[b + 2];
}

/* px_bit (optional, W*H + 1 entries): the absolute stream bit of each coded
 * pixel's first symbol, UINT64_MAX for run members, then the data end bit
 * (test data for the band exchange rehearsal: a band's bits start at its
 * first coded pixel's). */
static int encode_impl(const uint8_t *in, size_t in_len, uint32_t width, uint32_t height,
                       uint8_t channels, uint8_t channels_out,
                       uint8_t **out, size_t *out_len, nice_oracle_stats *stats, uint64_t *px_bit) {
    *out = NULL; *out_len = 0;
    if (channels < 3) return NICE_ORACLE_E_ARG;
    const size_t W = width, ch = channels;
    const size_t image_size = (size_t)height * W * ch;                 /* code.rs:85 */
    if (in_len < image_size) return NICE_ORACLE_E_ARG;
    sink_t sink = {0};
    /* header: code.rs:72-84 */
    sink_put(&sink, 'n'); sink_put(&sink, 'i'); sink_put(&sink, 'c'); sink_put(&sink, 'e');
    for (int s = 24; s >= 0; s -= 8) sink_put(&sink, (uint8_t)(width >> s));
    for (int s = 24; s >= 0; s -= 8) sink_put(&sink, (uint8_t)(height >> s));
    sink_put(&sink, channels_out);

    encout_t e = {0};
    for (int s = 0; s < N_STREAMS; ++s) e.occ[s] = (uint64_t *)calloc((size_t)STREAM_N[s], 8);

    /* ref tables: code.rs:141-145 (usize wrapping arithmetic) */
    const size_t rel_ref[11] = {ch, ch * W, ch * (W - 1), ch * (W - 3), 3 * ch,
                                ch * (3 * W - 1), 3 * ch * W, ch * (3 * W + 1), ch * (W + 3),
                                ch * 3 * (W + 1), ch * 3 * (W - 1)};
    const size_t back_ref[5] = {ch, ch * W, ch * (W - 1), 2 * ch, 2 * ch * W};
    const size_t rowb = ch * W;

    size_t position = 0, prev_position = 0;
    uint64_t n_coded = 0, n_br = 0, n_sd = 0, n_l2 = 0, n_luma = 0, n_rgb = 0, n_runpx = 0;
    uint64_t *cp_sym = NULL;   /* px_bit: first symbol index of each coded pixel (by pixel) */
    if (px_bit) {
        cp_sym = (uint64_t *)malloc(8 * ((size_t)height * W + 1));
        for (size_t i = 0; i < (size_t)height * W; ++i) { cp_sym[i] = UINT64_MAX; px_bit[i] = UINT64_MAX; }
        cp_sym[(size_t)height * W] = UINT64_MAX;
    }
    while (position < image_size) {                                      /* code.rs:159 */
        if (cp_sym) cp_sym[position / ch] = e.len;
        n_coded++;
        int done = 0;
        /* back references: code.rs:191-206 */
        for (int k = 0; k < 5 && !done; ++k) {
            if (position >= back_ref[k]) {
                size_t rp = position - back_ref[k];
                if (rgb_eq(in, position, rp)) {
                    add_symbol(&e, P_BACK_REF, S_PREFIX);
                    add_symbol(&e, (unsigned)k, S_BACK_REF);
                    done = 1; n_br++;
                }
            }
        }
        if (!done) {
            /* small diff: code.rs:208-247 (i16 arithmetic) */
            int d[3];
            for (int c = 0; c < 3; ++c)
                d[c] = (int)in[position + c] - (int)in[prev_position + c];
            if (position >= rowb) {
                for (int c = 0; c < 3; ++c)
                    d[c] = (int)in[position + c] -
                           ((int)in[position - rowb + c] + (int)in[prev_position + c]) / 2;
            }
            if (position > 0 && d[0] >= -3 && d[0] <= 3 && d[1] >= -3 && d[1] <= 3 &&
                d[2] >= -3 && d[2] <= 3) {
                add_symbol(&e, P_SMALL_DIFF, S_PREFIX);
                unsigned code = (unsigned)(3 + d[0]) + 7u * (unsigned)(3 + d[1]) +
                                49u * (unsigned)(3 + d[2]);
                add_symbol(&e, code, S_SMALL_DIFF);
                done = 1; n_sd++;
            }
        }
        if (!done && position >= rowb) {
            /* luma2: code.rs:252-292 (u8 wrapping arithmetic) */
            size_t rp = position - rowb;
            uint8_t a[3];
            for (int c = 0; c < 3; ++c)
                a[c] = (uint8_t)(((unsigned)in[rp + c] + (unsigned)in[prev_position + c]) / 2);
            uint8_t g = (uint8_t)(in[position + 1] - a[1]);
            uint8_t r = (uint8_t)((uint8_t)(in[position] - a[0]) - g);
            uint8_t b = (uint8_t)((uint8_t)(in[position + 2] - a[2]) - g);
            if (position > 0 && (g >= 224 || g < 32) && (r >= 240 || r < 16) &&
                (b >= 240 || b < 16)) {
                add_symbol(&e, P_LUMA2, S_PREFIX);
                add_symbol(&e, (uint8_t)(g + 32), S_LUMA2_BASE);
                add_symbol(&e, (uint8_t)(r + 16), S_LUMA2_R);
                add_symbol(&e, (uint8_t)(b + 16), S_LUMA2_B);
                done = 1; n_l2++;
            }
        }
        if (!done) {
            /* luma with relative refs: code.rs:293-339 */
            for (int k = 0; k < 11 && !done; ++k) {
                if (position >= rel_ref[k]) {
                    size_t rp = position - rel_ref[k];
                    uint8_t g = (uint8_t)(in[position + 1] - in[rp + 1]);
                    uint8_t r = (uint8_t)((uint8_t)(in[position] - in[rp]) - g);
                    uint8_t b = (uint8_t)((uint8_t)(in[position + 2] - in[rp + 2]) - g);
                    if (position > 0 && (g >= 224 || g < 32) && (r >= 240 || r < 16) &&
                        (b >= 240 || b < 16)) {
                        add_symbol(&e, P_LUMA, S_PREFIX);
                        add_symbol(&e, (unsigned)k, S_LUMA_REF);
                        add_symbol(&e, (uint8_t)(g + 32), S_LUMA_BASE);
                        add_symbol(&e, (uint8_t)(r + 16), S_LUMA_OTHER);
                        add_symbol(&e, (uint8_t)(b + 16), S_LUMA_OTHER);
                        done = 1; n_luma++;
                    }
                }
            }
        }
        if (!done) {
            /* rgb: code.rs:341-366 */
            add_symbol(&e, P_RGB, S_PREFIX);
            for (int c = 0; c < 3; ++c) {
                uint8_t v = (uint8_t)(in[position + c] - (position > 0 ? in[prev_position + c] : 0));
                if (position >= rowb)
                    v = (uint8_t)((int)in[position + c] -
                                  ((int)in[position - rowb + c] + (int)in[prev_position + c]) / 2);
                add_symbol(&e, v, S_RGB);
            }
            n_rgb++;
        }
        /* run: code.rs:371-407 */
        size_t run_length = 0, rlp = position + ch;
        while (rlp < image_size && rgb_eq(in, rlp, position)) { run_length++; rlp += ch; }
        if (run_length > 0) {
            n_runpx += run_length;
            position += run_length * ch;
            run_length -= 1;
            for (;;) {
                add_symbol(&e, (unsigned)(run_length % 8 + 5), S_PREFIX);
                if (run_length < 8) break;
                run_length /= 8;
            }
        }
        prev_position = position;                                           /* code.rs:412 */
        position += ch;
    }

    /* to_encoded_output: hfe.rs:51-117 */
    bitwriter_t bw = {&sink, 0, 0};
    uint8_t *aob[N_STREAMS];
    uint64_t *code[N_STREAMS];
    for (int s = 0; s < N_STREAMS; ++s) {
        int n = STREAM_N[s];
        aob[s] = (uint8_t *)malloc((size_t)n);
        code[s] = (uint64_t *)malloc(8 * (size_t)n);
        nice_oracle_code_lengths(e.occ[s], n, aob[s]);
        nice_oracle_canonical(aob[s], n, code[s]);
        uint8_t mx = 0;
        for (int i = 0; i < n; ++i) if (aob[s][i] > mx) mx = aob[s][i];
        if (stats) stats->max_aob[s] = mx;
        bw_write_8bits(&bw, 5, mx);                                     /* hfe.rs:98 */
        uint8_t fb = field_bits(mx);
        for (int i = 0; i < n; ++i) bw_write_8bits(&bw, fb, aob[s][i]); /* hfe.rs:100-103 */
    }
    size_t header_bytes = sink.len;
    uint8_t max_emit = 0;
    uint64_t n_long = 0, n_wrapped = 0;
    size_t cpi = 0;   /* px_bit: next coded pixel */
    for (size_t k = 0; k < e.len; ++k) {                                /* hfe.rs:110-113 */
        int s = e.v[k].stream, sym = e.v[k].sym;
        if (cp_sym) {
            while (cpi < (size_t)height * W && (cp_sym[cpi] == UINT64_MAX || cp_sym[cpi] < k)) ++cpi;
            if (cpi < (size_t)height * W && cp_sym[cpi] == k) px_bit[cpi] = 8ull * sink.len + bw.bit_offset;
        }
        if (aob[s][sym] > max_emit) max_emit = aob[s][sym];
        /* diagnostics: codes over 25 bits, and writes whose u8 `32 - bit_offset`
         * wraps (bitwriter.rs:63-64: pending + length > 32 mangles the cache) */
        n_long += aob[s][sym] > 25;
        n_wrapped += (unsigned)bw.bit_offset + aob[s][sym] > 32u;
        bw_write_24bits(&bw, aob[s][sym], (uint32_t)code[s][sym]);
    }
    if (px_bit) px_bit[(size_t)height * W] = 8ull * sink.len + bw.bit_offset;   /* the data end */
    sink_put(&sink, (uint8_t)(bw.cache >> 24));                           /* hfe.rs:115 */
    for (int s = 24; s >= 0; s -= 8) sink_put(&sink, (uint8_t)(bw.cache >> s)); /* code.rs:421-422 */

    if (stats) {
        stats->n_symbols = e.len;
        stats->n_coded = n_coded; stats->n_backref = n_br; stats->n_smalldiff = n_sd;
        stats->n_luma2 = n_l2; stats->n_luma = n_luma; stats->n_rgb = n_rgb;
        stats->n_run_pixels = n_runpx;
        stats->header_end = header_bytes;
        stats->max_emitted_aob = max_emit;
        stats->n_long_emits = n_long;
        stats->n_wrapped_emits = n_wrapped;
        int bin = 0;
        for (int s = 0; s < N_STREAMS; ++s)
            for (int i = 0; i < STREAM_N[s]; ++i, ++bin) {
                stats->hist[bin] = e.occ[s][i];
                stats->aob[bin] = aob[s][i];
                stats->hist_total += e.occ[s][i];
            }
    }
    int oom = sink.oom || e.oom;
    free(cp_sym);
    for (int s = 0; s < N_STREAMS; ++s) { free(aob[s]); free(code[s]); free(e.occ[s]); }
    free(e.v);
    if (oom) { free(sink.p); return NICE_ORACLE_E_OOM; }
    *out = sink.p;
    *out_len = sink.len;
    return 0;
}

int nice_oracle_encode(const uint8_t *in, size_t in_len, uint32_t width, uint32_t height,
                       uint8_t channels, uint8_t channels_out,
                       uint8_t **out, size_t *out_len, nice_oracle_stats *stats) {
    return encode_impl(in, in_len, width, height, channels, channels_out, out, out_len, stats, NULL);
}

int nice_oracle_encode_bitpos(const uint8_t *in, size_t in_len, uint32_t width, uint32_t height,
                              uint8_t channels, uint8_t **out, size_t *out_len, uint64_t *px_bit) {
    return encode_impl(in, in_len, width, height, channels, channels, out, out_len, NULL, px_bit);
}

/* ------------------------------------------------------------------------- */
/* Decoder: code.rs:464-687 + hfe.rs:173-222.                                  */
/* mode NICE_ORACLE_DEC_REFERENCE follows the reference literally: pixel       */
/* stride 3 after coded pixels (code.rs:659) and `channels` elsewhere; every   */
/* Rust panic (index out of bounds, read_exact EOF, over-long shift in the LUT */
/* fill) becomes an error code.  NICE_ORACLE_DEC_STRIDE uses `channels` as the */
/* stride everywhere (the evident intent), used only to check RGBA round trips.*/
/* ------------------------------------------------------------------------- */
typedef struct { uint16_t symbol; uint8_t aob; } lut_t;
#ifndef LUT_LAZY_BITS
#define LUT_LAZY_BITS 20
#endif
typedef struct {
    uint8_t max_aob; lut_t *lut; size_t lut_len;
    /* tables over LUT_LAZY_BITS: the 2^max LUT (hfe.rs:191-202) as its code
     * intervals, lower bounds descending (the domain check makes the code
     * complete and non-overlapping, so every window value falls in exactly
     * the interval whose LUT range holds it: same symbol and length) */
    int nlazy; uint64_t *zlo; uint16_t *zsym; uint8_t *zlen;
    /* tolerant tables (canonical order, decodable entries only) */
    int ncanon; uint32_t *clo; uint16_t *csym; uint8_t *clen;
} sslookup_t;

static int read_header_into_tree(bitreader_t *r, sslookup_t *sl, int n) {
    uint8_t mx;
    if (br_read_bitsu8(r, 5, &mx)) return NICE_ORACLE_E_PANIC;
    sl->max_aob = mx;
    uint8_t fb = field_bits(mx);
    uint8_t *a = (uint8_t *)malloc((size_t)n);
    uint64_t *code = (uint64_t *)malloc(8 * (size_t)n);
    for (int i = 0; i < n; ++i) {
        if (br_read_bitsu8(r, fb, &a[i])) { free(a); free(code); return NICE_ORACLE_E_PANIC; }
    }
    /* Domain check (DESIGN.md "decode domain"): a complete canonical code whose
     * longest length equals the 5-bit max.  Every stream the reference encoder
     * writes without a header spill satisfies it; outside it the reference fills
     * a 2^max table with overlapping/missing entries (and may allocate GiBs). */
    {
        uint64_t kraft = 0; uint8_t seen = 0; int ok = mx >= 1 && mx <= 31;
        for (int i = 0; i < n && ok; ++i) {
            if (a[i] < 1 || a[i] > mx) ok = 0;
            else { kraft += (uint64_t)1 << (mx - a[i]); if (a[i] > seen) seen = a[i]; }
        }
        if (!ok || seen != mx || kraft != ((uint64_t)1 << mx)) {
            free(a); free(code);
            return NICE_ORACLE_E_DOMAIN;
        }
    }
    nice_oracle_canonical(a, n, code);
    sl->lut_len = (size_t)1 << (mx & 63u);
    if (mx > LUT_LAZY_BITS) {
        sl->zlo = (uint64_t *)malloc(8 * (size_t)n);
        sl->zsym = (uint16_t *)malloc(2 * (size_t)n);
        sl->zlen = (uint8_t *)malloc((size_t)n);
        sl->nlazy = 0;
        for (int i = 0; i < n; ++i) {             /* insertion by lower bound, descending */
            uint64_t lo = code[i] << ((uint8_t)(mx - a[i]) & 63u);
            int k = sl->nlazy++;
            while (k > 0 && sl->zlo[k - 1] < lo) {
                sl->zlo[k] = sl->zlo[k - 1]; sl->zsym[k] = sl->zsym[k - 1]; sl->zlen[k] = sl->zlen[k - 1];
                --k;
            }
            sl->zlo[k] = lo; sl->zsym[k] = (uint16_t)i; sl->zlen[k] = a[i];
        }
        free(a); free(code);
        return 0;
    }
    sl->lut = (lut_t *)calloc(sl->lut_len, sizeof(lut_t));
    int rc = 0;
    for (int i = 0; i < n && !rc; ++i) {
        unsigned sh = ((uint8_t)(mx - a[i])) & 63u;
        uint64_t lo = code[i] << sh, hi = (code[i] + 1) << sh;
        for (uint64_t k = lo; k < hi; ++k) {
            if (k >= sl->lut_len) { rc = NICE_ORACLE_E_PANIC; break; }
            sl->lut[k].symbol = (uint16_t)i;
            sl->lut[k].aob = a[i];
        }
    }
    free(a); free(code);
    return rc;
}

/* Tolerant tables (NICE_ORACLE_DEC_TOLERANT).  The
 * writer puts each stream's max length into a 5-bit field with
 * `cache += v << (32 - k)` (hfe.rs:97-99, bitwriter.rs:17-35): a max above 31
 * keeps its low 5 bits in the field and ADDS `max >> 5` into the bits before it
 * that are still pending in the u32 cache: the low p bits of the previous
 * stream's last 7-bit length, p = (bits written so far) mod 8 (write_8bits
 * flushes one byte per call, so at most 7 bits are pending); carries out of
 * them fall off the top of the cache, as does all of stream 0's spill.
 * Repair, from the last stream down: the true max of stream t is the max of its
 * 7-bit lengths (its own last entry already repaired); it must agree with the
 * field mod 32; if it is >= 32, subtract the spill from those p bits mod 2^p.  Each stream must then
 * be a complete prefix code (Kraft sum exactly 1, 128-bit exact).  Codes follow
 * amount_of_bits_to_bcodes (hfe.rs:255-296) with usize wrapping; only lengths
 * <= 31 are decodable (longer ones are the zero-count symbols the Huffman
 * merge pushes deep), and the decodable codes must not overlap. */
static int tolerant_tables(bitreader_t *r, sslookup_t *L) {
    uint8_t field[N_STREAMS];
    uint8_t *a[N_STREAMS];
    int rc = 0;
    for (int t = 0; t < N_STREAMS; ++t) a[t] = NULL;
    for (int t = 0; t < N_STREAMS && !rc; ++t) {
        if (br_read_bitsu8(r, 5, &field[t])) { rc = NICE_ORACLE_E_PANIC; break; }
        uint8_t fb = field_bits(field[t]);            /* 7 for every 5-bit value */
        a[t] = (uint8_t *)malloc((size_t)STREAM_N[t]);
        for (int i = 0; i < STREAM_N[t]; ++i)
            if (br_read_bitsu8(r, fb, &a[t][i])) { rc = NICE_ORACLE_E_PANIC; break; }
    }
    for (int t = N_STREAMS - 1; t >= 0 && !rc; --t) {
        unsigned mx = 0;
        for (int i = 0; i < STREAM_N[t]; ++i) if (a[t][i] > mx) mx = a[t][i];
        if ((mx & 31u) != field[t] || mx > 127) { rc = NICE_ORACLE_E_DOMAIN; break; }
        if (mx >= 32 && t > 0) {
            /* the spill lands in the p bits still pending in the writer's cache
             * (the low p bits of the previous field, p = bits written mod 8);
             * carries out of them leave the u32 cache */
            unsigned bits = 0;
            for (int q = 0; q < t; ++q) bits += 5u + 7u * (unsigned)STREAM_N[q];
            const unsigned p = bits & 7u, m = (1u << p) - 1u;
            uint8_t *last = &a[t - 1][STREAM_N[t - 1] - 1];
            *last = (uint8_t)((*last & ~m) | ((*last - (mx >> 5)) & m));
        }
    }
    for (int t = 0; t < N_STREAMS && !rc; ++t) {
        const int n = STREAM_N[t];
        unsigned mx = 0, dm = 0;
        unsigned __int128 kraft = 0;
        for (int i = 0; i < n; ++i) {
            if (a[t][i] < 1) { rc = NICE_ORACLE_E_DOMAIN; break; }
            if (a[t][i] > mx) mx = a[t][i];
            if (a[t][i] <= 31 && a[t][i] > dm) dm = a[t][i];
        }
        if (rc) break;
        for (int i = 0; i < n; ++i) kraft += (unsigned __int128)1 << (mx - a[t][i]);
        if (kraft != ((unsigned __int128)1 << mx) || dm == 0) { rc = NICE_ORACLE_E_DOMAIN; break; }
        uint64_t *code = (uint64_t *)malloc(8 * (size_t)n);
        nice_oracle_canonical(a[t], n, code);
        sslookup_t *sl = &L[t];
        sl->max_aob = (uint8_t)dm;
        sl->clo = (uint32_t *)malloc(4 * (size_t)n);
        sl->csym = (uint16_t *)malloc(2 * (size_t)n);
        sl->clen = (uint8_t *)malloc((size_t)n);
        sl->ncanon = 0;
        /* decodable entries in canonical order: (length desc, symbol desc) */
        for (unsigned l = dm; l >= 1; --l)
            for (int i = n - 1; i >= 0; --i)
                if (a[t][i] == l) {
                    if (code[i] >> l) { rc = NICE_ORACLE_E_DOMAIN; break; }
                    int k = sl->ncanon++;
                    sl->clo[k] = (uint32_t)(code[i] << (dm - l));
                    sl->csym[k] = (uint16_t)i;
                    sl->clen[k] = (uint8_t)l;
                    /* intervals [lo, lo + 2^(dm-l)) descend without overlap */
                    if (k > 0 && (uint64_t)sl->clo[k] + ((uint64_t)1 << (dm - l)) > sl->clo[k - 1])
                        rc = NICE_ORACLE_E_DOMAIN;
                }
        free(code);
    }
    for (int t = 0; t < N_STREAMS; ++t) free(a[t]);
    return rc;
}

static int canon_lookup(const sslookup_t *sl, uint32_t v, unsigned *sym, uint8_t *len) {
    for (int k = sl->ncanon - 1; k >= 0; --k) {           /* shortest (lowest) codes first */
        uint64_t span = (uint64_t)1 << (sl->max_aob - sl->clen[k]);
        if (v >= sl->clo[k] && v < sl->clo[k] + span) { *sym = sl->csym[k]; *len = sl->clen[k]; return 0; }
    }
    return NICE_ORACLE_E_PANIC;                             /* bits match no decodable code */
}

/* Absolute-position reader with the same byte semantics (bytes past the end
 * read as the last stream byte) but no u32 cache: what the reference reader
 * computes whenever it terminates.  Used by NICE_ORACLE_DEC_STRIDE ("intent"). */
static uint32_t abs_peek(const uint8_t *p, size_t len, uint64_t bitpos, unsigned m) {
    uint64_t acc = 0;
    size_t b = (size_t)(bitpos >> 3);
    for (int k = 0; k < 8; ++k) {
        size_t i = b + (size_t)k;
        uint8_t v = i < len ? p[i] : (len ? p[len - 1] : 0);
        acc = (acc << 8) | v;
    }
    acc <<= (bitpos & 7);
    return m ? (uint32_t)(acc >> (64 - m)) : 0u;
}

typedef struct {
    bitreader_t r;       /* reference reader (cache + bit_offset) */
    int intent;          /* 1: absolute reader */
    uint64_t bitpos;     /* intent reader position */
} symreader_t;

static inline int read_next_symbol_x(symreader_t *sr, const sslookup_t *sl, unsigned *sym) {
    uint32_t v;
    if (sl->clo) {                                       /* tolerant tables */
        uint8_t l8;
        int e = canon_lookup(sl, abs_peek(sr->r.p, sr->r.len, sr->bitpos, sl->max_aob), sym, &l8);
        if (e) return e;
        sr->bitpos += l8;
        return 0;
    }
    if (sr->intent) {
        v = abs_peek(sr->r.p, sr->r.len, sr->bitpos, sl->max_aob);
    } else {
        /* Past the end the reference keeps shifting in its stale byte; a run-digit
         * pattern there never terminates (or overruns the output): report it. */
        if (sr->r.stale > 64) return NICE_ORACLE_E_PANIC;
        v = br_read_24bits_noclear(&sr->r, sl->max_aob);
        if (sr->r.hung) return NICE_ORACLE_E_HANG;
    }
    if (v >= sl->lut_len) return NICE_ORACLE_E_PANIC;
    lut_t l;
    if (sl->zlo) {                                       /* lazy LUT: first lower bound <= v */
        int lo = 0, hi = sl->nlazy - 1;
        while (lo < hi) {
            int mid = (lo + hi) >> 1;
            if (sl->zlo[mid] <= v) hi = mid; else lo = mid + 1;
        }
        l.symbol = sl->zsym[lo]; l.aob = sl->zlen[lo];
    } else {
        l = sl->lut[v];
    }
    if (sr->intent) sr->bitpos += l.aob;
    else sr->r.bit_offset = (uint8_t)(sr->r.bit_offset + l.aob);
    *sym = l.symbol;
    return 0;
}

static inline int read_next_symbol(bitreader_t *r, const sslookup_t *sl, unsigned *sym) {
    symreader_t sr;
    sr.r = *r; sr.intent = 0; sr.bitpos = 0;
    int rc = read_next_symbol_x(&sr, sl, sym);
    *r = sr.r;
    return rc;
}

int nice_oracle_decode(const uint8_t *s, size_t len, int mode, uint8_t **out, size_t *out_len,
                       uint32_t *w_out, uint32_t *h_out, uint8_t *ch_out) {
    *out = NULL; *out_len = 0;
    /* header: code.rs:469-483 (io::Read::read on a slice, magic not checked) */
    size_t pos = 0;
    uint8_t hb[13] = {0};
    {
        size_t take = len < 4 ? len : 4; pos += take;                   /* magic */
        uint8_t buf[4] = {0};
        for (int f = 0; f < 2; ++f) {
            size_t t = len - pos < 4 ? len - pos : 4;
            memcpy(buf, s + pos, t); pos += t;                         /* short read keeps old bytes */
            memcpy(hb + 4 + 4 * f, buf, 4);
        }
        uint8_t cb[1] = {0};
        if (pos < len) cb[0] = s[pos++];
        hb[12] = cb[0];
    }
    uint32_t width = ((uint32_t)hb[4] << 24) | ((uint32_t)hb[5] << 16) | ((uint32_t)hb[6] << 8) | hb[7];
    uint32_t height = ((uint32_t)hb[8] << 24) | ((uint32_t)hb[9] << 16) | ((uint32_t)hb[10] << 8) | hb[11];
    size_t ch = hb[12];
    *w_out = width; *h_out = height; *ch_out = (uint8_t)ch;
    const size_t W = width;
    const size_t image_size = W * (size_t)height * ch;
    uint8_t *o = (uint8_t *)calloc(image_size ? image_size : 1, 1);   /* see DESIGN.md: set_len */
    if (!o) return NICE_ORACLE_E_OOM;
    bitreader_t r;
    br_init(&r, s, len, pos);
    sslookup_t L[N_STREAMS];
    memset(L, 0, sizeof(L));
    int rc = 0;
    if (mode == NICE_ORACLE_DEC_TOLERANT) rc = tolerant_tables(&r, L);
    else for (int k = 0; k < N_STREAMS && !rc; ++k) rc = read_header_into_tree(&r, &L[k], STREAM_N[k]);
    const size_t rel_ref[11] = {ch, ch * W, ch * (W - 1), ch * (W - 3), 3 * ch,
                                ch * (3 * W - 1), 3 * ch * W, ch * (3 * W + 1), ch * (W + 3),
                                ch * 3 * (W + 1), ch * 3 * (W - 1)};
    const size_t back_ref[5] = {ch, ch * W, ch * (W - 1), 2 * ch, 2 * ch * W};
    const size_t rowb = ch * W;
    const int intent = (mode == NICE_ORACLE_DEC_STRIDE || mode == NICE_ORACLE_DEC_TOLERANT);
    const size_t step = intent ? ch : 3;                                /* code.rs:659 */
    symreader_t sr;
    sr.r = r; sr.intent = intent;
    sr.bitpos = (uint64_t)r.pos * 8 - (32u - r.bit_offset);             /* after the tables */
    unsigned prefix = 0, v = 0;
#define RS(stream, dst) do { int e_ = read_next_symbol_x(&sr, &L[stream], &(dst)); if (e_) { rc = e_; goto done; } } while (0)
#define IDX(i) do { if ((i) >= image_size) { rc = NICE_ORACLE_E_PANIC; goto done; } } while (0)
    if (rc) goto done;
    if (intent && (ch < 3)) { rc = NICE_ORACLE_E_ARG; goto done; }
    RS(S_PREFIX, prefix);                                               /* code.rs:550 */
    size_t position = 0, prev_pos = 0;
    while (position < image_size) {                                      /* code.rs:573 */
        switch (prefix) {
        case P_LUMA2: {                                                  /* code.rs:579-588 */
            unsigned gs, rs2, bs;
            RS(S_LUMA2_BASE, gs);
            uint8_t g = (uint8_t)(gs - 32);
            size_t up = position - rowb;
            IDX(position + 2); IDX(prev_pos + 2); IDX(up + 2);
            o[position + 1] = (uint8_t)(g + (uint8_t)(((unsigned)o[prev_pos + 1] + o[up + 1]) / 2));
            RS(S_LUMA2_R, rs2);
            o[position] = (uint8_t)((uint8_t)(rs2 - 16) + (uint8_t)(g + (uint8_t)(((unsigned)o[prev_pos] + o[up]) / 2)));
            RS(S_LUMA2_B, bs);
            o[position + 2] = (uint8_t)((uint8_t)(bs - 16) + (uint8_t)(g + (uint8_t)(((unsigned)o[prev_pos + 2] + o[up + 2]) / 2)));
            break;
        }
        case P_SMALL_DIFF: {                                             /* code.rs:589-618 */
            unsigned sd;
            RS(S_SMALL_DIFF, sd);
            int sdi = (int)(int16_t)sd;
            int rd = sdi % 7; sdi = (sdi - rd) / 7;
            int gd = sdi % 7; int bd = (sdi - gd) / 7;
            int rr, rg, rb;
            IDX(position + 2); IDX(prev_pos + 2);
            if (position >= rowb) {
                size_t vp = position - rowb;
                rr = ((int)o[vp] + o[prev_pos]) / 2;
                rg = ((int)o[vp + 1] + o[prev_pos + 1]) / 2;
                rb = ((int)o[vp + 2] + o[prev_pos + 2]) / 2;
            } else {
                rr = o[prev_pos]; rg = o[prev_pos + 1]; rb = o[prev_pos + 2];
            }
            o[position] = (uint8_t)(rd - 3 + rr);
            o[position + 1] = (uint8_t)(gd - 3 + rg);
            o[position + 2] = (uint8_t)(bd - 3 + rb);
            break;
        }
        case P_LUMA: {                                                   /* code.rs:619-629 */
            unsigned k, gs, rs2, bs;
            RS(S_LUMA_REF, k);
            if (k >= 11) { rc = NICE_ORACLE_E_PANIC; goto done; }
            size_t br = rel_ref[k];
            RS(S_LUMA_BASE, gs);
            uint8_t g = (uint8_t)(gs - 32);
            size_t rp = position - br;
            IDX(position + 2); IDX(rp + 2);
            o[position + 1] = (uint8_t)(g + o[rp + 1]);
            RS(S_LUMA_OTHER, rs2);
            o[position] = (uint8_t)((uint8_t)(rs2 - 16) + (uint8_t)(g + o[rp]));
            RS(S_LUMA_OTHER, bs);
            o[position + 2] = (uint8_t)((uint8_t)(bs - 16) + (uint8_t)(g + o[rp + 2]));
            break;
        }
        case P_BACK_REF: {                                               /* code.rs:630-637 */
            unsigned k;
            RS(S_BACK_REF, k);
            if (k >= 5) { rc = NICE_ORACLE_E_PANIC; goto done; }
            size_t rp = position - back_ref[k];
            IDX(position + 2); IDX(rp + 2);
            o[position] = o[rp]; o[position + 1] = o[rp + 1]; o[position + 2] = o[rp + 2];
            break;
        }
        case P_RGB: {                                                    /* code.rs:638-644 */
            size_t vp = position >= rowb ? position - rowb : prev_pos;
            unsigned a0, a1, a2;
            IDX(position + 2); IDX(prev_pos + 2); IDX(vp + 2);
            RS(S_RGB, a0);
            o[position] = (uint8_t)((int)(int16_t)a0 + ((int)o[vp] + o[prev_pos]) / 2);
            RS(S_RGB, a1);
            o[position + 1] = (uint8_t)((int)(int16_t)a1 + ((int)o[vp + 1] + o[prev_pos + 1]) / 2);
            RS(S_RGB, a2);
            o[position + 2] = (uint8_t)((int)(int16_t)a2 + ((int)o[vp + 2] + o[prev_pos + 2]) / 2);
            break;
        }
        default:
            if (intent) { rc = NICE_ORACLE_E_PANIC; goto done; }         /* digit where a pixel starts */
            break;                                                       /* eprintln!, continue */
        }
        prev_pos = position;
        position += step;
        /* intent: the stream ends with the last pixel (no extra prefix read) */
        if (intent && position >= image_size) break;
        RS(S_PREFIX, prefix);                                            /* code.rs:660 */
        if (prefix >= P_RUN1 && prefix <= P_RUN1 + 7) {
            uint8_t shift = 0;
            size_t run = 0;
            const size_t remaining = (image_size - position) / ch;
            while (prefix >= P_RUN1 && prefix <= P_RUN1 + 7) {
                run += (size_t)(prefix - 5) << (shift & 63u);
                shift = (uint8_t)(shift + 3);
                if (intent && run + 1 >= remaining) break;               /* run reaches the end */
                RS(S_PREFIX, prefix);
            }
            run += 1;
            if (intent && run > remaining) { rc = NICE_ORACLE_E_PANIC; goto done; }
            for (size_t i = 0; i < run; ++i) {                          /* code.rs:675-678 */
                size_t dst = position + i * ch;
                IDX(prev_pos + 2); IDX(dst + 2);
                memmove(o + dst, o + prev_pos, 3);
            }
            position += run * ch;
        }
    }
    (void)v;
done:
    for (int k = 0; k < N_STREAMS; ++k) {
        free(L[k].lut); free(L[k].clo); free(L[k].csym); free(L[k].clen);
        free(L[k].zlo); free(L[k].zsym); free(L[k].zlen);
    }
    if (rc) { free(o); return rc; }
    *out = o;
    *out_len = image_size;
    return 0;
#undef RS
#undef IDX
}

void nice_oracle_free(void *p) { free(p); }

/* ------------------------------------------------------------------------- */
/* Known-answer helpers mirroring the reference's inline tests.               */
/* ------------------------------------------------------------------------- */
/* bitwriter.rs:86-97: write_8bits (2,3) x3 then (2,0). Returns bytes written. */
int nice_oracle_kat_writer(uint8_t *out, int cap) {
    sink_t s = {0};
    bitwriter_t b = {&s, 0, 0};
    bw_write_8bits(&b, 2, 3); bw_write_8bits(&b, 2, 3);
    bw_write_8bits(&b, 2, 3); bw_write_8bits(&b, 2, 0);
    int n = (int)s.len < cap ? (int)s.len : cap;
    memcpy(out, s.p, (size_t)n);
    free(s.p);
    return n;
}

/* Sequence driver for the reader KATs (bitreader.rs:106-146).
 * ops[i] = 0: read_bitsu8(bits[i]); 1: read_24bits(bits[i]); 2: read_24bits_noclear(bits[i]). */
int nice_oracle_kat_reader(const uint8_t *data, size_t len, const int *ops, const int *bits,
                           int n, uint32_t *results) {
    bitreader_t r;
    br_init(&r, data, len, 0);
    for (int i = 0; i < n; ++i) {
        if (ops[i] == 0) {
            uint8_t v;
            if (br_read_bitsu8(&r, (uint8_t)bits[i], &v)) return -1;
            results[i] = v;
        } else if (ops[i] == 1) {
            results[i] = br_read_24bits(&r, (uint8_t)bits[i]);
        } else {
            results[i] = br_read_24bits_noclear(&r, (uint8_t)bits[i]);
        }
    }
    return 0;
}

/* hfe.rs:300-348: one 256-symbol stream with counts i*10, encoded through
 * to_encoded_output + appended cache, then decoded symbol by symbol.
 * Returns 0 if every symbol round-trips; fills the stream length and max_aob. */
int nice_oracle_kat_hfe(size_t *stream_len, uint8_t *max_aob) {
    const int n = 256;
    uint64_t *occ = (uint64_t *)calloc((size_t)n, 8);
    for (int i = 0; i < n; ++i) occ[i] = (uint64_t)i * 10;
    uint8_t *aob = (uint8_t *)malloc((size_t)n);
    uint64_t *code = (uint64_t *)malloc(8 * (size_t)n);
    nice_oracle_code_lengths(occ, n, aob);
    nice_oracle_canonical(aob, n, code);
    sink_t s = {0};
    bitwriter_t b = {&s, 0, 0};
    uint8_t mx = 0;
    for (int i = 0; i < n; ++i) if (aob[i] > mx) mx = aob[i];
    bw_write_8bits(&b, 5, mx);
    uint8_t fb = field_bits(mx);
    for (int i = 0; i < n; ++i) bw_write_8bits(&b, fb, aob[i]);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < i * 10; ++j) bw_write_24bits(&b, aob[i], (uint32_t)code[i]);
    sink_put(&s, (uint8_t)(b.cache >> 24));
    for (int sh = 24; sh >= 0; sh -= 8) sink_put(&s, (uint8_t)(b.cache >> sh));
    *stream_len = s.len;
    *max_aob = mx;
    bitreader_t r;
    br_init(&r, s.p, s.len, 0);
    sslookup_t sl = {0};
    int rc = read_header_into_tree(&r, &sl, n);
    for (int i = 0; i < n && !rc; ++i)
        for (int j = 0; j < i * 10 && !rc; ++j) {
            unsigned sym;
            if (read_next_symbol(&r, &sl, &sym) || sym != (unsigned)i) rc = 1;
        }
    free(sl.lut); free(s.p); free(occ); free(aob); free(code);
    return rc;
}

/* ------------------------------------------------------------------------- */
/* Synthetic inputs.                                           */
/* ------------------------------------------------------------------------- */
void nice_oracle_gen_syn_v1(uint8_t *px, uint32_t W, uint32_t H, uint32_t C, uint32_t seed) {
    static const int AMP[8] = {0, 1, 2, 3, 8, 24, 64, 256};
    uint32_t s = seed;
    for (uint32_t y = 0; y < H; ++y) {
        int amp = AMP[(8ull * y) / H];
        for (uint32_t x = 0; x < W; ++x) {
            uint8_t *p = px + ((size_t)y * W + x) * C;
            unsigned bx = W > 1 ? (200u * x) / (W - 1) : 0;
            unsigned by = H > 1 ? (200u * y) / (H - 1) : 0;
            unsigned base[3] = {bx, by, (bx + by) / 2};
            if (((x / 16) + (y / 16)) % 7 == 0) {
                p[0] = 40; p[1] = 80; p[2] = 120;
            } else {
                for (int c = 0; c < 3; ++c) {
                    s ^= s << 13; s ^= s >> 17; s ^= s << 5;
                    int n;
                    if (amp == 0) n = 0;
                    else if (amp < 256) n = (int)(s % (uint32_t)amp) - amp / 2;
                    else n = (int)(s & 255u);
                    p[c] = (uint8_t)((int)base[c] + n);
                }
            }
            if (C == 4) p[3] = 255;
        }
    }
}

void nice_oracle_gen_gradient(uint8_t *px, uint32_t W, uint32_t H, uint32_t C) {
    for (uint32_t y = 0; y < H; ++y)
        for (uint32_t x = 0; x < W; ++x) {
            uint8_t *p = px + ((size_t)y * W + x) * C;
            p[0] = (uint8_t)(W > 1 ? (255u * x) / (W - 1) : 0);
            p[1] = (uint8_t)(H > 1 ? (255u * y) / (H - 1) : 0);
            p[2] = (uint8_t)((W + H > 2) ? (255u * (x + y)) / (W + H - 2) : 0);
            if (C == 4) p[3] = 255;
        }
}

/* A frame whose small-diff symbol counts grow like Fibonacci numbers, so the
 * Huffman merge of hfe.rs:72-84 chains them: the rarest emitted symbols get
 * codes of K-1 bits or more (over 25 bits for K >= 28).  Test input for the
 * long-code writer path (bitwriter.rs:55-73 with bit_offset + length > 32).
 * Pixels are generated in raster order as pred + delta (code.rs:208-247:
 * pred = floor((U+L)/2) from row 1 on, L in row 0) with delta one of K fixed
 * small diffs drawn with weights F(k+2); a draw is rejected when it would
 * make the pixel a run member or a back reference (code.rs:191-206, 371-407)
 * or leave 0..255; pixels with no valid draw take a large jump (RGB / luma). */
/* Pixel i takes delta dl: in range, drifting toward mid-range, and coded
 * (not a run member) with no back reference k = 1..4.  Writes p on success. */
static int deep_try(uint8_t *px, size_t i, uint32_t W, uint32_t C, const int pred[3], const int dl[3]) {
    uint8_t *p = px + i * C;
    int v[3];
    for (int c = 0; c < 3; ++c) {
        v[c] = pred[c] + dl[c];
        if (v[c] < 0 || v[c] > 255) return 0;
        if ((pred[c] > 215 && dl[c] > 0) || (pred[c] < 40 && dl[c] < 0)) return 0;
    }
    for (int c = 0; c < 3; ++c) p[c] = (uint8_t)v[c];
    const size_t q = i * C;
    if (rgb_eq(px, q, q - C)) return 0;
    if (i >= W && rgb_eq(px, q, q - (size_t)W * C)) return 0;
    if (i >= W - 1 && W >= 1 && rgb_eq(px, q, q - (size_t)(W - 1) * C)) return 0;
    if (i >= 2 && rgb_eq(px, q, q - 2 * (size_t)C)) return 0;
    if (i >= 2 * (size_t)W && rgb_eq(px, q, q - 2 * (size_t)W * C)) return 0;
    return 1;
}

/* force (ascending pixel indices): those pixels take the rarest delta still
 * available, so the rarest (longest-code) symbols land there. */
static void gen_deep(uint8_t *px, uint32_t W, uint32_t H, uint32_t C, uint32_t seed, uint32_t K,
                     const uint64_t *force, size_t n_force, uint32_t flat_y0, uint32_t flat_y1) {
    if (K > 40) K = 40;
    if (K < 2) K = 2;
    int dl[40][3];
    uint64_t left[40], total = 0;
    uint64_t fa = 1, fb = 2;   /* F(2), F(3) */
    uint32_t s = seed ? seed : 1u;
    size_t fi = 0;
#define XS() (s ^= s << 13, s ^= s >> 17, s ^= s << 5, s)
    for (uint32_t k = 0; k < K; ++k) {
        /* distinct nonzero deltas, alternating in sign by rank */
        int c = (int)k + 1, sg = (k & 1) ? -1 : 1;
        dl[k][0] = sg * (1 + (c % 3));
        dl[k][1] = sg * ((c / 3) % 4);
        dl[k][2] = -sg * ((c / 12) % 4);
        left[k] = fa;
        total += fa;
        uint64_t t = fa + fb; fa = fb; fb = t;
    }
    const size_t N = (size_t)W * H;
    for (size_t i = 0; i < N; ++i) {
        uint8_t *p = px + i * C;
        if (C == 4) p[3] = 255;
        if (i == 0) { p[0] = 128; p[1] = 128; p[2] = 128; continue; }
        if (i / W >= flat_y0 && i / W < flat_y1) {   /* one flat colour: a single run, no draws */
            p[0] = 17; p[1] = 99; p[2] = 201;
            continue;
        }
        int pred[3];
        const uint8_t *L = px + (i - 1) * C;
        for (int c = 0; c < 3; ++c)
            pred[c] = i >= W ? ((int)px[(i - W) * C + c] + (int)L[c]) / 2 : (int)L[c];
        int ok = 0;
        while (fi < n_force && force[fi] < i) ++fi;
        if (fi < n_force && force[fi] == i)
            for (uint32_t k = 0; k < K && !ok; ++k)
                if (left[k] && deep_try(px, i, W, C, pred, dl[k])) { ok = 1; left[k] -= 1; total -= 1; }
        for (int tries = 0; tries < 48 && !ok && total; ++tries) {
            uint64_t r = ((uint64_t)XS() << 32 | XS()) % total;
            uint32_t k = 0;
            while (r >= left[k]) { r -= left[k]; ++k; }
            if (!deep_try(px, i, W, C, pred, dl[k])) continue;
            ok = 1;
            left[k] -= 1;
            total -= 1;
        }
        if (!ok)
            for (int c = 0; c < 3; ++c) p[c] = (uint8_t)(pred[c] + 64 + 37 * c + (XS() & 15));
    }
#undef XS
}

void nice_oracle_gen_deep_codes(uint8_t *px, uint32_t W, uint32_t H, uint32_t C, uint32_t seed, uint32_t K) {
    gen_deep(px, W, H, C, seed, K, NULL, 0, 0, 0);
}

void nice_oracle_gen_deep_codes_at(uint8_t *px, uint32_t W, uint32_t H, uint32_t C, uint32_t seed, uint32_t K,
                                   const uint64_t *force, size_t n_force) {
    gen_deep(px, W, H, C, seed, K, force, n_force, 0, 0);
}

/* as gen_deep_codes_at, with rows [flat_y0, flat_y1) one flat colour (a run
 * that consumes no draws, so the Fibonacci counts stay intact) */
void nice_oracle_gen_deep_codes_flat(uint8_t *px, uint32_t W, uint32_t H, uint32_t C, uint32_t seed, uint32_t K,
                                     const uint64_t *force, size_t n_force, uint32_t flat_y0, uint32_t flat_y1) {
    gen_deep(px, W, H, C, seed, K, force, n_force, flat_y0, flat_y1);
}

/* A frame of RGB-mode pixels (code.rs:341-366) whose residuals against the
 * prediction floor((U+L)/2) (L in row 0) take 11 values per channel with
 * geometric weights 2^-(k+1), except rows noise[0..n_noise) which are uniform
 * noise.  The Huffman tree of stream 0 is then a chain, so the noise rows'
 * residuals get long (but <= 25-bit) codes: over 32 bits per pixel
 * (enc_pack's over-cap path at the real cap). */
void nice_oracle_gen_rgb_field(uint8_t *px, uint32_t W, uint32_t H, uint32_t C, uint32_t seed,
                               const uint32_t *noise, size_t n_noise) {
    uint32_t s = seed ? seed : 1u;
#define XS() (s ^= s << 13, s ^= s >> 17, s ^= s << 5, s)
    const size_t N = (size_t)W * H;
    size_t ni = 0;
    for (size_t i = 0; i < N; ++i) {
        uint8_t *p = px + i * C;
        if (C == 4) p[3] = 255;
        const uint32_t y = (uint32_t)(i / W);
        while (ni < n_noise && noise[ni] < y) ++ni;
        const int is_noise = ni < n_noise && noise[ni] == y;
        const uint32_t r = XS();
        for (int c = 0; c < 3; ++c) {
            int pred = 0;
            if (i >= W) pred = ((int)px[(i - W) * C + c] + (int)px[(i - 1) * C + c]) / 2;
            else if (i > 0) pred = px[(i - 1) * C + c];
            /* geometric residual: value k (P = 2^-(k+1), k < 11) per channel */
            const uint32_t bits = (r >> (10 * c)) & 0x3FFu;
            const int k = bits ? __builtin_ctz(bits) : 10;
            p[c] = is_noise ? (uint8_t)(r >> (8 * c)) : (uint8_t)(pred + 40 + 13 * k);
        }
    }
#undef XS
}

/* ------------------------------------------------------------------------- */
/* image.rs:45-102 Image::calc_pos_from (5x5 sub-block boustrophedon order;   */
/* unused by the reference codec).  usize arithmetic, release wrapping;       */
/* returns UINT64_MAX where the reference would panic (division by zero).     */
/* ------------------------------------------------------------------------- */
uint64_t nice_oracle_calc_pos_from(uint64_t width, uint64_t height, uint64_t index) {
    const uint64_t SH = 5, SW = 5;                                        /* image.rs:3-4 */
    const uint64_t h_left = height % SH, w_left = width % SW;             /* image.rs:34-35 */
    const uint64_t image_size = width * height;                           /* image.rs:36 */
    const uint64_t width_block_size = width * SH;                         /* image.rs:37 */
    const uint64_t width_minus_leftover = width - width % SW;             /* image.rs:38 */
    const uint64_t h_minus_left_times_w = (height - height % SH) * width; /* image.rs:39 */
    uint64_t sub_h, sub_w, remainder, offset;
    sub_h = (index >= h_minus_left_times_w && index < image_size) ? h_left : SH;   /* :58-66 */
    if (width_block_size == 0) return UINT64_MAX;
    offset = index - index % width_block_size;                            /* :68 */
    remainder = index - offset;                                           /* :69 */
    sub_w = (remainder >= sub_h * width_minus_leftover && index < image_size) ? w_left : SW;   /* :71-78 */
    const uint64_t area = sub_w * sub_h;
    if (area == 0 || sub_w == 0) return UINT64_MAX;
    const uint64_t sub_mod2 = (remainder / area) & 1u;                    /* :79 */
    offset += remainder / area * sub_w;                                   /* :80 */
    remainder = remainder % area;                                         /* :81 */
    const uint64_t rows_mod2 = (remainder / sub_w) & 1u;                  /* :83 */
    if (sub_mod2 == 0) offset += remainder / sub_w * width;               /* :84-88 */
    else offset += (sub_h - remainder / sub_w - 1) * width;               /* :89-93 */
    offset += rows_mod2 == 1 ? sub_w - (remainder % sub_w) - 1 : remainder % sub_w;   /* :95 */
    return offset;
}
