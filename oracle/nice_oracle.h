/* nice_oracle.h -- TEST INFRASTRUCTURE ONLY (see nice_oracle.c header).
 * CPU restatement of the reference NICE2 encoder/decoder used as the parity
 * checker and the timed CPU baseline.  Never linked into the product. */
#ifndef NICE_ORACLE_H
#define NICE_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    NICE_ORACLE_OK = 0,
    NICE_ORACLE_E_ARG = -1,
    NICE_ORACLE_E_OOM = -2,
    NICE_ORACLE_E_PANIC = -3,  /* the reference would panic (index OOB, EOF in read_exact, ...) */
    NICE_ORACLE_E_DOMAIN = -4, /* code tables outside the decodable domain (see read_header_into_tree) */
    NICE_ORACLE_E_HANG = -5    /* the reference decoder would loop forever (bitreader.rs:88-97 u8 wrap) */
};

/* DEC_STRIDE: pixel stride = channels (intent); DEC_TOLERANT: DEC_STRIDE plus the
 * tolerant table header of SURVEY.md Appendix A.5 (spilled max fields repaired). */
enum { NICE_ORACLE_DEC_REFERENCE = 0, NICE_ORACLE_DEC_STRIDE = 1, NICE_ORACLE_DEC_TOLERANT = 2 };

typedef struct {
    uint8_t max_aob[10];       /* per-stream max code length (hfe.rs:97) */
    uint8_t max_emitted_aob;   /* max code length over emitted symbols */
    uint64_t n_symbols, n_coded, n_backref, n_smalldiff, n_luma2, n_luma, n_rgb, n_run_pixels;
    uint64_t header_end;       /* file bytes written before the first data symbol */
    uint64_t hist_total;
    uint64_t hist[858];        /* symbol counts, streams concatenated in id order */
    uint8_t aob[858];          /* code lengths, same layout */
    uint64_t n_long_emits;     /* emitted codes longer than 25 bits */
    uint64_t n_wrapped_emits;  /* writes with pending bits + length > 32 (bitwriter.rs:63-64 wrap) */
} nice_oracle_stats;

int nice_oracle_encode(const uint8_t *in, size_t in_len, uint32_t width, uint32_t height,
                       uint8_t channels, uint8_t channels_out,
                       uint8_t **out, size_t *out_len, nice_oracle_stats *stats);
int nice_oracle_decode(const uint8_t *s, size_t len, int mode, uint8_t **out, size_t *out_len,
                       uint32_t *w, uint32_t *h, uint8_t *ch);
void nice_oracle_free(void *p);

void nice_oracle_code_lengths(const uint64_t *counts, int n, uint8_t *aob);
void nice_oracle_canonical(const uint8_t *aob, int n, uint64_t *code);

int nice_oracle_kat_writer(uint8_t *out, int cap);
int nice_oracle_kat_reader(const uint8_t *data, size_t len, const int *ops, const int *bits,
                           int n, uint32_t *results);
int nice_oracle_kat_hfe(size_t *stream_len, uint8_t *max_aob);

void nice_oracle_gen_syn_v1(uint8_t *px, uint32_t W, uint32_t H, uint32_t C, uint32_t seed);
void nice_oracle_gen_gradient(uint8_t *px, uint32_t W, uint32_t H, uint32_t C);
uint64_t nice_oracle_calc_pos_from(uint64_t width, uint64_t height, uint64_t index);
void nice_oracle_gen_deep_codes(uint8_t *px, uint32_t W, uint32_t H, uint32_t C, uint32_t seed, uint32_t K);
/* encode, plus px_bit[i] = stream bit of coded pixel i's first symbol (UINT64_MAX: run member),
 * px_bit[W*H] = the data end bit */
int nice_oracle_encode_bitpos(const uint8_t *in, size_t in_len, uint32_t width, uint32_t height,
                              uint8_t channels, uint8_t **out, size_t *out_len, uint64_t *px_bit);
/* as gen_deep_codes_at; rows [flat_y0, flat_y1) one flat colour (a run) */
void nice_oracle_gen_deep_codes_flat(uint8_t *px, uint32_t W, uint32_t H, uint32_t C, uint32_t seed, uint32_t K,
                                     const uint64_t *force, size_t n_force, uint32_t flat_y0, uint32_t flat_y1);
/* RGB-mode frame with geometric residuals per channel; rows noise[] (ascending) uniform noise */
void nice_oracle_gen_rgb_field(uint8_t *px, uint32_t W, uint32_t H, uint32_t C, uint32_t seed,
                               const uint32_t *noise, size_t n_noise);
/* as gen_deep_codes; pixels force[0..n_force) (ascending) take the rarest symbols */
void nice_oracle_gen_deep_codes_at(uint8_t *px, uint32_t W, uint32_t H, uint32_t C, uint32_t seed, uint32_t K,
                                   const uint64_t *force, size_t n_force);

#ifdef __cplusplus
}
#endif
#endif
