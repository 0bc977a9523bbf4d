/* oracle/dct_oracle.h -- TEST INFRASTRUCTURE ONLY.  See dct_oracle.c. */
#ifndef DCT_ORACLE_H
#define DCT_ORACLE_H
#include <stdint.h>

void orc_dct_matrix(int n, double *d);
void orc_quant_matrix(int n, int quality, double *q);
void orc_dequant_matrix(int n, const double *q, double *dq);
int orc_clamp_quality(int quality);
void orc_forward(int n, const double *d, const double *x, double *out);
/* the same with the context's public tables as given (D = dct_matrix, T = transposed_dct) */
void orc_forward_tables(int n, const double *d, const double *t, const double *x, double *out);
void orc_inverse_tables(int n, const double *d, const double *t, const double *c, double *out);
void orc_inverse(int n, const double *d, const double *c, double *out);
double orc_variance(int n, const double *x);
void orc_adjust(int n, const double *src, double variance, int is_quantize, double *m);
void orc_quantize(int n, const double *qm, int adaptive, double variance, const double *c, int *q);
void orc_dequantize(int n, const double *dqm, int adaptive, double variance, const int *q, double *c);
void orc_block_from_pixels(const uint8_t *px, long stride, int row0, int col0, int n, double *x);
int orc_forward_plane(const uint8_t *px, long stride, int width, int height, int quality, int adaptive,
                      int16_t *out, double *fout, int nthreads);
int orc_inverse_plane(const int16_t *coef, const double *var, int nblocks, int quality, int adaptive,
                      double *recon);
int orc_plane_variance(const uint8_t *px, long stride, int width, int height, double *var);
uint64_t orc_splitmix(uint64_t seed, uint64_t i);
uint8_t orc_synth_pixel(uint64_t seed, int kind, int width, int x, int y);
void orc_synth_plane(uint64_t seed, int kind, int width, int height, uint8_t *px, long stride);

void orc_zigzag_order(int n, int *order);
int orc_rle_encode(int n, const int *coeffs, int *values, int *runs);
void orc_rle_decode(int n, const int *values, const int *runs, int count, int *coeffs);
long orc_rle_encode_plane(const int16_t *coef, long nblk, uint32_t *offsets, uint32_t *symbols);
int orc_huffman_bits(const int *coeffs);
void orc_huffman_bits_plane(const int16_t *coef, long nblk, uint32_t *bits);

#endif
