/*
 * host/frame_codec.c -- a plain C99 frame-level host of the batched C-ABI
 * (include/dct_amd.h): generates a synthetic frame on the device, runs the
 * forward DCT+quant hot path and the inverse, and prints a 64-bit FNV-1a
 * checksum of the int16 coefficient plane plus the round-trip PSNR
 * (tests/test_entropy.c:376-393 formula, clamped recon).  Then the same frame
 * through the fused round trip (dctq_round_trip_planes: must reproduce the
 * coefficients and the recon of the two calls) and the encoder
 * (dctq_encode_planes: run-length symbol count and an FNV-1a of the stream),
 * and the total of the per-block Huffman sizes (dctq_huffman_bits).
 *
 *   frame_codec WIDTH HEIGHT QUALITY ADAPTIVE SEED [KIND]
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dct_amd.h"

#define CHK(x)                                                                  \
    do {                                                                        \
        int rc_ = (x);                                                          \
        if (rc_) {                                                              \
            fprintf(stderr, "%s: %s\n", #x, dctq_error_string(rc_));            \
            return 1;                                                           \
        }                                                                       \
    } while (0)

int main(int argc, char **argv) {
    if (argc < 6) {
        fprintf(stderr, "usage: %s W H QUALITY ADAPTIVE SEED [KIND]\n", argv[0]);
        return 2;
    }
    int w = atoi(argv[1]), h = atoi(argv[2]), q = atoi(argv[3]), ad = atoi(argv[4]);
    uint64_t seed = strtoull(argv[5], NULL, 10);
    int kind = argc > 6 ? atoi(argv[6]) : 0;
    long long nblk = (long long)(w / 8) * (h / 8);
    void *px, *coef, *var, *rec;
    CHK(dctq_malloc(&px, (size_t)w * h));
    CHK(dctq_malloc(&coef, (size_t)nblk * 128));
    CHK(dctq_malloc(&var, (size_t)nblk * 4));
    CHK(dctq_malloc(&rec, (size_t)nblk * 256));
    dctq_plane pl = {(const uint8_t *)px, w, (long long)w * h, w, h, 1};
    CHK(dctq_synth(seed, kind, &pl, NULL));
    dctq_plan *plan;
    CHK(dctq_plan_create(q, ad, &plan));
    CHK(dctq_forward_quant(plan, &pl, (int16_t *)coef, (int32_t *)var, NULL));
    CHK(dctq_inverse(plan, (const int16_t *)coef, (const int32_t *)var, nblk, (float *)rec, NULL));
    CHK(dctq_synchronize(NULL));
    int16_t *hc = malloc((size_t)nblk * 128);
    float *hr = malloc((size_t)nblk * 256);
    uint8_t *hp = malloc((size_t)w * h);
    CHK(dctq_memcpy_dtoh(hc, coef, (size_t)nblk * 128));
    CHK(dctq_memcpy_dtoh(hr, rec, (size_t)nblk * 256));
    CHK(dctq_memcpy_dtoh(hp, px, (size_t)w * h));
    uint64_t fnv = 1469598103934665603ULL;
    const uint8_t *b = (const uint8_t *)hc;
    for (long long i = 0; i < nblk * 128; ++i) fnv = (fnv ^ b[i]) * 1099511628211ULL;
    double se = 0.0;
    int bw = w / 8;
    for (long long k = 0; k < nblk; ++k)
        for (int e = 0; e < 64; ++e) {
            int y = (int)(k / bw) * 8 + e / 8, x = (int)(k % bw) * 8 + e % 8;
            double r = hr[k * 64 + e];
            r = r < 0 ? 0 : r > 255 ? 255 : r;
            double d = hp[(long long)y * w + x] - r;
            se += d * d;
        }
    double mse = se / ((double)w * h);
    printf("fnv1a:%016llx\n", (unsigned long long)fnv);
    printf("psnr:%.4f\n", 10.0 * __builtin_log10(255.0 * 255.0 / mse));

    /* fused round trip: one launch, same coefficients, same recon within 1e-4 */
    void *coef2, *rec2;
    CHK(dctq_malloc(&coef2, (size_t)nblk * 128));
    CHK(dctq_malloc(&rec2, (size_t)nblk * 256));
    int16_t *c2p = (int16_t *)coef2;
    float *r2p = (float *)rec2;
    CHK(dctq_round_trip_planes(plan, &pl, 1, &c2p, NULL, &r2p, NULL));
    CHK(dctq_synchronize(NULL));
    int16_t *hc2 = malloc((size_t)nblk * 128);
    float *hr2 = malloc((size_t)nblk * 256);
    CHK(dctq_memcpy_dtoh(hc2, coef2, (size_t)nblk * 128));
    CHK(dctq_memcpy_dtoh(hr2, rec2, (size_t)nblk * 256));
    int same = 1;
    double maxd = 0.0;
    for (long long i = 0; i < nblk * 64; ++i) {
        same &= hc2[i] == hc[i];
        double d = hr2[i] - hr[i];
        if (d < 0) d = -d;
        if (d > maxd) maxd = d;
    }
    printf("fused:%s\n", same && maxd <= 1e-4 ? "ok" : "MISMATCH");

    /* encoder: coefficients + zigzag run-length symbols */
    void *off, *sym, *ws;
    const long long cap = 64 * nblk;
    CHK(dctq_malloc(&off, (size_t)(nblk + 1) * 4));
    CHK(dctq_malloc(&sym, (size_t)cap * 4));
    CHK(dctq_malloc(&ws, dctq_encode_workspace_bytes(nblk)));
    /* the most compact format the plan admits (include/dct_amd.h): dctq_encode_planes16's
       2-byte symbols are widened to the 4-byte (uint16)value | run << 16 here, so the digest
       is format-independent; the 4-byte entry point's stream must be the same */
    const int symbytes = dctq_plan_symbol_bytes(plan);
    if (symbytes == 2)
        CHK(dctq_encode_planes16(plan, &pl, 1, &c2p, (uint32_t *)off, (uint16_t *)sym, cap, ws, NULL));
    else
        CHK(dctq_encode_planes(plan, &pl, 1, &c2p, (uint32_t *)off, (uint32_t *)sym, cap, ws, NULL));
    CHK(dctq_synchronize(NULL));
    uint32_t total = 0;
    CHK(dctq_memcpy_dtoh(&total, (const char *)off + (size_t)nblk * 4, 4));
    uint32_t *hs = malloc((size_t)total * 4 + 4);
    CHK(dctq_memcpy_dtoh(hs, sym, (size_t)total * symbytes));
    if (symbytes == 2) {
        const uint16_t *h16 = (const uint16_t *)hs;
        for (long long i = (long long)total - 1; i >= 0; --i) {  /* in place, back to front */
            const uint32_t u = h16[i];
            const int32_t value = (int32_t)((u & 0x3FFu) ^ 0x200u) - 0x200;
            const uint32_t run = u ? u >> 10 : 64u;
            hs[i] = ((uint32_t)value & 0xFFFFu) | run << 16;
        }
        /* the default entry point: 4-byte symbols for every plan (DCTQ_ABI_VERSION 6) */
        void *sym4;
        CHK(dctq_malloc(&sym4, (size_t)cap * 4));
        CHK(dctq_encode_planes(plan, &pl, 1, &c2p, (uint32_t *)off, (uint32_t *)sym4, cap, ws, NULL));
        CHK(dctq_synchronize(NULL));
        uint32_t *h4 = malloc((size_t)total * 4 + 4);
        CHK(dctq_memcpy_dtoh(h4, sym4, (size_t)total * 4));
        printf("symbols4_equal:%d\n", memcmp(h4, hs, (size_t)total * 4) == 0);
        free(h4);
        CHK(dctq_free(sym4));
    }
    printf("abi_version:%d\n", dctq_abi_version());
    printf("symbol_bytes:%d\n", symbytes);
    uint64_t fs = 1469598103934665603ULL;
    const uint8_t *sb = (const uint8_t *)hs;
    for (long long i = 0; i < (long long)total * 4; ++i) fs = (fs ^ sb[i]) * 1099511628211ULL;
    printf("symbols:%u\n", total);
    printf("symbols_fnv1a:%016llx\n", (unsigned long long)fs);

    /* per-block Huffman size (the reference pipeline's get_encoded_size), summed */
    void *bits;
    CHK(dctq_malloc(&bits, (size_t)nblk * 4));
    CHK(dctq_huffman_bits((const int16_t *)coef2, nblk, (uint32_t *)bits, NULL));
    CHK(dctq_synchronize(NULL));
    uint32_t *hb = malloc((size_t)nblk * 4);
    CHK(dctq_memcpy_dtoh(hb, bits, (size_t)nblk * 4));
    unsigned long long tb = 0;
    for (long long i = 0; i < nblk; ++i) tb += hb[i];
    printf("huffman_bits:%llu\n", tb);
    dctq_free(bits);
    free(hb);
    dctq_free(coef2);
    dctq_free(rec2);
    dctq_free(off);
    dctq_free(sym);
    dctq_free(ws);
    free(hc2);
    free(hr2);
    free(hs);
    dctq_plan_destroy(plan);
    dctq_free(px);
    dctq_free(coef);
    dctq_free(var);
    dctq_free(rec);
    free(hc);
    free(hr);
    free(hp);
    return 0;
}
