/*
 * examples/icw_transcode.c -- a C host in the shape of the reference's transcode / playback
 * plumbing (transcode.c:82-100, playback.c:567-671): a reader hands raw blocks to the decode
 * boundary, which renders them on the MI355X through include/icw_amod.h.
 *
 *   icw_transcode in.wav out.wav [block_frames=576] [graph: master|shift|pmmix] [bits: 16|24]
 *
 * With ICW_TIMING=1 in the environment it times every boundary call (host buffers in and out,
 * the call returns when the block's bytes are in `out`, as the DecodeThread needs them) and prints
 * one JSON line on stdout: decode throughput and the per-block latency distribution (C1 of
 * SURVEY 8(d)).  File I/O is outside the timed calls.
 *
 * The WAV reader handles PCM u8/16/24/32 and IEEE float32 (the RWAVE formats of
 * xwave_reader.c:205-239); the output is stereo 16- or 24-bit PCM like the plugin's.
 */
#define _POSIX_C_SOURCE 199309L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../include/icw_amod.h"

static uint32_t rd32(const unsigned char *p) { return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24); }
static uint16_t rd16(const unsigned char *p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static void wr32(unsigned char *p, uint32_t v) { p[0] = v; p[1] = v >> 8; p[2] = v >> 16; p[3] = v >> 24; }
static void wr16(unsigned char *p, uint16_t v) { p[0] = v; p[1] = v >> 8; }

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static int cmp_d(const void *a, const void *b)
{
    double x = *(const double *)a, y = *(const double *)b;
    return (x > y) - (x < y);
}

static void node_defaults(icw_node *n, int mode)
{
    memset(n, 0, sizeof(*n));
    n->mode = mode;
    n->gain[0] = n->gain[1] = mode == ICW_MODE_MASTER ? 0.8 : 1.0;   /* in_cwave.h:166-167 */
    n->lock_gain = 1;
}

int main(int argc, char **argv)
{
    if (argc < 3) {
        fprintf(stderr, "usage: %s in.wav out.wav [block_frames] [master|shift|pmmix] [16|24]\n", argv[0]);
        return 2;
    }
    unsigned block = argc > 3 ? (unsigned)atoi(argv[3]) : 576;             /* NS_PERTIME */
    const char *gname = argc > 4 ? argv[4] : "shift";
    int bits = argc > 5 ? atoi(argv[5]) : 16;
    FILE *f = fopen(argv[1], "rb");
    if (!f) { perror(argv[1]); return 1; }
    unsigned char hdr[12];
    if (fread(hdr, 1, 12, f) != 12 || memcmp(hdr, "RIFF", 4) || memcmp(hdr + 8, "WAVE", 4)) {
        fprintf(stderr, "not a RIFF/WAVE file\n");
        return 1;
    }
    unsigned fmt_tag = 0, channels = 0, rate = 0, bps = 0;
    uint32_t data_bytes = 0;
    for (;;) {
        unsigned char ch[8];
        if (fread(ch, 1, 8, f) != 8) { fprintf(stderr, "no data chunk\n"); return 1; }
        uint32_t sz = rd32(ch + 4);
        if (!memcmp(ch, "fmt ", 4)) {
            unsigned char fm[40];
            size_t n = sz < sizeof(fm) ? sz : sizeof(fm);
            if (fread(fm, 1, n, f) != n) return 1;
            if (sz > n) fseek(f, (long)(sz - n), SEEK_CUR);
            fmt_tag = rd16(fm);
            channels = rd16(fm + 2);
            rate = rd32(fm + 4);
            bps = rd16(fm + 14);
            if (fmt_tag == 0xFFFE && n >= 26) fmt_tag = rd16(fm + 24);      /* WAVE_FORMAT_EXTENSIBLE */
        } else if (!memcmp(ch, "data", 4)) {
            data_bytes = sz;
            break;
        } else {
            fseek(f, (long)(sz + (sz & 1)), SEEK_CUR);
        }
    }
    uint32_t fmt;
    if (fmt_tag == 3 && bps == 32) fmt = ICW_FMT_F32;
    else if (fmt_tag == 1 && bps == 8) fmt = ICW_FMT_U8;
    else if (fmt_tag == 1 && bps == 16) fmt = ICW_FMT_I16;
    else if (fmt_tag == 1 && bps == 24) fmt = ICW_FMT_I24;
    else if (fmt_tag == 1 && bps == 32) fmt = ICW_FMT_I32;
    else { fprintf(stderr, "unsupported WAV format %u/%u\n", fmt_tag, bps); return 1; }
    const unsigned fsz = (bps / 8) * channels;
    const int64_t n_frames = data_bytes / fsz;

    /* configuration = load_config_default hot-path defaults (config.c:153-207) */
    icw_config cfg;
    memset(&cfg, 0, sizeof(cfg));
    cfg.sample_rate = rate; cfg.in_format = fmt; cfg.in_channels = channels;
    cfg.hilbert_type = 1; cfg.iir_kahan = 1; cfg.iir_subnorm_reject = 1; cfg.frmod_scaled = 1;
    cfg.need24bits = bits == 24; cfg.seed_left = ICW_SEED_LEFT; cfg.seed_right = ICW_SEED_RIGHT;
    cfg.render.dth_bits = 1.0; cfg.render.quantz_type = ICW_QUANTZ_MID_RISER;
    cfg.render.render_type = ICW_RENDER_ROUND; cfg.render.nshape_type = ICW_NSHAPE_FLAT;
    cfg.render.sign_bits16 = 16; cfg.render.sign_bits24 = 24;

    /* DSP list, head (Master) first, executed tail -> head */
    icw_node nodes[4];
    int nn = 1;
    node_defaults(&nodes[0], ICW_MODE_MASTER);
    nodes[0].tout[0] = nodes[0].tout[1] = ICW_S_ADD_REIM;
    if (!strcmp(gname, "shift")) {                     /* Shift(in -> A) + Master(A) */
        nodes[0].inputs[1] = 1;
        node_defaults(&nodes[1], ICW_MODE_SHIFT);
        nodes[1].inputs[0] = 1; nodes[1].n_out = 1;
        nodes[1].fr_shift[0] = 2.0; nodes[1].fr_shift[1] = -2.0;
        nodes[1].is_shift[0] = nodes[1].is_shift[1] = 1;
        nodes[1].lock_shift = nodes[1].sign_lock_shift = 1;
        nn = 2;
    } else if (!strcmp(gname, "pmmix")) {              /* PM(in->A) Shift(A->B) Mix(in+B->C) Master(C) */
        nodes[0].inputs[3] = 1;
        node_defaults(&nodes[1], ICW_MODE_MIX);
        nodes[1].inputs[0] = nodes[1].inputs[2] = 1; nodes[1].n_out = 3;
        node_defaults(&nodes[2], ICW_MODE_SHIFT);
        nodes[2].inputs[1] = 1; nodes[2].n_out = 2;
        nodes[2].fr_shift[0] = 2.0; nodes[2].fr_shift[1] = -2.0;
        nodes[2].is_shift[0] = nodes[2].is_shift[1] = 1;
        nodes[2].lock_shift = nodes[2].sign_lock_shift = 1;
        node_defaults(&nodes[3], ICW_MODE_PM);
        nodes[3].inputs[0] = 1; nodes[3].n_out = 1;
        nodes[3].pm_freq[0] = nodes[3].pm_freq[1] = 4.0;
        nodes[3].pm_level[0] = nodes[3].pm_level[1] = 0.5;
        nodes[3].is_pm[0] = nodes[3].is_pm[1] = 1;
        nodes[3].lock_freq = nodes[3].lock_level = 1;
        nn = 4;
    } else {
        nodes[0].inputs[0] = 1;
    }

    int status = 0;
    icw_mod_context *mc = icw_mod_context_create(&cfg, nodes, nn, -1, &status);
    if (!mc) { fprintf(stderr, "icw_mod_context_create: %s\n", icw_strerror(status)); return 1; }
    status = icw_mod_context_fopen(mc, rate, fmt, channels, n_frames, 0, 0, 0, 0, 0, cfg.need24bits);
    if (status) { fprintf(stderr, "fopen: %s\n", icw_strerror(status)); return 1; }
    const int osz = icw_mod_context_out_size(mc);

    FILE *o = fopen(argv[2], "wb");
    if (!o) { perror(argv[2]); return 1; }
    unsigned char wh[44];
    memcpy(wh, "RIFF", 4); wr32(wh + 4, (uint32_t)(36 + n_frames * osz)); memcpy(wh + 8, "WAVEfmt ", 8);
    wr32(wh + 16, 16); wr16(wh + 20, 1); wr16(wh + 22, 2); wr32(wh + 24, rate);
    wr32(wh + 28, rate * (uint32_t)osz); wr16(wh + 32, (uint16_t)osz); wr16(wh + 34, (uint16_t)(osz * 4));
    memcpy(wh + 36, "data", 4); wr32(wh + 40, (uint32_t)(n_frames * osz));
    fwrite(wh, 1, 44, o);

    unsigned char *in = (unsigned char *)malloc((size_t)block * fsz);
    char *out = (char *)malloc((size_t)block * osz);
    const char *te = getenv("ICW_TIMING");
    const int timing = te && te[0] == '1';
    const int64_t n_blocks = (n_frames + block - 1) / block;
    double *lat = timing ? (double *)malloc(sizeof(double) * (size_t)(n_blocks > 0 ? n_blocks : 1)) : NULL;
    int64_t nb = 0;
    double busy = 0.0;
    int64_t done = 0;
    while (done < n_frames) {                          /* the DecodeThread loop */
        unsigned n = (unsigned)((n_frames - done) < block ? (n_frames - done) : block);
        if (fread(in, fsz, n, f) != n) { fprintf(stderr, "short read\n"); return 1; }
        double t0 = timing ? now_s() : 0.0;
        int r = icw_amod_process_samples(out, mc, in, n);
        if (timing) {
            double dt = now_s() - t0;
            lat[nb++] = dt;
            busy += dt;
        }
        if (r < 0) { fprintf(stderr, "process: %s\n", icw_strerror(r)); return 1; }
        fwrite(out, (size_t)osz, (size_t)r, o);
        done += r;
    }
    icw_meters m;
    icw_mod_context_meters(mc, 0, &m);
    fprintf(stderr, "%lld frames, clips %u/%u, peak %.2f/%.2f dB, desubnorm %llu\n", (long long)done, m.clips[0],
            m.clips[1], m.peak_db[0], m.peak_db[1], (unsigned long long)m.desubnorm);
    if (timing && nb > 0) {
        const double first = lat[0];
        qsort(lat, (size_t)nb, sizeof(double), cmp_d);
        printf("{\"frames\": %lld, \"block_frames\": %u, \"blocks\": %lld, \"decode_s\": %.6f, "
               "\"msamples_per_s\": %.4f, \"block_us\": {\"min\": %.1f, \"p50\": %.1f, \"p99\": %.1f, "
               "\"max\": %.1f, \"first\": %.1f}, \"realtime_x\": %.1f}\n",
               (long long)done, block, (long long)nb, busy, 2.0 * (double)done / busy * 1e-6, lat[0] * 1e6,
               lat[nb / 2] * 1e6, lat[(nb * 99) / 100] * 1e6, lat[nb - 1] * 1e6, first * 1e6,
               (double)done / (double)rate / busy);
    }
    free(lat);
    fclose(o);
    fclose(f);
    free(in);
    free(out);
    icw_mod_context_destroy(mc);
    return 0;
}
