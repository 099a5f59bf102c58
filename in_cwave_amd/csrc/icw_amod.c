/*
 * icw_amod.c -- the drop-in decode boundary (include/icw_amod.h), in plain C on top of the
 * batched C ABI (include/icw.h).  A decoding context is a one-stream icw_ctx; every sample is
 * rendered by the gfx950 kernels (there is no CPU path).
 *
 * Mirrors: mod_context_init / mod_context_fopen (in_cwave.c:46-80, 207-236), the DSP half of
 * amod_process_samples (adv_modulator.c:604-760), amod_get_clips_peaks (adv_modulator.c:445-465)
 * over the decoding contexts, and the DSP-list primitives amod_add_lastdsp / amod_del_lastdsp /
 * amod_del_dsplist / amod_set_output_plug (adv_modulator.c:360-441) over them.
 */
#include <stdlib.h>
#include <string.h>

#include "../../include/icw_amod.h"

struct icw_mod_context {
    icw_ctx *ctx;
    icw_config cfg;
    int out_size;
};

icw_mod_context *icw_mod_context_create(const icw_config *cfg, const icw_node *nodes, int n_nodes, int device,
                                        int *status)
{
    int rc, accepted = 0;
    icw_mod_context *mc;
    if (status) *status = ICW_OK;
    if (!cfg) {
        if (status) *status = ICW_EINVAL;
        return NULL;
    }
    mc = (icw_mod_context *)calloc(1, sizeof(*mc));
    if (!mc) {
        if (status) *status = ICW_ENOMEM;
        return NULL;
    }
    mc->cfg = *cfg;
    rc = icw_create(cfg, nodes, n_nodes, 1, device, &mc->ctx, &accepted);
    if (rc != ICW_OK) {
        free(mc);
        if (status) *status = rc;
        return NULL;
    }
    mc->out_size = 2 * icw_render_size(mc->ctx);
    rc = icw_prepare(mc->ctx, 0);
    if (rc != ICW_OK) {
        icw_destroy(mc->ctx);
        free(mc);
        if (status) *status = rc;
        return NULL;
    }
    return mc;
}

icw_ctx *icw_mod_context_ctx(icw_mod_context *mc) { return mc ? mc->ctx : NULL; }

void icw_mod_context_destroy(icw_mod_context *mc)
{
    if (!mc) return;
    icw_destroy(mc->ctx);
    free(mc);
}

/* mod_context_fopen (in_cwave.c:207-236): need24bits is read first (the.cfg.need24bits, :212), the
 * reader and the clears follow, and the renders get the depth last (sound_render_set_outbits on both,
 * :233-234); the caller's next buffers are sized from the new out_size (playback.c:215, transcode.c:55) */
int icw_mod_context_fopen(icw_mod_context *mc, uint32_t sample_rate, uint32_t fmt, uint32_t channels,
                          int64_t n_samples, uint32_t fade_in_ms, uint32_t fade_out_ms, uint32_t sec_align,
                          int clr_nframe, int clr_hilb, int need24bits)
{
    int rc;
    if (!mc) return ICW_EINVAL;
    /* the arguments the context would refuse, before anything changes (icw_set_input repeats them) */
    if (fmt > ICW_FMT_CW_F32 || channels == 0 || sample_rate == 0 || sample_rate > ICW_MAX_FS_SRC || n_samples < 0)
        return ICW_EINVAL;
    rc = icw_set_input(mc->ctx, sample_rate, fmt, channels);
    if (rc != ICW_OK) return rc;
    mc->cfg.sample_rate = sample_rate;
    mc->cfg.in_format = fmt;
    mc->cfg.in_channels = channels;
    rc = icw_stream_open(mc->ctx, 0, n_samples, fade_in_ms, fade_out_ms, sec_align, clr_nframe, clr_hilb);
    if (rc == ICW_OK) rc = icw_set_outbits(mc->ctx, need24bits);
    /* out_size and the depth always describe the context as it now is, even after a device error part
     * way (the caller sizes its next buffers from them; after ICW_EDEVICE it should reopen the track) */
    mc->out_size = 2 * icw_render_size(mc->ctx);
    mc->cfg.need24bits = mc->out_size == 6 ? 1 : 0;
    return rc;
}

int icw_amod_process_samples(char *buf, icw_mod_context *mc, const void *tbuff, unsigned n_frames)
{
    /* bytes per channel sample: HRW_FMT_* (xwave_reader.c:553-580), then the CWAVE complex samples
     * (cw_slen, xwave_reader.c:246-252): the reader hands either kind to amod_process_samples */
    static const unsigned fmt_bytes[9] = {1, 2, 3, 4, 4, 16, 4, 6, 8};
    unsigned fsz;
    int rc;
    if (!mc || (n_frames && (!buf || !tbuff)) || mc->cfg.in_format > ICW_FMT_CW_F32) return ICW_EINVAL;
    if (n_frames == 0) return 0;                    /* EOF: nothing read */
    fsz = fmt_bytes[mc->cfg.in_format] * mc->cfg.in_channels;
    rc = icw_process_streams(mc->ctx, 0, 1, tbuff, (size_t)n_frames * fsz, buf,
                             (size_t)n_frames * (size_t)mc->out_size, (int)n_frames, 0u, NULL, NULL);
    return rc == ICW_OK ? (int)n_frames : rc;
}

int icw_mod_context_seek(icw_mod_context *mc, int64_t frame_pos, int reset_hilb)
{
    int rc;
    if (!mc) return ICW_EINVAL;
    rc = icw_stream_seek(mc->ctx, 0, frame_pos);
    if (rc == ICW_OK && reset_hilb) rc = icw_stream_reset_hilbert(mc->ctx, 0);
    return rc;
}

int icw_mod_context_out_size(const icw_mod_context *mc)
{
    return mc ? mc->out_size : ICW_EINVAL;
}

int icw_mod_context_meters(icw_mod_context *mc, int reset, icw_meters *m)
{
    if (!mc) return ICW_EINVAL;
    return icw_get_meters(mc->ctx, 0, reset, m);
}

int icw_amod_get_clips_peaks(icw_mod_context *const *mcs, int n, unsigned *lc, unsigned *rc, double *lpv,
                             double *rpv, int is_reset)
{
    unsigned cl[2] = {0u, 0u};
    double pk[2] = {ICW_SR_ZERO_SIGNAL_DB, ICW_SR_ZERO_SIGNAL_DB};
    int i, ch, st;
    icw_meters m;
    if (!mcs || n < 0 || !lc || !rc || !lpv || !rpv) return ICW_EINVAL;
    /* the reset clears every context first (am.l/r_clips = 0, am.l/r_peak = SR_ZERO_SIGNAL_DB) */
    if (is_reset)
        for (i = 0; i < n; ++i)
            if (mcs[i] && (st = icw_get_meters(mcs[i]->ctx, 0, 1, &m)) != ICW_OK) return st;
    for (i = 0; i < n; ++i) {
        if (!mcs[i]) continue;
        if ((st = icw_get_meters(mcs[i]->ctx, 0, 0, &m)) != ICW_OK) return st;
        for (ch = 0; ch < 2; ++ch) {
            cl[ch] += m.clips[ch];
            if (m.peak_db[ch] > pk[ch]) pk[ch] = m.peak_db[ch];
        }
    }
    *lc = cl[0];
    *rc = cl[1];
    *lpv = pk[0];
    *rpv = pk[1];
    return ICW_OK;
}

/* The list primitives over the contexts, in order, stopping at the first error (include/icw_amod.h).
 * The contexts hold the same list, so a list refused by graph_accept (ICW_EGRAPH) is refused by the
 * first context, before anything changed; only a device error after an earlier context took the edit
 * leaves them apart, and the host then re-sends the whole list (icw_set_graph) to each. */
int icw_amod_del_lastdsp(icw_mod_context *const *mcs, int n)
{
    int i, st;
    if (!mcs || n < 0) return ICW_EINVAL;
    for (i = 0; i < n; ++i)
        if (mcs[i] && (st = icw_graph_del_last(mcs[i]->ctx)) != ICW_OK) return st;
    return ICW_OK;
}

int icw_amod_del_dsplist(icw_mod_context *const *mcs, int n)
{
    int i, st;
    if (!mcs || n < 0) return ICW_EINVAL;
    for (i = 0; i < n; ++i)
        if (mcs[i] && (st = icw_graph_del_all(mcs[i]->ctx)) != ICW_OK) return st;
    return ICW_OK;
}

int icw_amod_add_lastdsp(icw_mod_context *const *mcs, int n, const icw_node *node)
{
    int i, st;
    if (!mcs || n < 0 || !node) return ICW_EINVAL;
    for (i = 0; i < n; ++i)
        if (mcs[i] && (st = icw_graph_add_last(mcs[i]->ctx, node)) != ICW_OK) return st;
    return ICW_OK;
}

int icw_amod_set_output_plug(icw_mod_context *const *mcs, int n, int index, int plug)
{
    int i, st;
    if (!mcs || n < 0) return ICW_EINVAL;
    for (i = 0; i < n; ++i)
        if (mcs[i] && (st = icw_graph_set_output_plug(mcs[i]->ctx, index, plug)) != ICW_OK) return st;
    return ICW_OK;
}
