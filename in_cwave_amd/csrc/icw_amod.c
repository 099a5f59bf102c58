/*
 * icw_amod.c -- the drop-in decode boundary (include/icw_amod.h), in plain C on top of the
 * batched C ABI (include/icw.h).  A decoding context is a one-stream icw_ctx; every sample is
 * rendered by the gfx950 kernels (there is no CPU path).
 *
 * Mirrors: mod_context_init / mod_context_fopen (in_cwave.c:46-80, 207-236), the DSP half of
 * amod_process_samples (adv_modulator.c:604-760), amod_get_clips_peaks (adv_modulator.c:445-465).
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
    return mc;
}

icw_ctx *icw_mod_context_ctx(icw_mod_context *mc) { return mc ? mc->ctx : NULL; }

void icw_mod_context_destroy(icw_mod_context *mc)
{
    if (!mc) return;
    icw_destroy(mc->ctx);
    free(mc);
}

int icw_mod_context_fopen(icw_mod_context *mc, uint32_t sample_rate, uint32_t fmt, uint32_t channels,
                          int64_t n_samples, uint32_t fade_in_ms, uint32_t fade_out_ms, uint32_t sec_align,
                          int clr_nframe, int clr_hilb)
{
    int rc;
    if (!mc) return ICW_EINVAL;
    rc = icw_set_input(mc->ctx, sample_rate, fmt, channels);
    if (rc != ICW_OK) return rc;
    mc->cfg.sample_rate = sample_rate;
    mc->cfg.in_format = fmt;
    mc->cfg.in_channels = channels;
    return icw_stream_open(mc->ctx, 0, n_samples, fade_in_ms, fade_out_ms, sec_align, clr_nframe, clr_hilb);
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
