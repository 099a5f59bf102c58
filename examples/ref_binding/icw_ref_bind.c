/*
 * icw_ref_bind.c -- reference-side binding helpers (see icw_ref_bind.h).  Built inside the
 * in_cwave tree with the reference's own headers; every field read here is a field of the
 * reference's types, and tests/test_ref_binding.py checks each name against in_cwave.h,
 * hblpf.h, sound_render.h and cwave.h.
 */
#include <string.h>

#include "icw_ref_bind.h"

int icw_config_from_ref(const IN_CWAVE_CFG *cfg, BOOL bypass_list, unsigned sample_rate,
                        unsigned fmt, unsigned channels, icw_config *out)
{
    memset(out, 0, sizeof(*out));
    out->sample_rate = sample_rate;
    out->in_format = fmt;
    out->in_channels = channels;
    out->hilbert_type = cfg->iir_filter_no;                       /* IX_LPF_HILB_TYPE0..5 */
    out->iir_kahan = !!cfg->iir_comp_config.is_kahan;
    out->iir_subnorm_reject = !!cfg->iir_comp_config.is_subnorm_reject;
    /* iir_comp_config.subnorm_thr is not used by the sums: the reject compares |w| with the
       BOOL is_subnorm_reject itself (hblpf.c:915, 1046) */
    out->frmod_scaled = !!cfg->is_frmod_scaled;
    out->need24bits = !!cfg->need24bits;
    out->bypass_list = !!bypass_list;
    out->seed_left = ICW_SEED_LEFT;                               /* in_cwave.c:69 */
    out->seed_right = ICW_SEED_RIGHT;                             /* in_cwave.c:70 */
    out->render.dth_bits = cfg->sr_config.dth_bits;
    out->render.quantz_type = cfg->sr_config.quantz_type;
    out->render.render_type = cfg->sr_config.render_type;
    out->render.nshape_type = cfg->sr_config.nshape_type;
    out->render.sign_bits16 = cfg->sr_config.sign_bits16;
    out->render.sign_bits24 = cfg->sr_config.sign_bits24;
    out->fp_check = !!cfg->is_fp_check;
    return ICW_OK;
}

static void node_from_ref(const NODE_DSP *s, icw_node *d)
{
    int i;
    memset(d, 0, sizeof(*d));
    d->mode = s->mode;
    d->gain[0] = s->l_gain;
    d->gain[1] = s->r_gain;
    for (i = 0; i < N_INPUTS && i < ICW_N_INPUTS; ++i)
        d->inputs[i] = s->inputs[i] ? 1 : 0;
    d->xch_mode = s->xch_mode;
    d->iq_invert[0] = s->l_iq_invert;
    d->iq_invert[1] = s->r_iq_invert;
    d->lock_gain = s->lock_gain;
    switch (s->mode) {
    case MODE_MASTER:
        d->tout[0] = s->dsp.mk_master.le.tout;
        d->tout[1] = s->dsp.mk_master.ri.tout;
        break;
    case MODE_SHIFT:
        d->n_out = s->dsp.mk_shift.n_out;
        d->fr_shift[0] = s->dsp.mk_shift.le.fr_shift;
        d->fr_shift[1] = s->dsp.mk_shift.ri.fr_shift;
        d->is_shift[0] = s->dsp.mk_shift.le.is_shift;
        d->is_shift[1] = s->dsp.mk_shift.ri.is_shift;
        d->lock_shift = s->dsp.mk_shift.lock_shift;
        d->sign_lock_shift = s->dsp.mk_shift.sign_lock_shift;
        break;
    case MODE_PM:
        d->n_out = s->dsp.mk_pm.n_out;
        d->pm_freq[0] = s->dsp.mk_pm.le.freq;
        d->pm_freq[1] = s->dsp.mk_pm.ri.freq;
        d->pm_phase[0] = s->dsp.mk_pm.le.phase;
        d->pm_phase[1] = s->dsp.mk_pm.ri.phase;
        d->pm_level[0] = s->dsp.mk_pm.le.level;
        d->pm_level[1] = s->dsp.mk_pm.ri.level;
        d->pm_angle[0] = s->dsp.mk_pm.le.angle;
        d->pm_angle[1] = s->dsp.mk_pm.ri.angle;
        d->is_pm[0] = s->dsp.mk_pm.le.is_pm;
        d->is_pm[1] = s->dsp.mk_pm.ri.is_pm;
        d->lock_freq = s->dsp.mk_pm.lock_freq;
        d->lock_phase = s->dsp.mk_pm.lock_phase;
        d->lock_level = s->dsp.mk_pm.lock_level;
        d->lock_angle = s->dsp.mk_pm.lock_angle;
        break;
    case MODE_MIX:
        d->n_out = s->dsp.mk_mix.n_out;
        break;
    default:                       /* copied as is: icw_create rejects it as amod_init does */
        break;
    }
}

int icw_nodes_from_ref(const NODE_DSP *head, icw_node *nodes, int max_nodes)
{
    int n = 0;
    for (; head; head = head->next) {
        if (n >= max_nodes)
            return ICW_EINVAL;
        node_from_ref(head, &nodes[n++]);
    }
    return n;
}

void icw_node_from_ref(const NODE_DSP *nd, icw_node *out)
{
    node_from_ref(nd, out);
}

int icw_node_index(const NODE_DSP *nd)
{
    int i = 0;
    for (; nd && nd->prev; nd = nd->prev)        /* the head (Master) has no prev */
        ++i;
    return i;
}

int icw_fmt_from_reader(const XWAVE_READER *xr)
{
    unsigned f;
    if (xr->type == XW_TYPE_CWAVE) {
        f = xr->spec.cwave.header.format;                         /* HCW_FMT_PCM_* 0..3 */
        return f <= 3 ? (int)(ICW_FMT_CW_F64 + f) : ICW_EINVAL;
    }
    if (xr->type == XW_TYPE_RWAVE) {
        f = xr->spec.rwave.format;                                /* HRW_FMT_* 0..4 = ICW_FMT_* */
        return f <= HRW_FMT_FLOAT32 ? (int)f : ICW_EINVAL;
    }
    return ICW_EINVAL;
}

int cfg_to_icw(const IN_CWAVE_CFG *cfg, icw_config *c, icw_node nodes[ICW_CFG_MAX_NODES])
{
    /* the track fields (rate, format, channels) are set per file by icw_mod_context_fopen */
    icw_config_from_ref(cfg, amod_get_bypass_list_flag(), 48000, ICW_FMT_I16, 2, c);
    return icw_nodes_from_ref(cfg->dsp_list, nodes, ICW_CFG_MAX_NODES);
}
