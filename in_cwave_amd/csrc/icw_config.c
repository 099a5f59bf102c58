/*
 * icw_config.c -- the reference's configuration file format (include/icw_config.h), host-only C.
 *
 * Restates load_config (config.c:813-915): defaults, then "KEY=args" lines up to the first bad
 * one; on any failure everything goes back to the defaults.  Tokens follow handle_string
 * (config.c:380-441): blank-separated, '%' escapes a blank or '%', a '%' before anything else is
 * dropped.  Values are read with sscanf as in handle_bool / _int / _unsigned / _double
 * (config.c:445-541), doubles optionally as 0x<64-bit pattern>.  Out-of-range values are clamped
 * (NODE_CHK, config.c:838-845; HANDLE_CHK, config.c:674).
 */
#include <ctype.h>
#include <inttypes.h>
#include <stdio.h>
#include <string.h>
#include <strings.h>

#include "../../include/icw_config.h"

#define CFG_MAX_LINE 2048             /* MAX_CONFIG_LINE, in_cwave.h:124 */
#define CFG_MAX_KEYW 80               /* MAX_CONFIG_KEYW */
#define CFG_MAX_ARGS (CFG_MAX_LINE - CFG_MAX_KEYW)

/* handle_string, read side: next token of *p into out (at most max_size - 2 chars kept) */
static void next_token(const char **p, char *out, size_t max_size)
{
    size_t cnt = 0;
    const char *s = *p;
    while (*s && (*s == ' ' || *s == '\t')) ++s;
    while (*s && !(*s == ' ' || *s == '\t')) {
        if (*s == '%') {
            ++s;
            if (*s == ' ' || *s == '\t' || *s == '%') {
                if (cnt + 2 < max_size) out[cnt++] = *s;
                ++s;
            }
        } else {
            if (cnt + 2 < max_size) out[cnt++] = *s;
            ++s;
        }
    }
    if (*s) ++s;
    out[cnt] = '\0';
    *p = s;
}

static int rd_bool(const char **p, int32_t *v)
{
    char tok[CFG_MAX_ARGS];
    int x;
    next_token(p, tok, sizeof(tok));
    if (sscanf(tok, "%d", &x) != 1) return 0;
    *v = x ? 1 : 0;
    return 1;
}

static int rd_int(const char **p, int32_t *v)
{
    char tok[CFG_MAX_ARGS];
    int x;
    next_token(p, tok, sizeof(tok));
    if (sscanf(tok, "%d", &x) != 1) return 0;
    *v = x;
    return 1;
}

static int rd_unsigned(const char **p, uint32_t *v)
{
    char tok[CFG_MAX_ARGS];
    unsigned x;
    next_token(p, tok, sizeof(tok));
    if (sscanf(tok, "%u", &x) != 1) return 0;
    *v = x;
    return 1;
}

static int rd_double(const char **p, double *v)
{
    char tok[CFG_MAX_ARGS];
    next_token(p, tok, sizeof(tok));
    if (tok[0] == '0' && (tok[1] == 'x' || tok[1] == 'X')) {
        uint64_t u;
        if (sscanf(tok + 2, "%" SCNx64, &u) != 1) return 0;
        memcpy(v, &u, 8);
        return 1;
    }
    return sscanf(tok, "%lg", v) == 1;
}

#define CLAMP(V, MI, MA) do { if ((V) < (MI)) (V) = (MI); if ((V) > (MA)) (V) = (MA); } while (0)

int icw_node_dsp_parse(const char *args, icw_node *n, char *name, size_t name_size)
{
    char nm[ICW_DSP_NAME_SIZE];
    const char *p = args;
    if (!args || !n) return ICW_EINVAL;
    memset(n, 0, sizeof(*n));
    next_token(&p, nm, sizeof(nm));
    if (name && name_size) {
        strncpy(name, nm, name_size - 1);
        name[name_size - 1] = '\0';
    }
#define RD(T, V) do { if (!rd_##T(&p, &(V))) return ICW_EINVAL; } while (0)
#define RC(T, V, MI, MA) do { RD(T, V); CLAMP(V, MI, MA); } while (0)
    RC(double, n->gain[0], 0.0, 2.0);                         /* MAX_GAIN */
    RC(double, n->gain[1], 0.0, 2.0);
    RD(bool, n->lock_gain);
    for (int i = 0; i < ICW_N_INPUTS; ++i) {
        int32_t b;
        RD(bool, b);
        n->inputs[i] = (uint8_t)b;
    }
    RC(int, n->xch_mode, ICW_XCH_NORMAL, ICW_XCH_MIXLR);      /* XCH_MAX */
    RD(bool, n->iq_invert[0]);
    RD(bool, n->iq_invert[1]);
    RC(int, n->mode, ICW_MODE_MASTER, ICW_MODE_MIX);
    switch (n->mode) {
    case ICW_MODE_MASTER:
        RC(int, n->tout[0], ICW_S_ADD_REIM, ICW_S_IM);
        RC(int, n->tout[1], ICW_S_ADD_REIM, ICW_S_IM);
        break;
    case ICW_MODE_SHIFT:
        RC(double, n->fr_shift[0], -20.0, 20.0);              /* MAX_FSHIFT */
        RD(bool, n->is_shift[0]);
        RC(double, n->fr_shift[1], -20.0, 20.0);
        RD(bool, n->is_shift[1]);
        RC(int, n->n_out, 1, ICW_N_INPUTS);
        RD(bool, n->lock_shift);
        RD(bool, n->sign_lock_shift);
        break;
    case ICW_MODE_PM:
        for (int c = 0; c < 2; ++c) {
            RC(double, n->pm_freq[c], 0.0, 40.0);             /* MAX_PMFREQ */
            RC(double, n->pm_phase[c], -1.0, 1.0);            /* MIN/MAX_PMPHASE */
            RC(double, n->pm_level[c], 0.0, 1.0);             /* MAX_PMLEVEL */
            RC(double, n->pm_angle[c], -1.0, 1.0);            /* MIN/MAX_PMANGLE */
            RD(bool, n->is_pm[c]);
        }
        RC(int, n->n_out, 1, ICW_N_INPUTS);
        RD(bool, n->lock_freq);
        RD(bool, n->lock_phase);
        RD(bool, n->lock_level);
        RD(bool, n->lock_angle);
        break;
    default:                                                  /* MODE_MIX */
        RC(int, n->n_out, 1, ICW_N_INPUTS);
        break;
    }
#undef RC
#undef RD
    return ICW_OK;
}

/* handle_string, write side: " " + token with blanks and '%' escaped */
static int put_token(char *buf, size_t size, size_t *pos, const char *s, size_t max_size)
{
    size_t cnt = 1;
    if (*pos + 1 >= size) return 0;
    buf[(*pos)++] = ' ';
    while (*s && cnt < max_size - 2) {
        if (*s == ' ' || *s == '\t' || *s == '%') {
            if (*pos + 2 >= size) return 0;
            buf[(*pos)++] = '%';
            buf[(*pos)++] = *s++;
            cnt += 2;
        } else {
            if (*pos + 1 >= size) return 0;
            buf[(*pos)++] = *s++;
            cnt += 1;
        }
    }
    buf[*pos] = '\0';
    return 1;
}

static int put_int(char *buf, size_t size, size_t *pos, int v)
{
    int k = snprintf(buf + *pos, size - *pos, " %d", v);
    if (k < 0 || (size_t)k >= size - *pos) return 0;
    *pos += (size_t)k;
    return 1;
}

/* handle_double_bin, write side: " 0x%08I64X" of the bit pattern (config.c:547-552) */
static int put_dbin(char *buf, size_t size, size_t *pos, double v)
{
    uint64_t u;
    memcpy(&u, &v, 8);
    int k = snprintf(buf + *pos, size - *pos, " 0x%08" PRIX64, u);
    if (k < 0 || (size_t)k >= size - *pos) return 0;
    *pos += (size_t)k;
    return 1;
}

int icw_node_dsp_format(const icw_node *n, const char *name, char *buf, size_t size)
{
    /* the write side prints every field with a leading blank; write_conf_line writes
     * "KEY=" + the string from its second character (config.c:365-371) */
    char tmp[CFG_MAX_LINE + 8];
    size_t tp = 0;
    if (!n || !buf) return ICW_EINVAL;
    tmp[0] = '\0';
#define PB(V) do { if (!put_int(tmp, sizeof(tmp), &tp, (V) ? 1 : 0)) return ICW_EINVAL; } while (0)
#define PI(V) do { if (!put_int(tmp, sizeof(tmp), &tp, (int)(V))) return ICW_EINVAL; } while (0)
#define PD(V) do { if (!put_dbin(tmp, sizeof(tmp), &tp, (V))) return ICW_EINVAL; } while (0)
    if (!put_token(tmp, sizeof(tmp), &tp, name ? name : "", ICW_DSP_NAME_SIZE)) return ICW_EINVAL;
    PD(n->gain[0]);
    PD(n->gain[1]);
    PB(n->lock_gain);
    for (int i = 0; i < ICW_N_INPUTS; ++i) PB(n->inputs[i]);
    PI(n->xch_mode);
    PB(n->iq_invert[0]);
    PB(n->iq_invert[1]);
    PI(n->mode);
    switch (n->mode) {
    case ICW_MODE_MASTER:
        PI(n->tout[0]);
        PI(n->tout[1]);
        break;
    case ICW_MODE_SHIFT:
        PD(n->fr_shift[0]); PB(n->is_shift[0]);
        PD(n->fr_shift[1]); PB(n->is_shift[1]);
        PI(n->n_out); PB(n->lock_shift); PB(n->sign_lock_shift);
        break;
    case ICW_MODE_PM:
        for (int c = 0; c < 2; ++c) {
            PD(n->pm_freq[c]); PD(n->pm_phase[c]); PD(n->pm_level[c]); PD(n->pm_angle[c]); PB(n->is_pm[c]);
        }
        PI(n->n_out); PB(n->lock_freq); PB(n->lock_phase); PB(n->lock_level); PB(n->lock_angle);
        break;
    case ICW_MODE_MIX:
        PI(n->n_out);
        break;
    default:
        return ICW_EINVAL;
    }
#undef PB
#undef PI
#undef PD
    const int k = snprintf(buf, size, "NODE_DSP=%s", tmp + 1);
    if (k < 0 || (size_t)k >= size) return ICW_EINVAL;
    return k;
}

/* defaults of config_list (config.c:113-207, 216-296) for the fields kept */
static void cfg_defaults(icw_file_config *o)
{
    const uint32_t sr = o->cfg.sample_rate, fmt = o->cfg.in_format, ch = o->cfg.in_channels;
    memset(o, 0, sizeof(*o));
    o->cfg.sample_rate = sr;
    o->cfg.in_format = fmt;
    o->cfg.in_channels = ch;
    o->cfg.hilbert_type = 1;                  /* IX_LPF_HILB_DEF */
    o->cfg.iir_kahan = 1;
    o->cfg.iir_subnorm_reject = 1;
    o->cfg.frmod_scaled = 1;
    o->cfg.need24bits = 1;                    /* DB_need24bits = TRUE */
    o->cfg.bypass_list = 0;
    o->cfg.seed_left = ICW_SEED_LEFT;
    o->cfg.seed_right = ICW_SEED_RIGHT;
    o->cfg.render.dth_bits = 1.0;             /* DEF_DITHER_BITS */
    o->cfg.render.quantz_type = ICW_QUANTZ_MID_RISER;
    o->cfg.render.render_type = ICW_RENDER_ROUND;
    o->cfg.render.nshape_type = ICW_NSHAPE_FLAT;
    o->cfg.render.sign_bits16 = 16;
    o->cfg.render.sign_bits24 = 24;
    o->subnorm_thr = 1.0E-150;                /* SBN_THR_DEF */
}

/* one "KEY=args" line; returns 1 if accepted */
static int cfg_line(icw_file_config *o, const char *key, const char *args)
{
    const char *p = args;
    int32_t b;
    uint32_t u;
    double d;
#define UNS(NAME, DST, MI, MA) if (!strcasecmp(key, NAME)) { if (!rd_unsigned(&p, &u)) return 0; CLAMP(u, (uint32_t)(MI), (uint32_t)(MA)); DST = u; return 1; }
#define BOOLK(NAME, DST) if (!strcasecmp(key, NAME)) { if (!rd_bool(&p, &b)) return 0; DST = b; return 1; }
#define DBL(NAME, DST, MI, MA) if (!strcasecmp(key, NAME)) { if (!rd_double(&p, &d)) return 0; CLAMP(d, MI, MA); DST = d; return 1; }
    {
        uint32_t ignore_u;
        int32_t ignore_b;
        UNS("VER_CONFIG", o->ver_config, 0u, 0xffffffffu)
        BOOLK("WAV_SUPPORT", ignore_b)
        BOOLK("RWAVE_SUPPORT", ignore_b)
        UNS("IBOX_PARENT", ignore_u, 0, 2)
        BOOLK("LAST_CHANCE", ignore_b)
        UNS("PLAY_SLEEP", ignore_u, 0, 100)
        BOOLK("DISABLE_SLEEP", ignore_b)
        UNS("SEC_ALIGN", o->sec_align, 0, 20)
        UNS("FADE_IN", o->fade_in, 0, 10000)
        UNS("FADE_OUT", o->fade_out, 0, 10000)
        BOOLK("FRMOD_SCALED", o->cfg.frmod_scaled)
        UNS("IIR_HBLPF_IX", o->cfg.hilbert_type, 0, 5)
        BOOLK("IIR_SUM_KAHAN", o->cfg.iir_kahan)
        BOOLK("IIR_SUBN_ZERO", o->cfg.iir_subnorm_reject)
        DBL("IIR_SUBN_THR", o->subnorm_thr, 1.0E-300, 1.0E-40)
        BOOLK("CLR_NFRAME_PT", o->clr_nframe)
        BOOLK("CLR_HILB_PT", o->clr_hilb)
        BOOLK("SHOW_LONGNUMB", ignore_b)
        BOOLK("FP_CHECK", o->fp_check)
        BOOLK("NEED24BITS", o->cfg.need24bits)
        DBL("DITHER_BITS", o->cfg.render.dth_bits, 0.0, 23.0)
        UNS("QUANTIZE_TYPE", o->cfg.render.quantz_type, 0, 1)
        UNS("RENDER_TYPE", o->cfg.render.render_type, 0, 4)
        UNS("NOISE_SHAPING", o->cfg.render.nshape_type, 0, ICW_NSHAPE_MAX)
        UNS("SIGNBITS16", o->cfg.render.sign_bits16, 2, 16)
        UNS("SIGNBITS24", o->cfg.render.sign_bits24, 2, 24)
        (void)ignore_u;
        (void)ignore_b;
    }
#undef UNS
#undef BOOLK
#undef DBL
    if (!strcasecmp(key, "NODE_DSP")) {
        if (o->n_nodes >= ICW_CFG_MAX_NODES) return 0;
        if (icw_node_dsp_parse(args, &o->nodes[o->n_nodes], o->names[o->n_nodes], ICW_DSP_NAME_SIZE) != ICW_OK)
            return 0;
        ++o->n_nodes;
        return 1;
    }
    return 0;                                  /* unknown key: the reference stops here */
}

int icw_config_load(const char *text, size_t len, icw_file_config *out, int *bad_line)
{
    char line[CFG_MAX_LINE + 1];
    size_t i = 0;
    int ln = 0, ok = 1;
    if (!out || (!text && len)) return ICW_EINVAL;
    if (bad_line) *bad_line = 0;
    cfg_defaults(out);
    while (i < len && ok) {
        /* read_conf_line (config.c:307-363): '\r' dropped, tabs -> blanks, overlong -> error */
        size_t cnt = 0;
        int has_graph = 0;
        ++ln;
        while (i < len && text[i] != '\n') {
            char c = text[i++];
            if (c == '\r') continue;
            if (cnt >= CFG_MAX_LINE - 1) { ok = 0; break; }
            line[cnt++] = c == '\t' ? ' ' : c;
        }
        if (!ok) break;
        if (i < len) ++i;                                      /* the '\n' */
        line[cnt] = '\0';
        for (size_t k = 0; k < cnt; ++k) {
            if (iscntrl((unsigned char)line[k])) { ok = 0; break; }
            if (isgraph((unsigned char)line[k])) has_graph = 1;
        }
        if (!ok || !has_graph) continue;
        char *eq = strchr(line, '=');
        if (!eq) { ok = 0; break; }
        *eq = '\0';
        char key[CFG_MAX_KEYW];
        const char *kp = line;
        next_token(&kp, key, sizeof(key));
        ok = cfg_line(out, key, eq + 1);
    }
    if (!ok || out->ver_config != ICW_CFG_VERSION) {
        if (bad_line) *bad_line = ok ? 0 : ln;
        cfg_defaults(out);                                     /* reset_config(FALSE) */
        out->ver_config = ICW_CFG_VERSION;
        return ICW_EINVAL;
    }
    out->cfg.fp_check = out->fp_check;                         /* FP_CHECK -> the device path */
    return ICW_OK;
}
