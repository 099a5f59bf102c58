/*
 * icw_config.h -- ingestion of the reference's configuration file (in_cwave.cfg): the hot-path
 * keys and the NODE_DSP= lines that define the DSP list, so a reference user's saved graph and
 * render settings drive icw_create unchanged.
 *
 * Reference interfaces replaced (file:line into the reference tree):
 *   icw_config_load     <- load_config (config.c:813-915) with read_conf_line (config.c:307-363),
 *                          handle_string / _bool / _int / _unsigned / _double (config.c:380-541) and
 *                          the config_list keys and bounds (config.c:113-296)
 *   icw_node_dsp_parse  <- handle_node_dsp, read side (config.c:663-774)
 *   icw_node_dsp_format <- handle_node_dsp, write side (config.c:565-652) + write_conf_line
 * Host-only text processing: no device is touched.
 */
#ifndef ICW_CONFIG_H_
#define ICW_CONFIG_H_

#include "icw.h"

#ifdef __cplusplus
extern "C" {
#endif

#define ICW_CFG_VERSION     10u      /* VERSION_CONFIG, config.c:50 */
#define ICW_CFG_MAX_NODES   64
#define ICW_DSP_NAME_SIZE   96       /* SIZE_DSP_NAME = MAX_DSP_NAME + 16 (in_cwave.h:199-200) */

/* The configuration a file defines.  cfg.sample_rate / in_format / in_channels are per track and
 * left at the values passed in; every other field is set from the file or its default. */
typedef struct icw_file_config {
    icw_config cfg;
    uint32_t sec_align, fade_in, fade_out;       /* SEC_ALIGN, FADE_IN, FADE_OUT */
    int32_t  clr_nframe, clr_hilb;               /* CLR_NFRAME_PT, CLR_HILB_PT */
    double   subnorm_thr;                        /* IIR_SUBN_THR: read and bounded, unused on the
                                                    path (the reject compares with 1.0, hblpf.c:1046) */
    int32_t  fp_check;                           /* FP_CHECK (also copied to cfg.fp_check) */
    uint32_t ver_config;                         /* VER_CONFIG */
    int32_t  n_nodes;                            /* NODE_DSP lines in file order = list head first */
    icw_node nodes[ICW_CFG_MAX_NODES];
    char     names[ICW_CFG_MAX_NODES][ICW_DSP_NAME_SIZE];
} icw_file_config;

/* load_config on a file image of `len` bytes: defaults first, then the lines in order up to the
 * first bad one.  A bad line, an unknown key, a wrong VER_CONFIG or more than ICW_CFG_MAX_NODES
 * nodes reset everything to the defaults (reset_config(FALSE)) and return ICW_EINVAL -- the
 * reference then runs with defaults and an empty DSP list (amod_init falls back to the default
 * Master).  *bad_line (nullable) gets the 1-based line that failed, 0 if none.  `out->cfg`'s
 * sample_rate / in_format / in_channels are kept as the caller set them. */
int icw_config_load(const char *text, size_t len, icw_file_config *out, int *bad_line);

/* The arguments of one NODE_DSP= line (after the '='): name, gains, lock, 27 inputs, channel
 * exchange, I/Q swaps, mode and the mode's parameters, out-of-range values clamped exactly as
 * HANDLE_CHK does.  name (nullable) receives the unescaped node name. */
int icw_node_dsp_parse(const char *args, icw_node *node, char *name, size_t name_size);

/* The NODE_DSP= line save_config would write for a node (doubles as 0x<16 hex digits>, names with
 * '%' escapes), NUL-terminated, without a newline.  Returns the length or a negative ICW_E*. */
int icw_node_dsp_format(const icw_node *node, const char *name, char *buf, size_t size);

#ifdef __cplusplus
}
#endif
#endif /* ICW_CONFIG_H_ */
