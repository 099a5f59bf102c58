/*
 * icw_ref_bind.h -- reference-side binding helpers: the glue a maintainer adds to the in_cwave
 * tree (next to in_cwave.c) to drive libicw from the reference's own configuration and reader
 * objects.  Compiled inside the reference tree only: it includes "in_cwave.h", which needs the
 * Win32 headers, so it is not built in this repository.
 *
 * What each helper maps (file:line into the reference tree):
 *   icw_config_from_ref  IN_CWAVE_CFG (in_cwave.h:435-459): iir_filter_no, iir_comp_config
 *                        (IIR_COMP_CONFIG, hblpf.h:130-135), is_frmod_scaled, need24bits,
 *                        sr_config (SR_VCONFIG, sound_render.h:142-150), is_fp_check; the render
 *                        seeds of mod_context_init (in_cwave.c:67-70); am.is_bypass_list
 *                        (adv_modulator.c:56, amod_get_bypass_list_flag in_cwave.h:624)
 *   icw_nodes_from_ref   a NODE_DSP list (in_cwave.h:273-287, MAKE_* :207-269), head first along
 *                        ->next, as amod_init walks it (adv_modulator.c:231-296)
 *   icw_node_from_ref    one NODE_DSP; icw_node_index its list position along ->prev
 *   icw_fmt_from_reader  XWAVE_READER (in_cwave.h:375-405): type, spec.rwave.format (HRW_FMT_*,
 *                        :324-330) or spec.cwave.header.format (HCW_FMT_*, cwave.h:70-80)
 *   cfg_to_icw           the two above in one call, as INTEGRATION.md 1 uses it
 */
#ifndef ICW_REF_BIND_H_
#define ICW_REF_BIND_H_

#include "in_cwave.h"
#include "icw.h"
#include "icw_config.h"

/* icw_config for a track of sample_rate / fmt (ICW_FMT_*) / channels; returns ICW_OK */
int icw_config_from_ref(const IN_CWAVE_CFG *cfg, BOOL bypass_list, unsigned sample_rate,
                        unsigned fmt, unsigned channels, icw_config *out);

/* Copies up to max_nodes nodes of the list starting at head; returns the node count or
 * ICW_EINVAL if the list is longer.  Locks are copied, not applied: icw_create applies them
 * exactly as amod_init does. */
int icw_nodes_from_ref(const NODE_DSP *head, icw_node *nodes, int max_nodes);

/* One node (for icw_graph_add_last / icw_amod_add_lastdsp after amod_add_lastdsp and the GUI's
 * field writes), and a node's position in its list along ->prev (0 = the head), for
 * icw_amod_set_output_plug (amod_set_output_plug takes the node itself, adv_modulator.c:436-441) */
void icw_node_from_ref(const NODE_DSP *nd, icw_node *out);
int icw_node_index(const NODE_DSP *nd);

/* ICW_FMT_* of an open reader, or ICW_EINVAL for a format libicw does not take */
int icw_fmt_from_reader(const XWAVE_READER *xr);

/* the.cfg (before amod_init takes the.cfg.dsp_list) -> icw_config + icw_node[ICW_CFG_MAX_NODES];
 * the track format fields are set by icw_mod_context_fopen later.  Returns the node count. */
int cfg_to_icw(const IN_CWAVE_CFG *cfg, icw_config *c, icw_node nodes[ICW_CFG_MAX_NODES]);

#endif /* ICW_REF_BIND_H_ */
