/*
 * icw_amod.h -- drop-in form of the in_cwave per-block decode boundary, for C hosts.
 *
 * The reference decodes one block per call of
 *     int amod_process_samples(char *buf, MOD_CONTEXT *mc);          in_cwave.h:648,
 *                                                                    adv_modulator.c:587-763
 * called by DecodeThread (playback.c:619, 576-frame blocks) and by
 * winampGetExtendedRead_getData (transcode.c:96, len/out_size frames).  That function first
 * reads the block (xwave_read_samples, xwave_reader.c:838-904) and then runs the DSP on
 * mc->xr->tbuff.  icw_amod keeps the reader where it is (file I/O, virtual zero tail) and
 * replaces the DSP half: the caller passes the raw block it read, the MI355X renders it.
 * INTEGRATION.md shows the 15-line binding in adv_modulator.c / in_cwave.c.
 *
 * One icw_mod_context is one decoding context (the reference's the.mc_playback or
 * the.mc_transcode, in_cwave.h:473-474): a single-stream icw_ctx plus the track bookkeeping.
 * Like MOD_CONTEXT it is driven by one thread at a time.
 */
#ifndef ICW_AMOD_H_
#define ICW_AMOD_H_

#include "icw.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct icw_mod_context icw_mod_context;

/* mod_context_init (in_cwave.c:46-80) + amod_init (adv_modulator.c:216-331).
 * Returns NULL on failure (*status holds the ICW_E* code).  The context is warmed (icw_prepare: one
 * call of silence, then the fresh state back), so the DecodeThread's first block (playback.c:619)
 * costs what the others do. */
icw_mod_context *icw_mod_context_create(const icw_config *cfg, const icw_node *nodes, int n_nodes,
                                        int device, int *status);
void icw_mod_context_destroy(icw_mod_context *mc);

/* mod_context_fopen (in_cwave.c:207-236): a new track with its own sample format.  The Hilbert
 * state and frame counter carry over unless clr_hilb / clr_nframe (is_clr_hilb_trk /
 * is_clr_nframe_trk, default FALSE).  need24bits is the.cfg.need24bits as the track opens
 * (in_cwave.c:212): both renders take that depth (sound_render_set_outbits, :233-234, icw_set_outbits),
 * their shaping state is reset, the RNG is not, and icw_mod_context_out_size follows (4 or 6 bytes
 * per frame, the out_size playback.c:215 / transcode.c:55 size their buffers with). */
int icw_mod_context_fopen(icw_mod_context *mc, uint32_t sample_rate, uint32_t fmt, uint32_t channels,
                          int64_t n_samples, uint32_t fade_in_ms, uint32_t fade_out_ms,
                          uint32_t sec_align, int clr_nframe, int clr_hilb, int need24bits);

/* The DSP half of amod_process_samples: render `n_frames` frames of raw interleaved input
 * (what xwave_read_samples left in xr->tbuff) into `buf` (interleaved L,R, 2 or 3 bytes LE
 * each).  Returns the number of frames rendered, or a negative ICW_E* code -- unlike the
 * reference's overloaded 0, EOF (n_frames == 0 -> 0) and errors are distinguishable. */
int icw_amod_process_samples(char *buf, icw_mod_context *mc, const void *tbuff, unsigned n_frames);

/* xwave_seek_samples (xwave_reader.c:752-785) moved the reader: the fade position follows.
 * Playback also resets the Hilbert converters on seek (playback.c:594): reset_hilb = 1. */
int icw_mod_context_seek(icw_mod_context *mc, int64_t frame_pos, int reset_hilb);

/* sound_render_size(L) + sound_render_size(R): output bytes per frame (4 or 6) at the depth the
 * last icw_mod_context_fopen set (icw_mod_context_create: cfg->need24bits) */
int icw_mod_context_out_size(const icw_mod_context *mc);

/* amod_get_clips_peaks (adv_modulator.c:445-465): reset clears the clips / peaks first and returns
 * the cleared values, as the reference does; the de-subnorm count is kept. */
int icw_mod_context_meters(icw_mod_context *mc, int reset, icw_meters *m);

/* amod_get_clips_peaks (adv_modulator.c:445-465) exactly: the reference keeps ONE set of meters in
 * its `am` singleton (adv_modulator.c:54-55), and every decoding context renders into it
 * (sound_render_value(&buf, lOut, &am.l_clips, &am.l_peak, ...), adv_modulator.c:757-758) -- the
 * playback and the transcode context alike (in_cwave.h:473-474).  Here each context keeps its own;
 * this call combines the n contexts the host decodes with into the reference's one set:
 *   - is_reset != 0 clears every context's clips and peaks FIRST and returns the cleared values
 *     (0 clips, ICW_SR_ZERO_SIGNAL_DB), as the reference clears am before reading it;
 *   - *lc / *rc: the clip counts summed over the contexts (unsigned, wrapping as the reference's
 *     InterlockedIncrement'ed counters wrap);
 *   - *lpv / *rpv: the largest peak in dB over the contexts (each context's samples in dB against
 *     its own render's bound, sound_render.c:769-780: the max over all samples, whichever context).
 * The de-subnorm counters are per context (mod_context_get_desubnorm_counter, in_cwave.c:300-310)
 * and stay with icw_mod_context_meters.  Pass NULL entries to skip a context that is not open. */
int icw_amod_get_clips_peaks(icw_mod_context *const *mcs, int n, unsigned *lc, unsigned *rc, double *lpv,
                             double *rpv, int is_reset);

/* The DSP-list primitives over the decoding contexts: the reference's list is one (am.head, shared
 * by both contexts, adv_modulator.c:51-52), and replace_output_plug clears the removed / re-plugged
 * node's old slot in every context (mod_context_clear_all_inouts, in_cwave.c:255-261).  Each applies
 * the icw.h primitive of the same name to the non-NULL contexts in order and stops at the first error,
 * which it returns.  The contexts hold the same list, so a refused edit (ICW_EGRAPH: amod_init's rules,
 * a Master added) is refused by the first context before any changed.  A device error (ICW_EDEVICE /
 * ICW_ENOMEM) after an earlier context took the edit leaves the contexts with different lists: the
 * host re-sends the whole list to each with icw_set_graph (which matches it by position) before the
 * next block.
 *   icw_amod_del_lastdsp      <- amod_del_lastdsp       (adv_modulator.c:378-390)
 *   icw_amod_del_dsplist      <- amod_del_dsplist       (adv_modulator.c:360-374)
 *   icw_amod_add_lastdsp      <- amod_add_lastdsp + the GUI's field writes (adv_modulator.c:394-411)
 *   icw_amod_set_output_plug  <- amod_set_output_plug   (adv_modulator.c:436-441): list node
 *                                `index` (0 = the Master at the head), slot n or -1 (clear only) */
int icw_amod_del_lastdsp(icw_mod_context *const *mcs, int n);
int icw_amod_del_dsplist(icw_mod_context *const *mcs, int n);
int icw_amod_add_lastdsp(icw_mod_context *const *mcs, int n, const icw_node *node);
int icw_amod_set_output_plug(icw_mod_context *const *mcs, int n, int index, int plug);

/* The context's one-stream icw_ctx, for the live edits of icw.h (icw_set_graph, icw_set_render,
 * icw_set_hilbert_filter / _config): the reference's GUI applies each edit to both decoding
 * contexts, the.mc_playback and the.mc_transcode (in_cwave.c:171-199, 457-469), so a port calls
 * them once per icw_mod_context.  The pointer lives as long as mc. */
icw_ctx *icw_mod_context_ctx(icw_mod_context *mc);

#ifdef __cplusplus
}
#endif
#endif /* ICW_AMOD_H_ */
