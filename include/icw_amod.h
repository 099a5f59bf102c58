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
 * Returns NULL on failure (*status holds the ICW_E* code). */
icw_mod_context *icw_mod_context_create(const icw_config *cfg, const icw_node *nodes, int n_nodes,
                                        int device, int *status);
void icw_mod_context_destroy(icw_mod_context *mc);

/* mod_context_fopen (in_cwave.c:207-236): a new track with its own sample format.  The Hilbert
 * state and frame counter carry over unless clr_hilb / clr_nframe (is_clr_hilb_trk /
 * is_clr_nframe_trk, default FALSE); the renders' shaping state is reset, the RNG is not. */
int icw_mod_context_fopen(icw_mod_context *mc, uint32_t sample_rate, uint32_t fmt, uint32_t channels,
                          int64_t n_samples, uint32_t fade_in_ms, uint32_t fade_out_ms,
                          uint32_t sec_align, int clr_nframe, int clr_hilb);

/* The DSP half of amod_process_samples: render `n_frames` frames of raw interleaved input
 * (what xwave_read_samples left in xr->tbuff) into `buf` (interleaved L,R, 2 or 3 bytes LE
 * each).  Returns the number of frames rendered, or a negative ICW_E* code -- unlike the
 * reference's overloaded 0, EOF (n_frames == 0 -> 0) and errors are distinguishable. */
int icw_amod_process_samples(char *buf, icw_mod_context *mc, const void *tbuff, unsigned n_frames);

/* xwave_seek_samples (xwave_reader.c:752-785) moved the reader: the fade position follows.
 * Playback also resets the Hilbert converters on seek (playback.c:594): reset_hilb = 1. */
int icw_mod_context_seek(icw_mod_context *mc, int64_t frame_pos, int reset_hilb);

/* sound_render_size(L) + sound_render_size(R): output bytes per frame (4 or 6) */
int icw_mod_context_out_size(const icw_mod_context *mc);

/* amod_get_clips_peaks (adv_modulator.c:445-465): reset clears the clips / peaks first and returns
 * the cleared values, as the reference does; the de-subnorm count is kept. */
int icw_mod_context_meters(icw_mod_context *mc, int reset, icw_meters *m);

/* The context's one-stream icw_ctx, for the live edits of icw.h (icw_set_graph, icw_set_render,
 * icw_set_hilbert_filter / _config): the reference's GUI applies each edit to both decoding
 * contexts, the.mc_playback and the.mc_transcode (in_cwave.c:171-199, 457-469), so a port calls
 * them once per icw_mod_context.  The pointer lives as long as mc. */
icw_ctx *icw_mod_context_ctx(icw_mod_context *mc);

#ifdef __cplusplus
}
#endif
#endif /* ICW_AMOD_H_ */
