/*
 * icw.h -- C ABI of in_cwave_amd: the MI355X-native Hilbert -> modulator-graph -> render
 * hot path of rat-and-catcher/in_cwave (V2.4.4), batched over many independent streams.
 *
 * Plain C types only (no torch, no HIP types).  Every entry point returns an int status:
 * ICW_OK (0) or a negative ICW_E* code -- an improvement over the reference's overloaded 0
 * return of amod_process_samples (adv_modulator.c:601-602), which cannot tell EOF from error.
 *
 * Reference interfaces replaced (file:line into the reference tree):
 *   icw_process_batch / icw_process_block
 *        <- int amod_process_samples(char *buf, MOD_CONTEXT *mc)      in_cwave.h:648,
 *           adv_modulator.c:587-763 (one block: n_frame -> unpack+Hilbert -> graph -> render)
 *   icw_create(cfg, nodes)     <- mod_context_init (in_cwave.c:46-80) + amod_init
 *                                 (adv_modulator.c:216-331: head==Master validation, L/R locks)
 *   icw_stream_open            <- mod_context_fopen (in_cwave.c:207-236) + the fade /
 *                                 sec_align arithmetic of xwave_reader_create
 *                                 (xwave_reader.c:688-725)
 *   icw_stream_reset_hilbert   <- mod_context_reset_hilbert / hq_rp_reset (lpf_hilbert_quad.c:160-165)
 *   icw_stream_reset_framecnt  <- mod_context_reset_framecnt (in_cwave.c:287-296)
 *   icw_get_meters             <- amod_get_clips_peaks (adv_modulator.c:445-465) and
 *                                 mod_context_get_desubnorm_counter (in_cwave.c:300-321)
 *   icw_render_size            <- sound_render_size (sound_render.c:684-687)
 *
 * Threading: a context is driven by one host thread at a time (as MOD_CONTEXT is driven by one
 * decode thread, playback.c:567-671); parameters are snapshotted per call (block granularity,
 * SURVEY 3.4).  Different contexts may be used concurrently from different threads / devices.
 */
#ifndef ICW_H_
#define ICW_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---- */
#define ICW_OK              0
#define ICW_EINVAL         -1   /* bad argument / unsupported configuration */
#define ICW_ENOMEM         -2   /* device or host allocation failed */
#define ICW_EDEVICE        -3   /* HIP runtime error */
#define ICW_EGRAPH         -4   /* DSP list rejected (no unique Master at head, bad plug ...) */
#define ICW_EUNSUPPORTED   -5   /* valid for the reference, not (yet) on this path */

/* ---- constants mirrored from in_cwave.h / sound_render.h / lpf_hilbert_quad.h ---- */
#define ICW_N_INPUTS        27  /* in[0], A[1]..Z[26]             in_cwave.h:244 */
#define ICW_MAX_IIR_ORDER   20  /* largest canned HB LPF order    hblpf.c:740-820 */
#define ICW_MAX_NS_TAPS     20  /* largest noise shaper            sound_render.c:75-235 */
#define ICW_HZ_SCALE        1000u
#define ICW_MAX_FS_SRC      2000000u

/* node modes (NODE_DSP.mode, in_cwave.h:283-287) */
#define ICW_MODE_MASTER 0
#define ICW_MODE_SHIFT  1
#define ICW_MODE_PM     2
#define ICW_MODE_MIX    3
/* master output conversions (in_cwave.h:152-155) */
#define ICW_S_ADD_REIM  0
#define ICW_S_SUB_REIM  1
#define ICW_S_RE        2
#define ICW_S_IM        3
/* channel exchange (in_cwave.h:186-193) */
#define ICW_XCH_NORMAL    0
#define ICW_XCH_SWAP      1
#define ICW_XCH_LEFTONLY  2
#define ICW_XCH_RIGHTONLY 3
#define ICW_XCH_MIXLR     4
/* real (RWAVE/WAV) input sample formats (HRW_FMT_*, in_cwave.h:318-323) */
#define ICW_FMT_U8   0
#define ICW_FMT_I16  1
#define ICW_FMT_I24  2
#define ICW_FMT_I32  3
#define ICW_FMT_F32  4
/* complex (CWAVE) input sample formats, ICW_FMT_CW_F64 + HCW_FMT_* (cwave.h:70-80).  The analytic
 * signal is used as read: the Hilbert converters are bypassed and keep their state, fades scale
 * I and Q alike (xwave_unpack_csample, xwave_reader.c:939-966); mono feeds R with L's I/Q. */
#define ICW_FMT_CW_F64      5     /* double Re, Im           HCW_FMT_PCM_DBL64 */
#define ICW_FMT_CW_I16      6     /* int16 Re, Im            HCW_FMT_PCM_INT16 */
#define ICW_FMT_CW_I16_F32  7     /* int16 Re, float Im      HCW_FMT_PCM_INT16_FLT32 */
#define ICW_FMT_CW_F32      8     /* float Re, Im            HCW_FMT_PCM_FLT32 */
/* render (sound_render.h:54-84) */
#define ICW_QUANTZ_MID_TREAD 0
#define ICW_QUANTZ_MID_RISER 1
#define ICW_RENDER_ROUND 0
#define ICW_RENDER_RPDF  1
#define ICW_RENDER_TPDF  2
#define ICW_RENDER_STPDF 3
#define ICW_RENDER_GAUSS 4
#define ICW_NSHAPE_FLAT  0
#define ICW_NSHAPE_MEW44 2
#define ICW_NSHAPE_MAX   17
/* default render seeds (in_cwave.c:69-70) */
#define ICW_SEED_LEFT   0x13579BDFu
#define ICW_SEED_RIGHT  0x479B22ABu
#define ICW_SR_ZERO_SIGNAL_DB (-555.0)

/* One DSP node (NODE_DSP, in_cwave.h:273-287, without list links / name).  Channel arrays are
 * [0]=left, [1]=right.  The list is passed head first: nodes[0] must be the Master. */
typedef struct icw_node {
    int32_t  mode;                    /* ICW_MODE_* */
    int32_t  n_out;                   /* output bus slot 1..26 (SHIFT/PM/MIX) */
    double   gain[2];                 /* l_gain / r_gain */
    uint8_t  inputs[ICW_N_INPUTS];    /* bus slots mixed into the node */
    uint8_t  pad_[1];
    int32_t  xch_mode;                /* ICW_XCH_* */
    int32_t  iq_invert[2];            /* l_iq_invert / r_iq_invert */
    int32_t  tout[2];                 /* MASTER: ICW_S_* */
    double   fr_shift[2];             /* SHIFT: signed shift, Hz */
    int32_t  is_shift[2];
    double   pm_freq[2], pm_phase[2], pm_level[2], pm_angle[2];   /* PM */
    int32_t  is_pm[2];
    /* L/R locks applied at icw_create exactly as amod_init does (adv_modulator.c:247-293) */
    int32_t  lock_gain, lock_shift, sign_lock_shift;
    int32_t  lock_freq, lock_phase, lock_level, lock_angle;
    int32_t  reserved_;
} icw_node;

/* SR_VCONFIG (sound_render.h:145-153) */
typedef struct icw_render_cfg {
    double   dth_bits;
    uint32_t quantz_type, render_type, nshape_type, sign_bits16, sign_bits24;
} icw_render_cfg;

/* Context-wide configuration (IN_CWAVE_CFG hot-path fields, in_cwave.h:435-459) */
typedef struct icw_config {
    uint32_t sample_rate;         /* Hz, <= ICW_MAX_FS_SRC */
    uint32_t in_format;           /* ICW_FMT_* */
    uint32_t in_channels;         /* 1 (mono: R fed with L) or >= 2 (channels > 2 skipped) */
    uint32_t hilbert_type;        /* IX_LPF_HILB_TYPE0..5 (default 1) */
    int32_t  iir_kahan;           /* IIR_SUM_KAHAN (default 1) */
    int32_t  iir_subnorm_reject;  /* IIR_SUBN_ZERO (default 1) */
    int32_t  frmod_scaled;        /* FRMOD_SCALED (default 1) */
    int32_t  need24bits;          /* NEED24BITS */
    int32_t  bypass_list;         /* am.is_bypass_list */
    uint32_t seed_left, seed_right;
    icw_render_cfg render;
    int32_t  fp_check;            /* FP_CHECK (default 0): the FC() arithmetic and census of
                                     fp_check.c:52-100 in the IIR (hblpf.c:928-950, 1058-1095) and
                                     the render (sound_render.c:403-489, 815-903); icw_get_fp_census */
} icw_config;

/* Per-stream meters.  The reference keeps one set, global in `am` (adv_modulator.c:54-56), that
 * both decoding contexts feed (adv_modulator.c:757-758); icw_amod_get_clips_peaks (icw_amod.h)
 * combines the per-context meters into it: clips summed, peaks maxed, a reset clearing all. */
typedef struct icw_meters {
    uint32_t clips[2];            /* InterlockedIncrement'ed clip counters, sound_render.c:782-795 */
    double   peak_db[2];          /* max 20*log10(|q|/hi_bound), SR_ZERO_SIGNAL_DB if silent */
    uint64_t desubnorm;           /* sum of the 4 IIR subnorm_cnt of the stream, hblpf.c:918/1049 */
} icw_meters;

typedef struct icw_ctx icw_ctx;

/* flags for icw_process_batch */
#define ICW_F_DEVICE_PTRS  1u     /* in/out are device pointers already resident in HBM */
#define ICW_F_DEBUG_PRE    2u     /* also write the 2 pre-render doubles/frame to dbg (tests) */
#define ICW_F_TIMING       4u     /* time the kernels with HIP events (icw_last_timing) */
#define ICW_F_DEBUG_INPUT  8u     /* tests: write the unpacked, faded samples the Hilbert converters get
                                     (what xwave_unpack_csample hands hq_rp_process, xwave_reader.c:
                                     974-998; R = L for mono) to dbg as double[n_streams][n_frames][2]:
                                     real input through the quadrature IIR, host pointers only */

/* Create a context for n_streams streams on HIP device `device` (-1: current device).
 * The DSP list is normalised exactly as amod_init (adv_modulator.c:216-331) does; a list it
 * would reject (no Master at head, 2 Masters, bad mode) is replaced by the default Master
 * (S_ADD_REIM, gain 0.8, input `in`) and *accepted is set to 0, like amod_init's return. */
int icw_create(const icw_config *cfg, const icw_node *nodes, int n_nodes, int n_streams,
               int device, icw_ctx **out, int *accepted);
int icw_destroy(icw_ctx *ctx);

/* Fresh reference state for streams [first, first+count): Hilbert rings zeroed, n_frame=0,
 * bus zeroed, renders re-seeded (mod_context_init, in_cwave.c:46-80). */
int icw_stream_init(icw_ctx *ctx, int first, int count);
/* Open a track on stream s (mod_context_fopen): track length in frames, fades in ms,
 * sec_align in s.  Resets the renders' shaping state (sound_render_set_outbits), not the RNG;
 * clears n_frame / Hilbert only if the flags say so (is_clr_nframe_trk / is_clr_hilb_trk). */
int icw_stream_open(icw_ctx *ctx, int s, int64_t n_samples, uint32_t fade_in_ms,
                    uint32_t fade_out_ms, uint32_t sec_align, int clr_nframe, int clr_hilb);
int icw_stream_reset_hilbert(icw_ctx *ctx, int s);
int icw_stream_reset_framecnt(icw_ctx *ctx, int s);
/* reader seek (xwave_seek_samples, xwave_reader.c:752-785): frame position inside the track,
 * virtual tail included, from which fades are evaluated */
int icw_stream_seek(icw_ctx *ctx, int s, int64_t frame_pos);
/* input format of the next blocks (a new track, mod_context_fopen): sample rate, ICW_FMT_*,
 * channels; applies to every stream of the context */
int icw_set_input(icw_ctx *ctx, uint32_t sample_rate, uint32_t fmt, uint32_t channels);

/* Live parameter changes (the GUI thread edits the DSP list, the renders and the
 * Hilbert converters while a decode thread runs).  Each applies to every stream of the context from
 * the next call on; a call already queued finishes with the old parameters.  Per-stream state
 * (bus slots, rings, MT19937, meters) carries over exactly as the reference carries it.
 *
 * icw_set_graph   <- amod_add_lastdsp / amod_del_lastdsp / amod_del_dsplist
 *                    (adv_modulator.c:358-400), the node-field writes of the GUI
 *                    (amod_gui_control.c:259-420, 1433-1482) and amod_set_bypass_list_flag
 *                    (adv_modulator.c:422-425): the whole new list, head first, normalised as
 *                    icw_create does (locks fanned out).  A list amod_init would reject (no Master
 *                    at the head, two Masters, unknown mode) returns ICW_EGRAPH with *accepted = 0
 *                    and leaves the running list in place.  The 27-slot bus keeps its values,
 *                    except the slots the reference clears: amod_del_lastdsp, amod_del_dsplist and
 *                    amod_set_output_plug go through replace_output_plug (adv_modulator.c:176-209),
 *                    which zeroes the removed / re-plugged node's old output slot in every context
 *                    (mod_context_clear_all_inouts, in_cwave.c:255-261).  The new list is matched to
 *                    the old one by position: an old Shift / PM / Mix node whose position is gone,
 *                    now holds a node of another mode, or whose n_out changed has its old slot
 *                    zeroed for every stream.  Edits that position matching cannot see (a re-plug to
 *                    the same slot, delete + add of an identical node) are the list primitives below:
 *                    a host that binds the GUI forwards each primitive as it happens, not a diff.
 * icw_clear_bus_slot <- mod_context_clear_all_inouts (in_cwave.c:255-261): bus slot 0..26 of
 *                    every stream to zero (the 4 doubles L re/im, R re/im).
 * icw_set_render  <- srenders_set_vcfg (in_cwave.c:457-469) -> sound_render_setup
 *                    (sound_render.c:625-629): the new SR_VCONFIG for both renders of every
 *                    stream; sound_render_recalc restarts prev_rnd, the shaper rings and
 *                    prev_ns_err, the MT19937 generators go on.  16/24 bits stay (need24bits;
 *                    a new track's depth is icw_set_outbits below).
 * icw_set_hilbert_filter <- mod_context_change_all_hilberts_filter (in_cwave.c:186-199): a
 *                    different type re-creates every converter (hq_rp_create: zero rings, phase 0,
 *                    de-subnorm counters 0); the same type changes nothing.  type 0..5.
 * icw_set_hilbert_config <- mod_context_change_all_hilberts_config (in_cwave.c:171-182) ->
 *                    iir_rp_setcfg (hblpf.c:1117-1127): Kahan / baseline summation and the
 *                    subnormal reject; the rings stay, the de-subnorm counters restart. */
int icw_set_graph(icw_ctx *ctx, const icw_node *nodes, int n_nodes, int bypass_list, int *accepted);
int icw_clear_bus_slot(icw_ctx *ctx, int slot);

/* The list primitives one by one, each with exactly the reference's bus clearing -- no position
 * matching.  replace_output_plug (adv_modulator.c:176-209) clears a Shift / PM / Mix node's OLD
 * output slot in every stream, also when it is re-plugged to the same slot; a Master clears nothing.
 *   icw_graph_del_last      <- amod_del_lastdsp (adv_modulator.c:378-390): the tail node goes and
 *                              its slot is cleared; a list of the Master alone is left as it is.
 *   icw_graph_del_all       <- amod_del_dsplist (adv_modulator.c:360-374): tail first, down to the
 *                              Master, each removed node's slot cleared.
 *   icw_graph_add_last      <- amod_add_lastdsp (adv_modulator.c:394-411) followed by the GUI's
 *                              field writes of the new node (amod_gui_control.c:1858): `node` is
 *                              appended after the tail, its L/R locks fanned out as amod_init does;
 *                              nothing is cleared.  A Master is refused (create_node_dsp, :112-123):
 *                              ICW_EGRAPH.
 *   icw_graph_set_output_plug <- amod_set_output_plug (adv_modulator.c:436-441, the GUI's plug
 *                              selector amod_gui_control.c:1125): node `index` (0 = the head) gets
 *                              output slot n (1..26), or keeps its slot with n = -1 ("remove only");
 *                              either way its old slot is cleared.
 * The field writes of existing nodes (gains, frequencies, inputs, locks) and the bypass flag clear
 * nothing: icw_set_graph with the same structure. */
int icw_graph_del_last(icw_ctx *ctx);
int icw_graph_del_all(icw_ctx *ctx);
int icw_graph_add_last(icw_ctx *ctx, const icw_node *node);
int icw_graph_set_output_plug(icw_ctx *ctx, int index, int n);
int icw_set_render(icw_ctx *ctx, const icw_render_cfg *render);
/* icw_set_outbits <- sound_render_set_outbits (sound_render.c:617-621), which mod_context_fopen
 *                    applies to both renders with the.cfg.need24bits at every track open
 *                    (in_cwave.c:212, 233-234; the GUI flips the flag between tracks,
 *                    amod_gui_control.c:1641): 16 (0) or 24 (!= 0) output bits for every stream of
 *                    the context.  New bounds, norm_mul and norm_shift, then sound_render_recalc:
 *                    prev_rnd, the shaper rings and prev_ns_err restart (also at an unchanged
 *                    depth), the MT19937 generators go on.  The peaks so far are kept in dB against
 *                    the old bound; icw_render_size follows the new depth. */
int icw_set_outbits(icw_ctx *ctx, int need24bits);
int icw_set_hilbert_filter(icw_ctx *ctx, uint32_t type);
int icw_set_hilbert_config(icw_ctx *ctx, int kahan, int subnorm_reject);

/* FIR Hilbert converter: the converter that CWAVE files record in their header (cwave.h:40,56-58:
 * "Hilbert FIR filter order" k_M, "Hilbert FIR filter parameter" k_beta; gui_cwave.c:159-172 shows
 * them; the converter program is not part of in_cwave).  With k_M > 0, real input is turned on the
 * device into the analytic signal such a file would hold -- a Kaiser-windowed (beta = k_beta)
 * Hilbert FIR of order k_M, odd taps m only, delay k_M/2:
 *     I[n] = x[n - k_M/2],  Q[n] = sum_{m odd <= k_M/2} g_m (x[n - k_M/2 - m] - x[n - k_M/2 + m]),
 *     g_m = 2 I0(beta sqrt(1 - (2m/k_M)^2)) / (pi m I0(beta)),  summed in ascending m with an FMA
 * per tap -- and the block continues as CWAVE input does (no quadrature IIR; graph and render as
 * for complex samples).  k_M = 0 restores the reference's own quadrature IIR Hilbert (the default).
 * k_M even, 2..ICW_FIR_MAX_ORDER.  Every stream's FIR history (its last k_M inputs) starts at zero;
 * icw_stream_init / icw_stream_reset_hilbert / icw_stream_open(clr_hilb) clear it too.
 * No reference implementation exists for this stage: its parity is unpinned. */
#define ICW_FIR_MAX_ORDER 4096
int icw_set_fir_hilbert(icw_ctx *ctx, int32_t k_M, double k_beta);
/* The taps of that design: g[k] = g_{2k+1}, k < nt = (k_M/2 + 1)/2.  Returns nt (or ICW_EINVAL). */
int icw_fir_taps(int32_t k_M, double k_beta, double *g, int n);

/* Process n_frames frames of every stream (the batched amod_process_samples).
 *   in  : stream s starts at (char*)in  + s*in_stride_bytes,  frames interleaved by channel
 *         in cfg->in_format (what xwave_read_samples leaves in xr->tbuff).
 *   out : stream s starts at (char*)out + s*out_stride_bytes, interleaved L,R, 2 or 3 bytes LE.
 *   dbg : ICW_F_DEBUG_PRE only -- double[n_streams][n_frames][2] pre-render values (lOut,rOut).
 * Host pointers are staged through pinned buffers; host buffers that are pinned themselves
 * (icw_host_alloc, hipHostMalloc, hipHostRegister) are copied block by block on a copy stream,
 * beside the kernels of the other launch blocks.  With ICW_F_DEVICE_PTRS nothing crosses PCIe.  hip_stream: the hipStream_t the call is ordered on (it starts after the work queued there,
 * and the stream's later work sees its results; the call returns before the kernels finish).
 * NULL: with host pointers the context's own stream (the call returns when its output is in
 * `out`); with ICW_F_DEVICE_PTRS the legacy default stream (stream 0, torch's default stream): the
 * call starts after the work queued there and returns when its output is in place.
 * icw_get_meters / icw_n_frame / icw_get_state wait for the context's work.  Returns ICW_OK. */
int icw_process_batch(icw_ctx *ctx, const void *in, size_t in_stride_bytes, void *out,
                      size_t out_stride_bytes, int n_frames, unsigned flags, void *dbg,
                      void *hip_stream);
/* Same for a subset of streams [first, first+count) (e.g. one decode thread's stream). */
int icw_process_streams(icw_ctx *ctx, int first, int count, const void *in,
                        size_t in_stride_bytes, void *out, size_t out_stride_bytes,
                        int n_frames, unsigned flags, void *dbg, void *hip_stream);

/* Warm a FRESH context (no call made yet) for calls of up to n_frames frames per stream (0: 4096,
 * the longest one-launch call of one stream): one call of silence through the path its
 * configuration takes, then the fresh state back (icw_stream_init).  The pinned staging, the device
 * buffers and the lazily loaded kernel code objects are then in place, so the first real call costs
 * what the later ones do -- the DecodeThread's first block (playback.c:619) included.
 * icw_mod_context_create calls it.  ICW_EINVAL once a call has been made, or once per-stream state
 * was set another way (icw_stream_open, _seek, _reset_hilbert, _reset_framecnt, icw_set_state), since
 * the closing icw_stream_init would wipe it.  Context-wide settings (icw_set_input, _set_graph,
 * _set_render, _set_outbits, the Hilbert setters) may come first: the warm-up runs with them. */
int icw_prepare(icw_ctx *ctx, int n_frames);

int icw_synchronize(icw_ctx *ctx);
/* Pinned (page-locked) host memory for a call's in / out buffers: their copies then overlap the
 * kernels (cudaMallocHost-style helper; the reference's buffers are the caller's own).  0 / ICW_ENOMEM. */
int icw_host_alloc(size_t bytes, void **p);
int icw_host_free(void *p);
/* Whether a host buffer takes the block-by-block copies on a context of `device`: 1 when it is
 * page-locked and was pinned while `device` was current or pinned portable (icw_host_alloc,
 * hipHostMallocPortable, hipHostRegisterPortable), 0 otherwise (the call then stages it through the
 * context's own pinned buffers: correct for any host memory, without the overlap). */
int icw_host_pinned(const void *p, int device);
/* Meters of stream s (amod_get_clips_peaks, adv_modulator.c:445-465).  reset != 0 clears the clip
 * counters and peaks FIRST, as the reference does, so the call returns 0 clips and
 * ICW_SR_ZERO_SIGNAL_DB peaks; the de-subnorm count is not reset (mod_context_get_desubnorm_counter,
 * in_cwave.c:300-310).  Waits for the context's running work. */
int icw_get_meters(icw_ctx *ctx, int s, int reset, icw_meters *m);
int icw_render_size(const icw_ctx *ctx);     /* bytes per output channel-sample: 2 or 3 */
int icw_n_frame(icw_ctx *ctx, int s, uint64_t *n_frame);

/* Serialisable per-stream state (checkpoint / resume).  Canonical layout documented
 * in DESIGN.md: IIR histories most-recent-first, Hilbert phases, n_frame, bus, render state. */
size_t icw_state_size(const icw_ctx *ctx);
int icw_get_state(icw_ctx *ctx, int s, void *blob, size_t size);
int icw_set_state(icw_ctx *ctx, int s, const void *blob, size_t size);

/* Kernel timing of the last icw_process_* call, measured with HIP events on the stream the
 * kernels ran on (bench.py roofline).  ms[0] = IIR state kernel total, ms[1] = output kernel
 * total, launches[0..1] = launch counts. */
int icw_last_timing(icw_ctx *ctx, double ms[2], int launches[2]);

/* IIR state kernel (the serial recurrence) the last real-input icw_process_* call ran: ICW_K1_*.
 * The host picks the row-broadcast kernel for small batches (its waves fit two per CU on half
 * the chip, Kahan sum with the reject) and the lane-per-chain kernel otherwise;
 * ICW_K1_MODE=plain|row in the environment at icw_create forces one (A/B runs).  Codes 1 and 2
 * named two archived experiments (tools/k1_experimental.hip) and are no longer returned. */
#define ICW_K1_LANE   0   /* icw_iir_state: one lane per DF-II chain */
#define ICW_K1_ROW    3   /* icw_iir_row: one 16-lane DPP row per chain */
#define ICW_K1_FC     4   /* icw_iir_state_fc: FP_CHECK (cfg.fp_check) arithmetic and census */
int icw_last_k1_kernel(const icw_ctx *ctx);

/* FP-exception census of stream s (FP_EXCEPT_STATS, fp_check.h:62-72) when cfg.fp_check is set:
 * counts[0] Hilbert left (mc->fes_hilb_left), [1] Hilbert right, [2] render left (fes_sr_left),
 * [3] render right; each {total, snan, qnan, ninf, nden, pden, pinf}.  reset != 0 clears them
 * afterwards (except_stats_reset, fp_check.c:36-48). */
#define ICW_FES_N 7
int icw_get_fp_census(icw_ctx *ctx, int s, int reset, uint32_t counts[4][ICW_FES_N]);

const char *icw_version(void);
const char *icw_strerror(int status);

/* The C ABI's version, for bindings to check at load time against the header they were built with.
 *   1  rounds 1-4;
 *   2  icw_mod_context_fopen takes need24bits (its 11th argument, in_cwave.c:212) -- a binding built
 *      against version 1 would pass an undefined bit depth. */
#define ICW_ABI_VERSION 2
int icw_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* ICW_H_ */
