/*
 * icw_device.h -- data structures shared by the host orchestration (icw_host.cpp) and the
 * gfx950 kernels (icw_kernels.hip).  Plain structs passed by value as kernel arguments or
 * placed in device memory; no HIP types.
 */
#ifndef ICW_DEVICE_H_
#define ICW_DEVICE_H_

#include <stddef.h>
#include <stdint.h>

#define ICW_MAX_OPS   64     /* DSP ops (nodes) per graph on the device path */
#define ICW_MAX_REG_OPS 16   /* ops of a graph the frame-parallel register program accepts */
#define ICW_MAX_REGS  8      /* value registers: `in`, node outputs, persistent slots */
#define ICW_K2_TILE   256    /* frames per output-kernel tile (= workgroup size) */
#define ICW_K2_TPW    4      /* consecutive tiles per output-kernel workgroup */
#define ICW_HIST_PITCH 20    /* doubles per chain in the delay-line state */
#define ICW_RSTATE    42     /* doubles of render state per channel: prev_rnd, prev_ns_err, E[20], O[20] */
#define ICW_FES_PITCH 8      /* u32 per FP-exception census (7 used: FP_EXCEPT_STATS, fp_check.h:62-72) */

struct IcwProg;

/* Arguments of the input prep kernel (one thread = one frame). */
struct IcwK0Args {
    uint32_t lds_guard;            /* dynamic LDS bytes: > 0 keeps the launch off the CUs K1 holds */
    const unsigned char *in;       /* stream s at in + s*in_stride */
    size_t in_stride;
    uint32_t fmt, csz, fsz, nch;   /* sample format, channel/frame bytes, channels */
    int32_t n_streams, T;
    long long t0;                  /* block offset into the call */
    const long long *pos;          /* [n_streams] reader position at the call's start */
    const long long *fade;         /* [n_streams][3] n_samples, n_fade_in, n_fade_out */
    const uint32_t *hq_phase;      /* [n_streams][2] Hilbert phase at the call's start */
    int32_t dedup;                 /* mono dedup: the right chains' rows are not needed */
    double *xd;                    /* [n_chains][x_pitch]: each chain's own filter input sequence;
                                      complex input: rows s*4 + ch*2 + {0: I, 1: Q} hold the samples */
    size_t x_pitch;
};

/* Arguments of the FIR Hilbert converter kernels (KF / KF2, the CWAVE converter of cwave.h:40,56-58:
 * a Kaiser-windowed Hilbert FIR of order M = k_M, window parameter k_beta).  A workgroup stages the
 * inputs x[t - M .. t + tile) of its channels (unpacked and faded like K0, the M before the block
 * from the history) in LDS and forms the analytic signal I = x[n - M/2],
 * Q = sum_m g_m (x[n - M/2 - m] - x[n - M/2 + m]); KF writes it to the complex rows K2 reads for
 * CWAVE input, KF2 takes it through the graph and render itself. */
#define ICW_FIR_MAX_M  4096   /* largest FIR order */
struct IcwFirArgs {
    const unsigned char *in;       /* stream s at in + s*in_stride */
    size_t in_stride;
    uint32_t fmt, csz, fsz, nch;   /* real sample format, channel/frame bytes, file channels */
    int32_t n_streams, T;
    long long t0;                  /* block offset into the call */
    const long long *pos;          /* [n_streams] reader position at the call's start */
    const long long *fade;         /* [n_streams][3] n_samples, n_fade_in, n_fade_out */
    int32_t M, nt;                 /* order (even), odd taps m = 1, 3, .., 2nt-1 <= M/2 */
    const double *g;               /* [nt] g_m = 2 w(m) / (pi m) */
    const double *hist_in;         /* [n_streams][2][M] the channel's last M inputs, oldest first */
    double *hist_out;              /* the same after this block (the other buffer) */
    double *xd;                    /* [n_streams*4][x_pitch] rows s*4 + ch*2 + {0: I, 1: Q} */
    size_t x_pitch;
    int32_t zero;                  /* always 0: keeps the lane's 4 output strides opaque (no LDS read pairing) */
    int32_t sig;                   /* KF2: the program's chain signature (IcwProg.sig; 0: not a chain), so the
                                      launcher can pick the signature form (icw_fir_sig) */
    int32_t tile0;                 /* KF2: index of the first tile icw_fir_graph's grid covers (set by the launcher) */
    int32_t lr_same;               /* KF2, mono input: a Master-only chain whose two gains are the same double, so
                                      both output channels are one computation (icw_fir_sig) */
};

/* Arguments of the call-end bookkeeping kernel: one thread per stream.  During a call every
 * kernel reads the call-start position / phases / frame counter and adds its block offset; this
 * kernel advances them once, after the last block. */
struct IcwAdvArgs {
    uint32_t lds_guard;            /* dynamic LDS bytes: > 0 keeps the launch off the CUs K1 holds */
    int32_t n_streams, cw;
    long long n;                   /* frames processed by the call */
    uint32_t *hq_phase;
    long long *pos;
    unsigned long long *n_frame;
    unsigned long long ssr;
    int32_t scaled;
    const int *err;                /* with err_copy: the hand-off flag is copied next to the output, */
    int *err_copy;                 /* so a small host-pointer call reads both with one copy */
    uint32_t *done;                /* K5 zero-copy call: `seq` stored here (host memory, system scope) */
    uint32_t seq;                  /* after the output and the flag, so the host can poll for it */
};

/* Arguments of the serial graph kernel (bus form; one lane = one stream, loops over frames). */
struct IcwK4Args {
    uint32_t lds_guard;            /* dynamic LDS bytes: > 0 keeps the launch off the CUs K1 holds */
    const double *iq;              /* [n_streams][T][4] `in` per frame (lre, lim, rre, rim) */
    int32_t n_streams, T;
    long long t0;
    const unsigned long long *n_frame;   /* call-start frame counters */
    unsigned long long ssr;
    int32_t scaled;
    uint32_t sample_rate;
    const IcwProg *prog;
    double *bus;                   /* [n_streams][27][4] */
    double *pre;                   /* [n_streams][pre_stride] (lOut, rOut) per frame */
    size_t pre_stride;
};

/* Arguments of the IIR state kernel (one lane = one DF-II chain). */
struct IcwK1Args {
    const double *xd;              /* K0 output: per-chain filter inputs */
    size_t x_pitch;
    uint32_t nch;
    int32_t n_streams, n_chains, T;
    double *hist;                  /* [n_chains][ICW_HIST_PITCH], index 0 = most recent w */
    unsigned long long *sncnt;     /* [n_chains] subnorm rejections */
    double *w;                     /* [n_chains][w_pitch]: rows [0,N) history, [N,N+T) block */
    size_t w_pitch;
    uint32_t *lr_equal;            /* [n_streams][2] per filter (I, Q): the right converter's chain is
                                      bit-identical to the left one (state) */
    uint32_t *info_dup;            /* [n_streams][2] lr_equal at this block's start (for K2) */
    const uint32_t *hq_phase;      /* [n_streams][2] call-start Hilbert phases (zero-input parity) */
    long long t0;                  /* block offset into the call */
    int *err;                      /* set by a bounded spin that gave up (never in a healthy run) */
    int32_t wg_waves;              /* waves per workgroup of the plain / row kernels (1..4) */
    uint32_t lds_hold;             /* LDS bytes a K1 workgroup holds (static + dynamic): the CU's whole
                                      LDS keeps every LDS-using workgroup off K1's CUs; 0: static only */
    int32_t dedup;                 /* mono, every stream's converters identical: left chains only */
    double pc[20];                 /* loop-back coefficients -a[i+1]/a0 */
    uint32_t *fes;                 /* FP_CHECK: [n_streams][4][ICW_FES_PITCH] census (Hilbert L, R,
                                      render L, R); null: no FC() arithmetic */
};

/* One compiled DSP node (adv_modulator.c:637-751), executed in list order tail -> head. */
struct IcwOp {
    int32_t mode;                  /* ICW_MODE_* */
    int32_t n_in;                  /* inputs, in bus-slot order */
    int32_t in_reg[27];            /* value register each input resolves to */
    int32_t out_reg;               /* register the node's output lands in (not MASTER) */
    uint32_t in_mask;              /* bus-program form: bit k = reads bus slot k */
    int32_t out_slot;              /* bus-program form: slot written (n_out) */
    int32_t xch, iqinv[2];
    int32_t tout[2];
    int32_t act[2];                /* is_shift / is_pm per channel */
    int32_t neg[2];                /* shift: negative frequency -> sin_v = -sin_v */
    double gain[2];
    double f[2];                   /* effective (scaled) frequency */
    double pp[2], lp[2], fa[2];    /* PM: fphase*PI, flevel*PI, fangle */
    int32_t tslot[2];              /* Shift / PM channel: column of the per-frame rotation table */
    int32_t wb_slot;               /* register form: the slot whose final value this op writes (its
                                      output goes to the persistent bus at a block's last frame), -1 */
    int32_t chain_in;              /* chain program: bit 0 reads `in`, bit 1 the previous op's output */
    int32_t unit_gain[2];          /* gain[c] == 1.0: a scalar test for the kernels (an FP64 compare of an
                                      SGPR value is a VALU instruction) */
};

/* A compiled DSP list.  Register form (frame-parallel output kernel): every slot read resolves at
 * compile time to `in`, an earlier op of the same frame or a never-written (constant) slot.  Bus
 * form (serial graph kernel, is_bus = 1): the reference's own bus semantics, for lists that read a
 * slot before it is written in the frame -- a one-frame delay, feedback included. */
struct IcwProg {
    int32_t n_ops;
    int32_t is_bus;
    int32_t n_regs;
    int32_t bypass;                /* am.is_bypass_list: only the Master, on raw `in` */
    int32_t needs_omega;           /* some Shift / PM node is active: the frame's norm_omega is used */
    int32_t n_trig;                /* active Shift / PM channels = columns of the rotation table */
    int32_t n_persist;             /* slots read before any write in the frame and never written */
    int32_t chain;                 /* register form where every op reads only `in` and / or the op just
                                      before it: values stay in registers (no LDS register file) */
    int32_t sig;                   /* chain programs: op count | (mode | chain_in << 2) << (4 + 4 i), ops in
                                      execution order; the fused FIR kernel runs a few of these straight
                                      (ICW_SIG_*, icw_kernels.hip); 0: not a chain */
    int32_t persist_reg[ICW_MAX_REGS], persist_slot[ICW_MAX_REGS];
    IcwOp ops[ICW_MAX_OPS];
};

/* Render constants computed on the host by the sound_render_recalc arithmetic
 * (sound_render.c:499-581), so pow() runs once on the CPU exactly as in the reference. */
struct IcwRenderK {
    double norm_mul, dth_mul, hi, lo, round_offset;
    double clip_abs;               /* min(hi, -lo): a q with |q| below it clips at neither bound */
    double spec_thr;               /* K3r: a 20-sample block whose every x * norm_mul is <= this in magnitude,
                                      after a block whose every |q| < clip_abs, clips nowhere (render_consts);
                                      -1: no clamp-free blocks */
    int32_t sign_delta, norm_shift, is24;
    int32_t render_type, ns_kind, ns_n;
    int32_t lo1, hi1;              /* (int)lo + 1, (int)hi - 1: the clamp's integer bounds (scalar) */
    int32_t unit_mul;              /* norm_mul == 1.0 (scalar test, as IcwOp.unit_gain) */
    double ns_c[40];
};

/* Arguments of the serial render kernel (one lane = one channel's SOUND_RENDER). */
struct IcwK3Args {
    const double *pre;             /* [n_streams][T][2] pre-render values from the output kernel */
    size_t pre_stride;             /* doubles per stream */
    int32_t n_streams, T;
    unsigned char *out;            /* stream s at out + s*out_stride */
    size_t out_stride;
    uint32_t *mt;                  /* [624][mt_pitch] MT19937 state words, generator g = s*2 + ch */
    int32_t *mt_idx;               /* [n_gen] index of the next word (624: twist needed) */
    double *rs;                    /* [n_gen][ICW_RSTATE]: prev_rnd, prev_ns_err, E[20], O[20] */
    uint32_t *clips;               /* [n_streams][2] */
    unsigned long long *peak_bits; /* [n_streams][2] */
    int32_t n_gen, mt_pitch;
    IcwRenderK rk;
    double *dith;                  /* rnd * dth_mul per sample (K3a -> the render); null: ROUND.  dith_gm 0:
                                      time-major [T][dith_pitch] (K3b, K3f: a lane per channel reads one
                                      row coalesced); 1: generator-major [n_gen][dith_pitch] (K3r and the
                                      frame-parallel renders read runs of one channel; K3a writes 512-byte runs) */
    size_t dith_pitch;
    uint32_t *fes;                 /* FP_CHECK census, as in IcwK1Args; null: no FC() */
    int32_t row;                   /* render kernel: 1 row broadcast (K3r, small batches), 0 lane per channel */
    int32_t dith_gm;               /* layout of dith (above) */
    int32_t comp;                  /* K3r: 1 with a companion wave (staging and flush off the chain's wave) */
    int32_t *err;                  /* nonzero after a companion hand-off that never came (never in a healthy run) */
    /* the split dither generator (icw_launch_dither; null wbuf: the one-kernel K3a, ICW_DITHER=coop) */
    uint32_t *wbuf;                /* [n_gen][wpitch] tempered MT words of a chunk (K3t -> K3s) */
    size_t wpitch, wcap;           /* words per generator row; rows' capacity in words (chunking) */
    int32_t *dflag;                /* [n_gen] a rejected dsopen pair in the chunk: K3f redoes the channel */
    uint32_t *dbk;                 /* [n_gen][ICW_DBK] the chunk's starting generator state (K3t -> K3f) */
};
#define ICW_DBK 628                /* u32 per backup: 624 words, idx, pad, prev_rnd (a double at 626) */

/* Arguments of the output kernel (frame-parallel: Kahan output sums, unmix, graph, render). */
struct IcwK2Args {
    const double *w;               /* [n_chains][w_pitch] */
    size_t w_pitch;
    int32_t n_streams, T, n_chains, nch;
    long long t0;                  /* block offset into the call */
    const uint32_t *hq_phase;      /* [n_streams][2] call-start Hilbert phases */
    const unsigned long long *n_frame;   /* [n_streams] call-start frame counters */
    unsigned long long ssr;
    int32_t scaled;
    uint32_t sample_rate;
    const IcwProg *prog;
    double *bus;                   /* [n_streams][27][4] persistent bus */
    unsigned char *out;            /* stream s at out + s*out_stride */
    size_t out_stride;
    double *pre;                   /* nullable [n_streams][T][2] pre-render doubles */
    size_t pre_stride;             /* in doubles, per stream */
    int32_t do_render;             /* elementwise ROUND/flat render in this kernel */
    int32_t n_regs;                /* DSP value registers (sizes the dynamic LDS register file) */
    uint32_t *clips;               /* [n_streams][2] */
    unsigned long long *peak_bits; /* [n_streams][2] max |q| as ordered bits */
    IcwRenderK rk;
    double pc[20], pd[20], d0;
    const uint32_t *info_dup;      /* [n_streams][2] K1's flags: the converters were identical at block start */
    const double *xin;             /* complex input: K0's I/Q rows (then w is unused) */
    size_t x_pitch;
    int32_t cw;
    double *iq_out;                /* bus-form graph: write `in` here [n_streams][T][4], skip the rest */
    int32_t trig;                  /* prog.needs_omega: instantiate the Shift / PM code */
    unsigned long long *sncnt;     /* [n_chains] de-subnorm rejections (hblpf.c:1046-1050), counted
                                      here from the block's w rows; null: not counted */
    const double *trig_tab;        /* nullable [T][trig_pitch]: (cos, sin) per active Shift / PM channel
                                      for streams whose call-start counter equals stream 0's */
    int32_t trig_pitch;
    int32_t trig_perm_q;           /* the table's row order (icw_trig_index) */
    int32_t zero;                  /* always 0: an offset the compiler cannot fold (keeps loads in a loop) */
    uint32_t *fes;                 /* FP_CHECK census, as in IcwK1Args; null: no FC() */
    int32_t tpw;                   /* tiles per workgroup (1..ICW_K2_TPW), set by the launcher */
    const double *dith;            /* nullable: a dithered render with the flat shaper, rendered here
                                      frame-parallel -- K3a's rnd * dth_mul, generator-major
                                      [n_streams * 2][dith_pitch] (row 2s + ch, frame t of the block) */
    size_t dith_pitch;
};

/* Per-frame rotation table (one thread per frame): the Shift / PM factors depend only on the frame
 * counter, so streams in step share them -- computed once per block, not once per stream. */
struct IcwTrigArgs {
    uint32_t lds_guard;            /* dynamic LDS bytes: > 0 keeps the launch off the CUs K1 holds */
    const IcwProg *prog;
    const unsigned long long *n_frame;   /* the reference stream's call-start counter (stream 0) */
    long long t0;
    int32_t T, scaled, trig_pitch;
    unsigned long long ssr;
    uint32_t sample_rate;
    double *tab;                   /* [T][trig_pitch], rows in icw_trig_index order */
    int32_t perm_q;                /* 0: row t at t; > 0 (KF2): row t at (t & 7) * perm_q + (t >> 3) */
};


/* FC() of fp_check.c:52-100 (except_stats_check): a NaN or a denormal becomes 0.0, an infinity
 * +-INF_HUGE_VALUE (65535.0, fp_check.h:60); each is counted in FP_EXCEPT_STATS order total, snan,
 * qnan, ninf, nden, pden, pinf.  _fpclass calls a NaN with the quiet bit (mantissa bit 51) clear
 * signaling.  Counters are per thread; the kernels add them to the census at the end. */
struct IcwFes {
    uint32_t c[7];
};

#if defined(__HIPCC__) || defined(__HIP__)
/* not inlined: FP_CHECK is a diagnostic mode, and inlined FC() branches at every operation of the
 * unrolled sums multiply the code size (and the build time) of the FC kernels */
__device__ __noinline__ double icw_fc(double v, IcwFes &f)
{
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned ex = (unsigned)((u >> 52) & 0x7ffu);
    const unsigned long long man = u & 0xfffffffffffffull;
    if (ex == 0x7ffu) {
        ++f.c[0];
        if (man) { ++f.c[((man >> 51) & 1u) ? 2 : 1]; return 0.0; }
        if (u >> 63) { ++f.c[3]; return -65535.0; }
        ++f.c[6];
        return 65535.0;
    }
    if (ex == 0u && man) { ++f.c[0]; ++f.c[(u >> 63) ? 4 : 5]; return 0.0; }
    return v;
}

/* the same value without counting (a product whose FC() another kernel already counted) */
__device__ __forceinline__ double icw_fc_nc(double v)
{
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned ex = (unsigned)((u >> 52) & 0x7ffu);
    if (ex == 0x7ffu) return (u & 0xfffffffffffffull) ? 0.0 : ((u >> 63) ? -65535.0 : 65535.0);
    return ex == 0u ? (v == 0.0 ? v : 0.0) : v;
}

__device__ __forceinline__ void icw_fes_flush(const IcwFes &f, uint32_t *dst)
{
#pragma unroll
    for (int k = 0; k < 7; ++k)
        if (f.c[k]) atomicAdd(dst + k, f.c[k]);
}
#endif

/* K5 icw_stream1: the four kernels of a one-stream, one-block call in one workgroup */
#define ICW_S1_MAX 4096   /* frames: the output phase runs T / 256 tiles in turn */
struct IcwS1Args {
    IcwK0Args k0;
    IcwK1Args k1;
    IcwK2Args k2;
    IcwAdvArgs adv;
    IcwTrigArgs trig;              /* the block's rotation table (has_trig), computed beside the recurrence */
    int32_t has_trig;
    unsigned long long *stamps;    /* diagnostic: [4][2] phase-boundary stamps (null: none) */
    int32_t ovl;                   /* request (host) / set (launcher): output phase beside the recurrence */
    int32_t rows_off;              /* ovl: the w rows' offset in dynamic LDS (doubles, after K2's registers) */
    int32_t lpitch;                /* ovl: doubles per w row in LDS (T + N + 1, even) */
};
#define ICW_S1_OVL_LDS (128 * 1024)   /* ovl: dynamic LDS budget (register file + w rows) */

#endif
