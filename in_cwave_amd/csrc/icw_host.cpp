/*
 * icw_host.cpp -- host side of the in_cwave_amd C ABI (include/icw.h): context lifecycle,
 * DSP-list normalisation and compilation, per-stream state in HBM, block scheduling of the
 * gfx950 kernels, meters and state (de)serialisation.
 *
 * There is no CPU compute path here: every sample goes through icw_kernels.hip.  A missing or
 * unusable HIP device is an error (ICW_EDEVICE), never a fallback.
 */
#include <hip/hip_runtime_api.h>

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <list>
#include <map>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/icw.h"
#include "icw_device.h"
#include "icw_tables.inc"

extern "C" hipError_t icw_launch_unpack(const IcwK0Args *a, hipStream_t st);
extern "C" hipError_t icw_launch_iir_state(const IcwK1Args *a, int nord, int kahan, int subn, hipStream_t st);
extern "C" hipError_t icw_launch_iir_row(const IcwK1Args *a, int nord, int kahan, int subn, hipStream_t st);
extern "C" hipError_t icw_launch_iir_fc(const IcwK1Args *a, int nord, int kahan, int subn, hipStream_t st);
extern "C" hipError_t icw_launch_render(const IcwK3Args *a, hipStream_t st);
extern "C" hipError_t icw_launch_dither(const IcwK3Args *a, hipStream_t st);
extern "C" hipError_t icw_launch_dither_lane(const IcwK3Args *a, hipStream_t st);
extern "C" hipError_t icw_launch_output(const IcwK2Args *a, int nord, int kahan, hipStream_t st);
extern "C" hipError_t icw_launch_trig_table(const IcwTrigArgs *a, hipStream_t st);
extern "C" hipError_t icw_launch_graph_serial(const IcwK4Args *a, hipStream_t st);
extern "C" hipError_t icw_launch_advance(const IcwAdvArgs *a, hipStream_t st);
extern "C" hipError_t icw_launch_stream1(const IcwS1Args *a, int nord, hipStream_t st);
extern "C" hipError_t icw_launch_fir(const IcwFirArgs *a, hipStream_t st);
extern "C" hipError_t icw_launch_fir_graph(const IcwFirArgs *f, const IcwK2Args *a, int in_step, hipStream_t st);
extern "C" size_t icw_fir_graph_lds(int M, int nt, int nch, int n_regs);

#define ICW_PI_H (3.1415926535897932384626433832795029)

namespace {

double u2d(unsigned long long u)
{
    double d;
    memcpy(&d, &u, 8);
    return d;
}

/* frames per kernel launch: bounds the w scratch buffer (n_chains * (T+N) doubles) */
constexpr int kMaxBlockFrames = 1 << 16;
constexpr int kDefBlockFrames = 1 << 14;   /* launch block: shorter pipeline fill / drain */
constexpr int kSets = 3;                    /* most block scratch sets (ICW_SETS); default 2 */
constexpr double kAutoTaper = 0.85;          /* tail block ratio where the taper is on by default */
constexpr double kRowTaper = 0.25;           /* tail ratio of the row kernel's long blocks (no serial render) */
/* FIR converter + serial render: the first blocks grow by this ratio from kFirRenderFirst frames, so
 * that each block's converter and dither generator (one stream, ~30 us per 1 000 frames of c5fir) are
 * done before the render of the block before it ends (K3c: ~52 us per 1 000 frames).  Round 4's 2.5
 * was set for K3r at ~2.6x the converter + generator; with K3c the ratio is ~1.7, and 2.5 left ~1 ms of
 * gaps per c5fir step (profiles/r06_c5fir_fill.txt).  2 048 / 1.5 measured best of the first-block x
 * ramp grid, c5fir 9 110 -> 9 482 Msamples/s over three runs (profiles/r06_c5fir_ramp_ab.txt).
 * Running the generator beside the converter on a stream of its own removed the gaps but lowered
 * the render's clock more than that (same file). */
constexpr double kFirRenderRamp = 1.5;
constexpr int kFirRenderFirst = 2048;
/* the fused FIR converter on device buffers with nothing after it (no serial render, no host copies
 * to overlap): one launch block per 2^20 frames.  At 65 536 each block paid a rotation-table launch
 * and two ~12 us gaps beside its 0.26 ms kernel, 13 % of a c2fir step */
constexpr int kMaxFirBlockFrames = 1 << 20;
constexpr int kRowRenderMax = 2048;          /* channels up to which the render runs a row per channel */
constexpr size_t kPinnedStage = 1u << 20;   /* host-pointer calls up to this size stage through pinned memory */

struct DevState {
    double *hist = nullptr;               /* [chains][20] */
    unsigned long long *sncnt = nullptr;  /* [chains] */
    uint32_t *hq_phase = nullptr;         /* [streams][2] */
    long long *pos = nullptr;             /* [streams] */
    long long *fade = nullptr;            /* [streams][3] */
    unsigned long long *n_frame = nullptr;/* [streams] */
    double *bus = nullptr;                /* [streams][27][4] */
    uint32_t *clips = nullptr;            /* [streams][2] */
    unsigned long long *peak_bits = nullptr; /* [streams][2] */
    int *err = nullptr;                   /* kernel hand-off timeout flag */
    /* serial render state (only when the render is not ROUND/flat) */
    uint32_t *mt = nullptr;               /* [624][2*streams] */
    int32_t *mt_idx = nullptr;            /* [2*streams] */
    double *rs = nullptr;                 /* [2*streams][ICW_RSTATE] */
    uint32_t *lr_equal = nullptr;         /* [streams][2] right converters bit-identical to left ones, per filter */
    uint32_t *fes = nullptr;              /* FP_CHECK: [streams][4][ICW_FES_PITCH] FP-exception census */
};

/* streams confined to disjoint CU sets: K1 on k1_cus CUs spread over the device, the rest on
 * the other CUs (hipExtStreamCreateWithCUMask) */
struct CuSplit {
    int k1_cus = 0, rest_cus = 0;
    hipStream_t k1 = nullptr, rest = nullptr, dith = nullptr, render = nullptr;
};

}  // namespace

struct icw_ctx {
    icw_config cfg{};
    std::vector<icw_node> nodes;
    int n_streams = 0;
    int device = 0;
    int nord = 0;
    double pc[20]{}, pd[20]{}, d0 = 0.0;
    IcwRenderK rk{};
    IcwProg prog{};
    IcwProg *d_prog = nullptr;
    DevState st;
    /* host mirrors of meters that survive "reset" semantics */
    std::vector<double> peak_db;          /* [streams][2] */
    /* scratch */
    /* double-buffered block scratch: block b uses set b & 1, so the output kernel of block b
     * (second stream) overlaps the IIR state kernel of block b+1 */
    double *w[kSets] = {};
    size_t w_bytes[kSets] = {};
    double *xd[kSets] = {};
    size_t xd_bytes[kSets] = {};
    uint32_t *info_dup[kSets] = {};
    hipStream_t stream2 = nullptr;
    hipEvent_t k1done[kSets] = {}, k2done[kSets] = {}, join = nullptr;
    hipEvent_t k0done[kSets] = {};
    bool cu_split = true;                 /* ICW_CU_SPLIT=0 disables the partition */
    /* ICW_K1_WPC: K1 waves per CU.  Two: measured under a working partition, 4 per CU (one per
     * SIMD) made K1 +21 % slower even alone (C3, 4-wave workgroups), 3 per CU +27 % beside K2, and 1
     * per CU leaves the frame-parallel kernels too few CUs (C4 K2 2.57 -> 3.70 ms) */
    int k1_wpc = 2;
    /* ICW_REST_CUS: at most this many CUs for the frame-parallel kernels beside K1 (0: all the rest).
     * Default (-1): all but 32 (4 per XCD) -- idle CUs leave K1 power headroom: C3 41.6-42.2k ->
     * 42.6-42.9k, C4 20.9k -> 21.1-21.3k Msamples/s at 160 and 176 (profiles/r04_rest_cus.txt);
     * below 160 K2 falls behind (C3 38.0k at 144 and 128) */
    int rest_cus = -1;
    double fir_ramp = 0.0;                /* ICW_FIR_RAMP: the ramp of a FIR + serial-render call (0: kFirRenderRamp) */
    /* ICW_K1_WG: K1 waves per workgroup.  Default 1 for the lane kernel, 2 for the row kernel: its I and
     * Q filter waves of the same streams then share a CU, so the second one reads the channel rows
     * (one per channel since round 3) from the L2 / L1 the first one filled (C2 +0.7 %, C5 +0.4 %; the
     * lane kernel loses 2-2.5 % on C3 / C4 with 2) */
    int k1_wg = 1;
    bool k1_wg_env = false;
    bool k1_lds = false;                  /* ICW_K1_LDS=1: K1 workgroups hold the CU's LDS (A/B) */
    bool fill_drain = true;               /* ICW_FILL_DRAIN=0: first K0 / last K2 stay partitioned (A/B) */
    uint32_t lds_cu = 0;                  /* LDS bytes per CU a workgroup may hold */
    int max_block = kDefBlockFrames;      /* ICW_BLOCK: frames per launch block */
    bool block_env = false;               /* ICW_BLOCK given */
    bool dedup_ok = true;                 /* ICW_DEDUP=0 disables the mono K1 dedup (A/B) */
    int max_sets = 2;                     /* ICW_SETS: block scratch sets (2..kSets) */
    /* block schedule of long calls (plan_blocks): a short first block (the pipeline fill is K0 of
     * block 0 alone: C3 +2.5 %, C4 +1.4 %) and an optional geometric tail (the drain is K2 / K3 of
     * the last block alone).  The tail pays only if K0 + K2 (and K3) of a block fit beside K1 of a
     * block r times shorter: in C3 / C4 they take 0.87 / 0.94 of K1's time per frame, and r = 0.85
     * measured C3 -4 %, C4 -8 %; in C5 (K1r, K2 0.12 and the row render K3r 0.64 of K1r on their own
     * streams) r = 0.85 measured +2 %.  So it is on by default for the row kernel with a serial
     * render only (icw_process_streams). */
    int first_block = 4096;               /* ICW_FIRST_BLOCK (0: uniform blocks) */
    bool first_block_env = false;
    double taper = -1.0;                  /* ICW_TAPER: tail block ratio (0: no tail; -1: auto) */
    int taper_min = 1024;                 /* ICW_TAPER_MIN: smallest tail block */
    /* dither generation (K3a) runs on its own stream, double-buffered like the block scratch */
    hipStream_t stream3 = nullptr;
    hipEvent_t ditdone[kSets] = {};
    double *dith[kSets] = {};
    size_t dith_bytes[kSets] = {};
    /* the split dither generator's chunk buffers (icw_launch_dither): tempered words, rejection flags,
     * starting-state backups; one set, used in order on the dither stream */
    uint32_t *dwords = nullptr, *dbk = nullptr;
    int32_t *dflag = nullptr;
    size_t dwords_bytes = 0, dbk_bytes = 0, dflag_bytes = 0;
    size_t dwcap = 0;                     /* words per generator row of dwords */
    unsigned char *d_in = nullptr, *d_out = nullptr;
    size_t d_in_bytes = 0, d_out_bytes = 0;
    double *d_pre = nullptr;
    size_t d_pre_bytes = 0;
    double *d_xin = nullptr;              /* ICW_F_DEBUG_INPUT: K0's rows of the call, [2*streams][n_frames] */
    size_t d_xin_bytes = 0;
    /* small host-pointer calls (the one-stream drop-in, 576-frame blocks): inputs and outputs are
     * staged through this pinned buffer, so the copies are asynchronous and the call waits once */
    unsigned char *h_stage = nullptr;
    unsigned char *h_stage_dev = nullptr; /* the same memory as the device addresses it */
    size_t h_stage_bytes = 0;
    /* ICW_ZEROCOPY=0: small calls copy the staging buffer to and from HBM instead of the kernels
     * reading the input from, and writing the output to, the pinned buffer directly */
    bool zero_copy = true;
    bool spin_wait = true;                /* ICW_SPIN=0: K5 zero-copy calls wait on the stream instead */
    uint32_t s1_seq = 0;                  /* K5 completion sequence number (host-polled) */
    /* the serial render (K4 bus-form graph + K3b) runs on a fourth stream, one block behind K2:
     * its inputs are double-buffered like the block scratch */
    hipStream_t stream4 = nullptr;
    /* copy stream of the block-pipelined host I/O (pinned host buffers): per-block H2D / D2H */
    hipStream_t stream_io = nullptr;
    std::vector<hipEvent_t> ev_io;        /* H2D of launch block b done */
    hipEvent_t k3done[kSets] = {};
    double *rpre[kSets] = {};             /* per-block pre-render buffer for the serial render */
    size_t rpre_bytes[kSets] = {};
    double *iq[kSets] = {};               /* per-block `in` buffer for the bus-form graph */
    size_t iq_bytes[kSets] = {};
    double *trig = nullptr;               /* per-block rotation table [T][2 * n_trig] */
    size_t trig_bytes = 0;
    /* per stream: known on the host to have bit-identical left / right converters (fresh or reset
     * state, or a set_state with equal halves, and no stereo block since) -- mono calls over such
     * streams run K1 on the left chains only */
    std::vector<char> lr_known;
    /* host mirror of every stream's modulator frame counter (the device's n_frame, advanced by the same
     * arithmetic as icw_advance): a call whose streams are all in step has every Shift / PM factor in
     * the shared rotation table, so the fused FIR kernel takes its variant without the per-stream
     * fallback (whose out-of-line call cost it scratch spills) */
    std::vector<unsigned long long> nf_host;
    bool serial_render = false;
    bool render_state = false;            /* needs_render_state: the state blob carries the render words */
    uint32_t mt_seed_state[2][624];       /* seeded MT19937 states for L / R (mtrnd_init_seed) */
    hipStream_t stream = nullptr;
    std::vector<hipEvent_t> ev;
    int n_cu = 256;
    int k1_mode = -1;         /* K1 variant: -1 auto (row / plain), 0 plain lanes, 3 row broadcast
                                 (ICW_K1_MODE=plain|row, A/B runs) */
    bool dither_lane = false; /* ICW_DITHER=lane: lane-per-channel dither generator (A/B only) */
    bool dither_coop = false; /* ICW_DITHER=coop: the one-kernel wave-per-channel generator K3a (A/B only) */
    bool k3r_comp = true;     /* ICW_K3R_COMP=0: the row render without its companion wave (K3r, A/B) */
    int render_row = -1;      /* serial render kernel: -1 auto (row broadcast for <= kRowRenderMax
                                 channels), 0 lane per channel, 1 row (ICW_RENDER=serial|row) */
    bool serialize = false;   /* ICW_SERIALIZE=1: every kernel on the caller's stream (profiling) */
    double last_ms[2]{};
    int last_launches[2]{};
    int last_k1 = -1;                     /* ICW_K1_* of the last real-input call */
    /* FIR Hilbert converter (icw_set_fir_hilbert): order (0: the quadrature IIR), taps, and the
     * per-stream input history [streams][2][M], double-buffered by launch block (fir_par) */
    int fir_M = 0, fir_nt = 0;
    double fir_beta = 0.0;
    double *d_fir_g = nullptr;
    double *fir_hist[2] = {};
    int fir_par = 0;
    bool fir_fuse = true;                 /* ICW_FIR_FUSED=0: KF + K2 as two kernels (A/B) */
    bool stream1 = true;                  /* ICW_STREAM1=0: one-stream calls keep the four kernels (A/B) */
    bool s1_ovl = true;                   /* ICW_S1_OVL=0: K5's output phase after the recurrence (A/B) */
    bool chain_ok = true;                 /* ICW_CHAIN=0: chain programs keep the LDS register file (A/B) */
    unsigned long long *s1_stamps = nullptr;   /* ICW_S1_STAMPS=1: K5 phase stamps, printed per call */
    unsigned long long calls = 0;         /* icw_process_* calls so far (icw_prepare needs a fresh context) */
    /* per-stream state set by an entry point other than a call (stream_open, seek, set_state, the
     * resets): icw_prepare's closing icw_stream_init would wipe it, so it refuses.  Context-wide
     * setters (set_outbits, set_render, ...) leave it false: the warm-up runs with them. */
    bool touched = false;
    std::mutex mu;
};

namespace {

int set_dev(icw_ctx *c)
{
    return hipSetDevice(c->device) == hipSuccess ? ICW_OK : ICW_EDEVICE;
}

template <class T>
int dalloc(T **p, size_t n)
{
    *p = nullptr;
    if (n == 0) n = 1;
    if (hipMalloc((void **)p, n * sizeof(T)) != hipSuccess) return ICW_ENOMEM;
    if (hipMemset(*p, 0, n * sizeof(T)) != hipSuccess) return ICW_EDEVICE;
    return ICW_OK;
}

/* bytes per channel sample: HRW_FMT_* (xwave_reader.c:553-580), CWAVE cw_slen (xwave_reader.c:246-252) */
unsigned fmt_size(unsigned fmt)
{
    static const unsigned sz[9] = {1, 2, 3, 4, 4, 16, 4, 6, 8};
    return fmt < 9 ? sz[fmt] : 0;
}

/* amod_init (adv_modulator.c:216-331): accept the list only if its head is the one and only
 * Master and every mode is known; apply the L/R locks.  Otherwise the default Master. */
bool graph_accept(std::vector<icw_node> &n)
{
    if (n.empty() || n[0].mode != ICW_MODE_MASTER) return false;
    bool was_master = false;
    for (auto &t : n) {
        if (t.lock_gain) { t.gain[1] = t.gain[0]; t.iq_invert[1] = t.iq_invert[0]; }
        switch (t.mode) {
        case ICW_MODE_MASTER:
            if (was_master) return false;
            was_master = true;
            break;
        case ICW_MODE_SHIFT:
            if (t.lock_shift) {
                t.fr_shift[1] = t.sign_lock_shift ? -t.fr_shift[0] : t.fr_shift[0];
                t.is_shift[1] = t.is_shift[0];
            }
            break;
        case ICW_MODE_PM:
            if (t.lock_freq) { t.pm_freq[1] = t.pm_freq[0]; t.is_pm[1] = t.is_pm[0]; }
            if (t.lock_phase) t.pm_phase[1] = t.pm_phase[0];
            if (t.lock_level) t.pm_level[1] = t.pm_level[0];
            if (t.lock_angle) t.pm_angle[1] = t.pm_angle[0];
            break;
        case ICW_MODE_MIX:
            break;
        default:
            return false;
        }
    }
    return true;
}

icw_node default_master()
{
    icw_node n;
    memset(&n, 0, sizeof(n));
    n.mode = ICW_MODE_MASTER;
    n.gain[0] = n.gain[1] = 0.8;           /* DEF_GAIN_MASTER, in_cwave.h:167 */
    n.tout[0] = n.tout[1] = ICW_S_ADD_REIM;
    n.inputs[0] = 1;                       /* adv_modulator.c:112-118 */
    n.lock_gain = 1;
    return n;
}

/* DGET_SCALED_FR (adv_modulator.c:35-39) */
double scaled_fr(double f) { return (double)((unsigned)(f * ((double)ICW_HZ_SCALE) + 0.5)); }

/* Compile the normalised DSP list into register form.  Execution order is tail -> head
 * (adv_modulator.c:637).  Each input slot resolves to the value most recently written in the
 * same frame; a slot never written by any node reads its persistent bus value.  A slot read
 * before its writer runs (a one-frame delay, doc 3.1) is not yet on the device path. */
/* per-op parameters shared by the register and bus forms */
void op_params(const icw_node &n, IcwOp &op)
{
    op.mode = n.mode;
    op.wb_slot = -1;
    op.xch = n.xch_mode;
    op.iqinv[0] = n.iq_invert[0];
    op.iqinv[1] = n.iq_invert[1];
    op.gain[0] = n.gain[0];
    op.gain[1] = n.gain[1];
    op.unit_gain[0] = op.gain[0] == 1.0;
    op.unit_gain[1] = op.gain[1] == 1.0;
    op.out_slot = n.mode == ICW_MODE_MASTER ? 0 : n.n_out;
    op.in_mask = 0;
    for (int k = 0; k < ICW_N_INPUTS; ++k)
        if (n.inputs[k]) op.in_mask |= 1u << k;
    for (int c = 0; c < 2; ++c) {
        op.tout[c] = n.tout[c];
        if (n.mode == ICW_MODE_SHIFT) {
            op.act[c] = n.is_shift[c];
            double f = n.fr_shift[c];
            op.neg[c] = f < 0.0;
            if (f < 0.0) f = -f;
            op.f[c] = f;   /* scaled below if frmod_scaled */
        } else if (n.mode == ICW_MODE_PM) {
            op.act[c] = n.is_pm[c];
            op.f[c] = n.pm_freq[c];
            op.pp[c] = n.pm_phase[c] * ICW_PI_H;              /* fphase * PI */
            op.lp[c] = n.pm_level[c] * ICW_PI_H;              /* flevel * PI */
            op.fa[c] = n.pm_angle[c];
        }
    }
}

/* norm_omega is only read by active Shift / PM nodes (adv_modulator.c:519-583): frame-parallel
 * kernels skip the counter arithmetic and its division otherwise */
void set_needs_omega(IcwProg &P)
{
    P.needs_omega = 0;
    P.n_trig = 0;
    for (int i = 0; i < P.n_ops; ++i) {
        IcwOp &op = P.ops[i];
        op.tslot[0] = op.tslot[1] = -1;
        if (op.mode != ICW_MODE_SHIFT && op.mode != ICW_MODE_PM) continue;
        for (int c = 0; c < 2; ++c)
            if (op.act[c]) {
                op.tslot[c] = P.n_trig++;     /* a column of the per-frame rotation table */
                P.needs_omega = 1;
            }
    }
}

/* Bus form: the list as the reference runs it (tail -> head, or the head alone when bypassed) */
int compile_bus(const std::vector<icw_node> &nodes, int bypass, IcwProg &P)
{
    memset(&P, 0, sizeof(P));
    P.is_bus = 1;
    P.bypass = bypass;
    std::vector<int> order;
    if (bypass) order.push_back(0);
    else for (int i = (int)nodes.size() - 1; i >= 0; --i) order.push_back(i);
    if ((int)order.size() > ICW_MAX_OPS) return ICW_EUNSUPPORTED;
    for (size_t oi = 0; oi < order.size(); ++oi) {
        const icw_node &n = nodes[order[oi]];
        if (n.mode != ICW_MODE_MASTER && (n.n_out < 1 || n.n_out >= ICW_N_INPUTS)) return ICW_EGRAPH;
        op_params(n, P.ops[oi]);
    }
    P.n_ops = (int)order.size();
    P.n_regs = 1;
    set_needs_omega(P);
    return ICW_OK;
}

/* Register form for the frame-parallel output kernel; ICW_EUNSUPPORTED when a slot is read
 * before it is written in the frame (one-frame delay) or the list exceeds the register budget --
 * the caller then compiles the bus form.
 *
 * Value registers live in K2's LDS (8 KB each per 256-frame workgroup), so they are allocated by
 * liveness: `in` is register 0 for the frame; a node's output takes the lowest register whose value
 * has had its last reader (an op may write over its own inputs: it reads them all first); a slot
 * read but never written in the frame is loaded once per workgroup and keeps its register.  A
 * written slot's final value goes to the persistent bus from the op that writes it (wb_slot), at
 * the block's last frame, so it need not stay live to the end.  PM -> Shift -> Mix -> Master
 * (C4) takes 2 registers instead of 4, which lets K2 keep 4 waves per SIMD. */
int compile_graph(const std::vector<icw_node> &nodes, int bypass, IcwProg &P)
{
    memset(&P, 0, sizeof(P));
    P.bypass = bypass;
    std::vector<int> order;
    if (bypass) order.push_back(0);
    else for (int i = (int)nodes.size() - 1; i >= 0; --i) order.push_back(i);
    if ((int)order.size() > ICW_MAX_REG_OPS) return ICW_EUNSUPPORTED;
    const int n_ops = (int)order.size();

    bool written_any[ICW_N_INPUTS] = {false};
    for (int i : order)
        if (nodes[i].mode != ICW_MODE_MASTER) {
            const int o = nodes[i].n_out;
            if (o < 0 || o >= ICW_N_INPUTS) return ICW_EGRAPH;
            written_any[o] = true;
        }
    /* values: 0 = `in`, then persistent slots and op outputs in order of appearance */
    std::vector<int> last_use(1, -1), def_op(1, -1);
    std::vector<char> pinned(1, 0);
    std::vector<std::vector<int>> reads(n_ops);
    std::vector<int> out_val(n_ops, -1);
    int cur[ICW_N_INPUTS];
    for (int k = 0; k < ICW_N_INPUTS; ++k) cur[k] = -1;
    cur[0] = 0;
    std::vector<int> persist_val, persist_slot;
    for (int oi = 0; oi < n_ops; ++oi) {
        const icw_node &n = nodes[order[oi]];
        if (!bypass) {
            for (int k = 0; k < ICW_N_INPUTS; ++k) {
                if (!n.inputs[k]) continue;
                int v = cur[k];
                if (v < 0) {
                    if (written_any[k]) return ICW_EUNSUPPORTED;   /* delayed (feedback) read */
                    v = (int)last_use.size();
                    last_use.push_back(-1);
                    def_op.push_back(-1);
                    pinned.push_back(1);
                    persist_val.push_back(v);
                    persist_slot.push_back(k);
                    cur[k] = v;
                }
                reads[oi].push_back(v);
                last_use[v] = oi;
            }
        }
        if (n.mode != ICW_MODE_MASTER) {
            const int v = (int)last_use.size();
            last_use.push_back(-1);
            def_op.push_back(oi);
            pinned.push_back(0);
            out_val[oi] = v;
            cur[n.n_out] = v;
        }
    }
    /* the op that leaves each written slot its final value */
    std::vector<int> wb(n_ops, -1);
    for (int k = 0; k < ICW_N_INPUTS; ++k)
        if (written_any[k] && cur[k] >= 0) wb[def_op[cur[k]]] = k;
    /* physical registers */
    std::vector<int> phys(last_use.size(), -1), holder(ICW_MAX_REGS, -1);
    phys[0] = 0;
    holder[0] = 0;
    for (size_t q = 0; q < persist_val.size(); ++q) {
        int r = 1;
        while (r < ICW_MAX_REGS && holder[r] >= 0) ++r;
        if (r >= ICW_MAX_REGS) return ICW_EUNSUPPORTED;
        phys[persist_val[q]] = r;
        holder[r] = persist_val[q];
    }
    int n_regs = 1 + (int)persist_val.size();
    for (int oi = 0; oi < n_ops; ++oi) {
        IcwOp &op = P.ops[oi];
        const icw_node &n = nodes[order[oi]];
        op.mode = n.mode;
        for (int v : reads[oi]) op.in_reg[op.n_in++] = phys[v];
        op_params(n, op);
        op.wb_slot = wb[oi];
        /* free the registers whose values were read for the last time by this op */
        for (int r = 0; r < ICW_MAX_REGS; ++r) {
            const int v = holder[r];
            if (v >= 0 && !pinned[v] && last_use[v] <= oi) holder[r] = -1;
        }
        if (out_val[oi] >= 0) {
            int r = 0;
            while (r < ICW_MAX_REGS && holder[r] >= 0) ++r;
            if (r >= ICW_MAX_REGS) return ICW_EUNSUPPORTED;
            phys[out_val[oi]] = r;
            holder[r] = out_val[oi];
            op.out_reg = r;
            n_regs = std::max(n_regs, r + 1);
        }
    }
    P.n_ops = n_ops;
    P.n_regs = n_regs;
    for (size_t q = 0; q < persist_val.size(); ++q) {
        P.persist_reg[q] = phys[persist_val[q]];
        P.persist_slot[q] = persist_slot[q];
    }
    P.n_persist = (int)persist_val.size();
    /* chain program (C2's Shift -> Master, C4's PM -> Shift -> Mix(in + B) -> Master): every op reads
     * only `in` and / or the output of the op just before it.  Reads are in slot order and `in` is
     * slot 0, so the sum is 0.0 + in + prev in the reference's order (adv_modulator.c:655-665) */
    P.chain = P.n_persist == 0 ? 1 : 0;
    for (int oi = 0; oi < n_ops && P.chain; ++oi) {
        int bits = 0;
        for (int v : reads[oi]) {
            if (v == 0 && !(bits & 1) && !(bits & 2)) bits |= 1;
            else if (oi > 0 && v == out_val[oi - 1] && v >= 0 && !(bits & 2)) bits |= 2;
            else P.chain = 0;
        }
        P.ops[oi].chain_in = bits;
    }
    /* the signature of a chain of plain ops (the device runs it straight, icw_chain_sig): no channel
     * exchange or I/Q swap, both channels of a Shift / PM rotating, a Master summing re + im */
    P.sig = 0;
    bool plain = P.chain && n_ops <= 6;
    for (int oi = 0; oi < n_ops && plain; ++oi) {
        const IcwOp &op = P.ops[oi];
        plain = op.xch == ICW_XCH_NORMAL && !op.iqinv[0] && !op.iqinv[1];
        if (op.mode == ICW_MODE_MASTER) plain &= op.tout[0] == ICW_S_ADD_REIM && op.tout[1] == ICW_S_ADD_REIM;
        else if (op.mode != ICW_MODE_MIX) plain &= op.act[0] && op.act[1];
    }
    if (plain) {
        P.sig = n_ops;
        for (int oi = 0; oi < n_ops; ++oi) P.sig |= ((P.ops[oi].mode & 3) | (P.ops[oi].chain_in << 2)) << (4 + 4 * oi);
        /* bit 30: every op but the Master has gain 1.0 on both channels (ICW_SIG_UNIT) */
        bool unit = true;
        for (int oi = 0; oi < n_ops; ++oi)
            if (P.ops[oi].mode != ICW_MODE_MASTER) unit &= P.ops[oi].gain[0] == 1.0 && P.ops[oi].gain[1] == 1.0;
        if (unit) P.sig |= 1 << 30;
    }
    set_needs_omega(P);
    return ICW_OK;
}

/* sound_render_recalc arithmetic (sound_render.c:499-581) */
void render_consts(const icw_render_cfg &cfg, int is24, IcwRenderK &k)
{
    memset(&k, 0, sizeof(k));
    k.dth_mul = pow(2.0, cfg.dth_bits) - 1.0;
    if (cfg.quantz_type == ICW_QUANTZ_MID_TREAD) { k.round_offset = 0.5; k.sign_delta = 0; }
    else { k.round_offset = 0.0; k.sign_delta = -1; }
    if (is24) {
        long long hib = 0x800000LL;
        k.norm_shift = 24 - (int)cfg.sign_bits24;
        hib >>= k.norm_shift;
        k.hi = (double)hib;
        k.lo = -(double)(hib + 1 + k.sign_delta);
        k.norm_mul = (k.norm_shift < 8) ? (double)(0x100 >> k.norm_shift)
                                         : 1.0 / (double)(1ULL << (k.norm_shift - 8));
    } else {
        long long hib = 0x8000LL;
        k.norm_shift = 16 - (int)cfg.sign_bits16;
        hib >>= k.norm_shift;
        k.hi = (double)hib;
        k.lo = -(double)(hib + 1 + k.sign_delta);
        k.norm_mul = 1.0 / (double)(1ULL << k.norm_shift);
    }
    k.lo -= (double)k.sign_delta;
    k.clip_abs = std::min(k.hi, -k.lo);
    k.lo1 = (int32_t)k.lo + 1;
    k.hi1 = (int32_t)k.hi - 1;
    k.unit_mul = k.norm_mul == 1.0;
    k.is24 = is24;
    k.render_type = (int)cfg.render_type;
    unsigned t = cfg.nshape_type > ICW_NSHAPE_MAX ? ICW_NSHAPE_FLAT : cfg.nshape_type;
    k.ns_kind = icw_ns_kind[t];
    k.ns_n = icw_ns_n[t];
    const int nc = k.ns_kind == 2 ? 2 * k.ns_n : k.ns_n;
    for (int i = 0; i < nc; ++i) k.ns_c[i] = u2d(icw_ns_c[t][i]);
    /* K3r's clamp-free blocks (icw_render_row).  Without a clip the error fed back is small: with
     * q = input + d and the integer trunc(q) + delta (mid-riser) or trunc(q +- 0.5) (mid-tread),
     * |ev| = |(double)val - input| <= 1.5 + Dm, Dm the largest |rnd * dth_mul| of the render type
     * (sound_render.c:711-751: RPDF |dsopen| / SQRT2 < 0.708, TPDF and STPDF < 1, GAUSS 12 / (2 SQRT6)
     * < 2.45), so a FIR shaper's output |prev_ns_err| <= B (1.5 + Dm), B = sum |c_i|.  A block whose
     * inputs all have |x * norm_mul| <= spec_thr, after a block without a clip (so the shaper history
     * holds only such errors), then has |q| <= spec_thr + B (1.5 + Dm) + Dm + 0.5 < clip_abs for every
     * sample: nothing clips and the clamp is the identity, so the block runs without it.  The IIR
     * shaper feeds back its own output: never. */
    k.spec_thr = -1.0;
    static const bool spec = !getenv("ICW_K3R_SPEC") || atoi(getenv("ICW_K3R_SPEC")) != 0;
    if (spec && k.ns_kind != 2 && cfg.render_type <= ICW_RENDER_GAUSS) {
        static const double cdm[5] = {0.0, 0.708, 1.0, 1.0, 2.45};
        double B = 0.0;
        if (k.ns_kind == 1)
            for (int i = 0; i < k.ns_n; ++i) B += fabs(k.ns_c[i]);
        const double Dm = cfg.render_type == ICW_RENDER_ROUND ? 0.0 : fabs(k.dth_mul) * cdm[cfg.render_type];
        const double thr = k.clip_abs - B * (1.5 + Dm) * 1.001 - Dm - 0.5 - 1.0;
        if (thr > 0.0) k.spec_thr = thr;             /* NaN / inf dth_mul: never */
    }
}

/* The normalised list (graph_accept) as the device program: register form, or the bus form when a
 * slot is read before its writer runs.  With frmod_scaled the PM frequencies are scaled from f
 * (dsp_pm) and the Shift ones from |f| (dsp_shift), as DGET_SCALED_FR does per frame. */
int build_prog(const icw_config &cfg, std::vector<icw_node> nodes, IcwProg &P)
{
    /* by value: the context keeps the list as given (unscaled), so that the list primitives can edit
     * and recompile it */
    if (cfg.frmod_scaled)
        for (auto &n : nodes)
            if (n.mode == ICW_MODE_PM)
                for (int ch = 0; ch < 2; ++ch) n.pm_freq[ch] = scaled_fr(n.pm_freq[ch]);
    int rc = compile_graph(nodes, cfg.bypass_list, P);
    if (rc == ICW_EUNSUPPORTED) rc = compile_bus(nodes, cfg.bypass_list, P);
    if (rc) return rc;
    if (cfg.frmod_scaled)
        for (int i = 0; i < P.n_ops; ++i)
            if (P.ops[i].mode == ICW_MODE_SHIFT)
                for (int ch = 0; ch < 2; ++ch) P.ops[i].f[ch] = scaled_fr(P.ops[i].f[ch]);
    return ICW_OK;
}

/* A render with the flat shaper is elementwise: ns_empty returns 0.0 (sound_render.c:396-400), so
 * prev_ns_err stays 0.0 (:800) and sound_render_value (:754-809) is a function of the sample and its
 * dither term alone.  ROUND draws no dither; RPDF / TPDF / STPDF / GAUSS take theirs from K3a (the
 * MT19937 stream is serial per channel, the render is not), so all of them render inside the output
 * kernel, frame-parallel (ICW_DITH_PAR=0: the dithered ones through the serial render, A/B).  A noise
 * shaper feeds each sample's error into the next: serial per channel, in the serial render kernel --
 * as is every render behind a bus-form graph (frame-serial, hands lOut / rOut over) or with FP_CHECK
 * (the FC() render arithmetic lives in the serial render kernel only). */
bool dith_par_on()
{
    static const bool on = !getenv("ICW_DITH_PAR") || atoi(getenv("ICW_DITH_PAR")) != 0;
    return on;
}

bool needs_serial(const icw_config &cfg, const IcwRenderK &rk, const IcwProg &P)
{
    const bool elementwise = rk.ns_kind == 0 && (cfg.render.render_type == ICW_RENDER_ROUND || dith_par_on());
    return !elementwise || P.is_bus || cfg.fp_check;
}

/* the per-channel render state (MT19937 words, prev_rnd, shaper rings): a serial render, or a dithered
 * one rendered frame-parallel (its generator still runs, K3a) */
bool needs_render_state(const icw_config &cfg, const IcwRenderK &rk, const IcwProg &P)
{
    return needs_serial(cfg, rk, P) || cfg.render.render_type != ICW_RENDER_ROUND;
}

bool render_cfg_ok(const icw_render_cfg &r)
{
    return r.sign_bits16 >= 2 && r.sign_bits16 <= 16 && r.sign_bits24 >= 2 && r.sign_bits24 <= 24 &&
           r.quantz_type <= 1 && r.render_type <= 4;
}

int grow(void **p, size_t *cur, size_t need)
{
    if (*cur >= need) return ICW_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cur = 0;
    if (hipMalloc(p, need) != hipSuccess) return ICW_ENOMEM;
    *cur = need;
    return ICW_OK;
}

/* The stream set for a K1 of k1_cus CUs (a multiple of the XCD count): K1's CUs are spread evenly
 * over the XCDs and their shader engines, the other streams get the remaining CUs.
 * Queue CU-mask bits on gfx950 are dealt round-robin: bit b selects XCD b % 8, and within it the
 * (b / 8)-th CU, whose shader-engine group is again (b / 8) % 4 (measured, tools/cumask_probe.hip).
 * An XCD with no bit set in a mask runs that queue's work on ALL of its CUs, so each mask must
 * name CUs in every XCD: the K1 mask is bits [0, k1_cus), the rest its complement. */
/* wait for every kernel and copy of the context (they run on several streams, the caller's among
 * them); host-side state changes and reads happen only between calls */
/* Launch blocks of one call: (offset, frames) pairs of at most Tb frames.  A block pipeline fills
 * with K0 of the first block alone and drains with K2 (and the serial render) of the last block
 * alone, each on the whole chip (sF).  For calls of many blocks both ends are made short:
 *   - the first block is `first` frames, long enough that K1 of it covers K0 of the next full one;
 *   - the tail shrinks geometrically (ratio r) down to `tmin`, so that K2 of every tail block, which
 *     runs beside K1 of the next one, stays no longer than that K1 (C4: K2 ~0.8 K1 per frame).
 * With `ramp` > 1 the blocks after the first grow by that ratio up to Tb (the FIR converter's fill,
 * below).  Block sizes stay multiples of 64 frames; short calls keep uniform blocks. */
std::vector<std::pair<int, int>> plan_blocks(int n_frames, int Tb, int first, double r, int tmin, double ramp = 0.0)
{
    std::vector<std::pair<int, int>> bl;
    std::vector<int> tail;
    const bool shape = n_frames >= 4 * Tb;
    if (shape && r > 0.0) {
        for (double x = Tb * r; x >= tmin; x *= r) tail.push_back(((int)x) & ~63);
        long sum = 0;
        for (int v : tail) sum += v;
        if (sum > n_frames / 2) tail.clear();
    }
    int t = 0;
    double grow = 0.0;
    if (shape && first >= 64 && first < Tb) {
        bl.emplace_back(0, first);
        t = first;
        if (ramp > 1.0) grow = first * ramp;
    }
    long tail_sum = 0;
    for (int v : tail) tail_sum += v;
    const int body_end = n_frames - (int)tail_sum;
    while (t < body_end) {
        int T = std::min(Tb, body_end - t);
        if (grow > 0.0 && grow < Tb) {
            T = std::min(T, std::max(64, ((int)grow) & ~63));
            grow *= ramp;
        }
        bl.emplace_back(t, T);
        t += T;
    }
    for (int v : tail) {
        bl.emplace_back(t, v);
        t += v;
    }
    return bl;
}

/* page-locked host memory (hipHostMalloc / hipHostRegister) that device `dev` may copy from: the DMA
 * engines read it directly, so an asynchronous copy does not block the host thread.  Memory pinned
 * while another device was current counts only if it was pinned portable (hipHostMallocPortable /
 * hipHostRegisterPortable, as icw_host_alloc does): the shards of icw_group_process hand slices of one
 * caller buffer to contexts on different devices.  Anything else takes the whole-call staging copies.
 * A pageable pointer makes the query fail; the error is cleared so that it does not surface as the
 * call's own. */
bool host_pinned(const void *p, int dev)
{
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost && (a.device == dev || (a.allocationFlags & hipHostMallocPortable));
}

/* wait for a K5 call's sequence number in host memory; the stream is queried now and then, so a
 * failed launch or a device fault ends the wait with an error instead of a hang */
bool poll_done(const uint32_t *flag, uint32_t seq, hipStream_t st)
{
    for (unsigned it = 1;; ++it) {
        if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq) return true;
        if ((it & 255u) == 0u) {
            const hipError_t q = hipStreamQuery(st);
            if (q == hipSuccess) return __atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq;
            if (q != hipErrorNotReady) return false;
        }
        __builtin_ia32_pause();
    }
}

hipError_t quiesce(icw_ctx *c)
{
    (void)c;
    return hipDeviceSynchronize();
}

/* The CU-masked stream sets are shared by the contexts of a device (created on first use, destroyed
 * with the device's last context), so a process that opens many contexts does not multiply queues.
 * Sharing only adds ordering between contexts that run on the same device at the same time. */
std::mutex g_split_mu;
std::list<std::pair<int, CuSplit>> g_splits;     /* list: entries never move */
std::map<int, int> g_live;                       /* device -> live contexts */

void split_ref(int device, int delta)
{
    std::lock_guard<std::mutex> lk(g_split_mu);
    if ((g_live[device] += delta) > 0) return;
    for (auto it = g_splits.begin(); it != g_splits.end();) {
        if (it->first != device) { ++it; continue; }
        for (hipStream_t q : {it->second.k1, it->second.rest, it->second.dith, it->second.render})
            if (q) (void)hipStreamDestroy(q);
        it = g_splits.erase(it);
    }
}

const CuSplit *cu_split(icw_ctx *c, int k1_cus)
{
    std::lock_guard<std::mutex> lk(g_split_mu);
    const int rest_cus = c->rest_cus >= 0 ? c->rest_cus : std::max(c->n_cu - k1_cus - 32, c->n_cu / 2);
    for (auto &x : g_splits)
        if (x.first == c->device && x.second.k1_cus == k1_cus && x.second.rest_cus == rest_cus) return &x.second;
    const int n = c->n_cu, words = (n + 31) / 32;
    std::vector<uint32_t> mk(words, 0u), mr(words, 0u);
    std::vector<char> used(n, 0);
    for (int i = 0; i < k1_cus && i < n; ++i) used[i] = 1;
    int n_rest = 0;
    for (int cu = 0; cu < n; ++cu) {
        if (used[cu]) mk[cu / 32] |= 1u << (cu % 32);
        else if (rest_cus == 0 || n_rest++ < rest_cus) mr[cu / 32] |= 1u << (cu % 32);
    }
    CuSplit x;
    x.k1_cus = k1_cus;
    x.rest_cus = rest_cus;
    if (hipExtStreamCreateWithCUMask(&x.k1, (uint32_t)words, mk.data()) != hipSuccess ||
        hipExtStreamCreateWithCUMask(&x.rest, (uint32_t)words, mr.data()) != hipSuccess ||
        hipExtStreamCreateWithCUMask(&x.dith, (uint32_t)words, mr.data()) != hipSuccess ||
        hipExtStreamCreateWithCUMask(&x.render, (uint32_t)words, mr.data()) != hipSuccess) {
        for (hipStream_t q : {x.k1, x.rest, x.dith, x.render})
            if (q) (void)hipStreamDestroy(q);
        return nullptr;
    }
    g_splits.emplace_back(c->device, x);
    return &g_splits.back().second;
}

/* modified Bessel function I0 by its power series sum ((x/2)^k / k!)^2, to a relative 1e-17 */
double bessel_i0(double x)
{
    const double h = x / 2.0;
    double sum = 1.0, term = 1.0;
    for (int k = 1; k < 1000; ++k) {
        term *= h / (double)k;
        const double t2 = term * term;
        sum += t2;
        if (t2 < sum * 1e-17) break;
    }
    return sum;
}

/* FIR histories of streams [f, f+n) to zero (a fresh or reset converter) */
bool fir_clear(icw_ctx *c, size_t f, size_t n, hipStream_t st)
{
    bool ok = true;
    const size_t row = 2 * (size_t)c->fir_M;
    for (double *h : c->fir_hist)
        if (h) ok &= hipMemsetAsync(h + f * row, 0, n * row * sizeof(double), st) == hipSuccess;
    return ok;
}

void free_all(icw_ctx *c)
{
    DevState &s = c->st;
    void *ptrs[] = {c->s1_stamps, s.mt, s.mt_idx, s.rs, s.lr_equal, s.fes, s.err, s.hist, s.sncnt, s.hq_phase, s.pos, s.fade,
                    s.n_frame, s.bus, s.clips, s.peak_bits, c->d_prog, c->trig, c->d_in, c->d_out, c->d_pre, c->d_xin,
                    c->d_fir_g, c->fir_hist[0], c->fir_hist[1], c->dwords, c->dbk, c->dflag};
    for (void *p : ptrs)
        if (p) (void)hipFree(p);
    for (int p = 0; p < kSets; ++p) {
        for (void *q : {(void *)c->info_dup[p], (void *)c->w[p], (void *)c->xd[p], (void *)c->dith[p],
                        (void *)c->rpre[p], (void *)c->iq[p]})
            if (q) (void)hipFree(q);
        for (hipEvent_t e : {c->ditdone[p], c->k1done[p], c->k2done[p], c->k0done[p], c->k3done[p]})
            if (e) (void)hipEventDestroy(e);
    }
    if (c->h_stage) (void)hipHostFree(c->h_stage);
    if (c->stream3) (void)hipStreamDestroy(c->stream3);
    if (c->stream4) (void)hipStreamDestroy(c->stream4);
    if (c->stream_io) (void)hipStreamDestroy(c->stream_io);
    for (auto e : c->ev_io) (void)hipEventDestroy(e);
    if (c->join) (void)hipEventDestroy(c->join);
    if (c->stream2) (void)hipStreamDestroy(c->stream2);
    for (auto e : c->ev) (void)hipEventDestroy(e);
    if (c->stream) (void)hipStreamDestroy(c->stream);
}

/* filter coefficients of cfg.hilbert_type exactly as iir_rp_create (hblpf.c:849-856) */
void set_filter(icw_ctx *c)
{
    const int t = (int)c->cfg.hilbert_type;
    c->nord = icw_hb_order[t];
    const double a0 = u2d(icw_hb_a[t][0]);
    c->d0 = u2d(icw_hb_b[t][0]) / a0;
    for (int i = 0; i < ICW_MAX_IIR_ORDER; ++i) c->pc[i] = c->pd[i] = 0.0;
    for (int i = 0; i < c->nord; ++i) {
        c->pc[i] = -u2d(icw_hb_a[t][i + 1]) / a0;
        c->pd[i] = u2d(icw_hb_b[t][i + 1]) / a0;
    }
}

/* renders of streams [f, f + n) as sound_render_init leaves them (in_cwave.c:69-70): MT19937
 * seeded (mtrnd_init_seed), next draw twists, shaping state zero.  Synchronous. */
bool seed_renders(icw_ctx *c, size_t f, size_t n, hipStream_t st)
{
    DevState &s = c->st;
    const size_t G = (size_t)c->n_streams * 2;
    std::vector<uint32_t> col((size_t)624 * n * 2);
    for (int i = 0; i < 624; ++i)
        for (size_t k = 0; k < n * 2; ++k) col[(size_t)i * n * 2 + k] = c->mt_seed_state[k & 1][i];
    std::vector<int32_t> idx(n * 2, 624);
    bool ok = hipMemcpy2DAsync(s.mt + f * 2, G * 4, col.data(), n * 2 * 4, n * 2 * 4, 624, hipMemcpyHostToDevice,
                               st) == hipSuccess;
    ok &= hipMemcpyAsync(s.mt_idx + f * 2, idx.data(), idx.size() * 4, hipMemcpyHostToDevice, st) == hipSuccess;
    ok &= hipMemsetAsync(s.rs + f * 2 * ICW_RSTATE, 0, n * 2 * ICW_RSTATE * sizeof(double), st) == hipSuccess;
    ok &= hipStreamSynchronize(st) == hipSuccess;   /* the host sources live until here */
    return ok;
}

/* the serial render's per-channel state, allocated when a live change first needs it.  Until then
 * every render was ROUND + flat, which draws no random numbers and keeps no shaping state, so the
 * freshly seeded state is the reference's state at this point. */
int ensure_render_state(icw_ctx *c)
{
    DevState &s = c->st;
    if (s.mt) return ICW_OK;
    const size_t S = (size_t)c->n_streams;
    int rc = dalloc(&s.mt, (size_t)624 * S * 2);
    rc |= dalloc(&s.mt_idx, S * 2);
    rc |= dalloc(&s.rs, S * 2 * ICW_RSTATE);
    if (rc == ICW_OK && !seed_renders(c, 0, S, c->stream)) rc = ICW_EDEVICE;
    if (rc != ICW_OK) {
        for (void *p : {(void *)s.mt, (void *)s.mt_idx, (void *)s.rs})
            if (p) (void)hipFree(p);
        s.mt = nullptr;
        s.mt_idx = nullptr;
        s.rs = nullptr;
        return rc == ICW_ENOMEM ? ICW_ENOMEM : ICW_EDEVICE;
    }
    return ICW_OK;
}

/* The device keeps each channel's largest |q| and get_meters turns it into dB against the render's
 * current hi bound.  Before a render change moves that bound, the peaks so far are folded into the
 * host's dB meters against the old bound (the reference converts every sample with the bound of
 * its time, sound_render.c:769-780) and the device maxima start again. */
bool fold_peaks(icw_ctx *c)
{
    const size_t n = (size_t)c->n_streams * 2;
    std::vector<unsigned long long> pb(n);
    bool ok = hipMemcpy(pb.data(), c->st.peak_bits, n * 8, hipMemcpyDeviceToHost) == hipSuccess;
    ok &= hipMemset(c->st.peak_bits, 0, n * 8) == hipSuccess;
    if (!ok) return false;
    for (size_t i = 0; i < n; ++i) {
        double mx;
        memcpy(&mx, &pb[i], 8);
        const double cv = mx ? 20.0 * log10(mx / c->rk.hi) : ICW_SR_ZERO_SIGNAL_DB;
        if (cv > c->peak_db[i]) c->peak_db[i] = cv;
    }
    return true;
}

/* mod_context_clear_all_inouts (in_cwave.c:255-261): slot `slot` of every stream's bus to zero.
 * The context's work has been waited for (quiesce). */
int clear_slot(icw_ctx *c, int slot)
{
    if (slot < 0 || slot >= ICW_N_INPUTS) return ICW_OK;
    const size_t pitch = (size_t)ICW_N_INPUTS * 4 * sizeof(double);
    return hipMemset2D(c->st.bus + (size_t)slot * 4, pitch, 0, 4 * sizeof(double), (size_t)c->n_streams) == hipSuccess
               ? ICW_OK : ICW_EDEVICE;
}

/* the device's Hilbert phases of streams [first, ...): [stream][L, R] */
const uint32_t *ds_phase_of(const icw_ctx *c, int first) { return c->st.hq_phase + (size_t)first * 2; }

/* the output slot replace_output_plug clears for node n (adv_modulator.c:180-205): Shift / PM / Mix
 * own one, a Master none (-1) */
int plug_slot(const icw_node &n)
{
    return (n.mode == ICW_MODE_SHIFT || n.mode == ICW_MODE_PM || n.mode == ICW_MODE_MIX) ? n.n_out : -1;
}

/* A live list edit (the caller holds c->mu and has waited for the context's work): compile the
 * normalised list nv, install the program, then zero the bus slots the reference's edit clears.  The
 * program goes to the device first, so a failed copy leaves the old program and the old bus on both
 * sides; a failed clear after it returns ICW_EDEVICE with the new program in place (the context is
 * quiesced, so the order of the two steps changes no output). */
int apply_graph(icw_ctx *c, std::vector<icw_node> &nv, int bypass, const std::vector<int> &clears)
{
    icw_config cfg = c->cfg;
    cfg.bypass_list = bypass;
    IcwProg P;
    int rc = build_prog(cfg, nv, P);
    if (rc) return rc;
    if (!c->chain_ok) P.chain = P.sig = 0;
    const bool serial = needs_serial(cfg, c->rk, P), rstate = needs_render_state(cfg, c->rk, P);
    if (rstate && (rc = ensure_render_state(c))) return rc;
    if (hipMemcpy(c->d_prog, &P, sizeof(IcwProg), hipMemcpyHostToDevice) != hipSuccess) return ICW_EDEVICE;
    c->cfg.bypass_list = cfg.bypass_list;
    c->nodes = nv;
    c->prog = P;
    c->serial_render = serial;
    c->render_state = rstate;
    for (int slot : clears)
        if (clear_slot(c, slot) != ICW_OK) return ICW_EDEVICE;
    return ICW_OK;
}

}  // namespace

extern "C" {

const char *icw_version(void) { return "in_cwave_amd 0.1 (gfx950)"; }

int icw_abi_version(void) { return ICW_ABI_VERSION; }

const char *icw_strerror(int s)
{
    switch (s) {
    case ICW_OK: return "ok";
    case ICW_EINVAL: return "invalid argument";
    case ICW_ENOMEM: return "out of memory";
    case ICW_EDEVICE: return "HIP device error";
    case ICW_EGRAPH: return "DSP list rejected";
    case ICW_EUNSUPPORTED: return "configuration not supported on the device path";
    }
    return "unknown";
}

int icw_create(const icw_config *cfg, const icw_node *nodes, int n_nodes, int n_streams, int device,
               icw_ctx **out, int *accepted)
{
    if (!cfg || !out || n_streams <= 0 || n_nodes < 0 || (n_nodes > 0 && !nodes)) return ICW_EINVAL;
    *out = nullptr;
    if (cfg->hilbert_type > 5 || cfg->in_format > ICW_FMT_CW_F32 || cfg->in_channels == 0 ||
        cfg->sample_rate == 0 || cfg->sample_rate > ICW_MAX_FS_SRC)
        return ICW_EINVAL;
    if (!render_cfg_ok(cfg->render)) return ICW_EINVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return ICW_EDEVICE;
    icw_ctx *c = new (std::nothrow) icw_ctx();
    if (!c) return ICW_ENOMEM;
    c->cfg = *cfg;
    if (device < 0) {
        if (hipGetDevice(&device) != hipSuccess) { delete c; return ICW_EDEVICE; }
    }
    c->device = device;
    if (set_dev(c)) { delete c; return ICW_EDEVICE; }
    c->nodes.assign(nodes, nodes + n_nodes);
    const bool ok = graph_accept(c->nodes);
    if (!ok) c->nodes.assign(1, default_master());
    if (accepted) *accepted = ok ? 1 : 0;
    int rc = build_prog(*cfg, c->nodes, c->prog);
    if (rc) { delete c; return rc; }
    set_filter(c);
    render_consts(cfg->render, cfg->need24bits, c->rk);
    c->serial_render = needs_serial(*cfg, c->rk, c->prog);
    c->render_state = needs_render_state(*cfg, c->rk, c->prog);
    for (int ch = 0; ch < 2; ++ch) {
        uint32_t *st = c->mt_seed_state[ch];
        st[0] = ch ? cfg->seed_right : cfg->seed_left;         /* mtrnd_init_seed, mt_jrnd.c:28-47 */
        for (uint32_t j = 1; j < 624; ++j) st[j] = 1812433253u * (st[j - 1] ^ (st[j - 1] >> 30)) + j;
    }
    c->n_streams = n_streams;
    const size_t S = (size_t)n_streams, C = S * 4;
    rc = ICW_OK;
    DevState &s = c->st;
    rc |= dalloc(&s.hist, C * ICW_HIST_PITCH);
    rc |= dalloc(&s.sncnt, C);
    rc |= dalloc(&s.hq_phase, S * 2);
    rc |= dalloc(&s.pos, S);
    rc |= dalloc(&s.fade, S * 3);
    rc |= dalloc(&s.n_frame, S);
    rc |= dalloc(&s.bus, S * ICW_N_INPUTS * 4);
    rc |= dalloc(&s.clips, S * 2);
    rc |= dalloc(&s.peak_bits, S * 2);
    rc |= dalloc(&s.err, 1);
    if (c->render_state) {
        rc |= dalloc(&s.mt, (size_t)624 * S * 2);
        rc |= dalloc(&s.mt_idx, S * 2);
        rc |= dalloc(&s.rs, S * 2 * ICW_RSTATE);
    }
    rc |= dalloc(&s.lr_equal, S * 2);
    if (cfg->fp_check) rc |= dalloc(&s.fes, S * 4 * ICW_FES_PITCH);
    for (int p = 0; p < kSets; ++p) rc |= dalloc(&c->info_dup[p], S * 2);
    rc |= dalloc(&c->d_prog, 1);
    if (rc == ICW_OK && hipMemcpy(c->d_prog, &c->prog, sizeof(IcwProg), hipMemcpyHostToDevice) != hipSuccess)
        rc = ICW_EDEVICE;
    if (rc == ICW_OK && hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) rc = ICW_EDEVICE;
    if (rc == ICW_OK && hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking) != hipSuccess) rc = ICW_EDEVICE;
    if (rc == ICW_OK && hipStreamCreateWithFlags(&c->stream3, hipStreamNonBlocking) != hipSuccess) rc = ICW_EDEVICE;
    if (rc == ICW_OK && hipStreamCreateWithFlags(&c->stream4, hipStreamNonBlocking) != hipSuccess) rc = ICW_EDEVICE;
    if (rc == ICW_OK && hipStreamCreateWithFlags(&c->stream_io, hipStreamNonBlocking) != hipSuccess) rc = ICW_EDEVICE;
    for (int p = 0; p < kSets && rc == ICW_OK; ++p)
        if (hipEventCreateWithFlags(&c->k1done[p], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&c->k2done[p], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&c->ditdone[p], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&c->k0done[p], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&c->k3done[p], hipEventDisableTiming) != hipSuccess)
            rc = ICW_EDEVICE;
    if (rc == ICW_OK && hipEventCreateWithFlags(&c->join, hipEventDisableTiming) != hipSuccess) rc = ICW_EDEVICE;
    if (rc != ICW_OK) {
        free_all(c);
        delete c;
        return rc < 0 ? (rc == ICW_ENOMEM ? ICW_ENOMEM : ICW_EDEVICE) : ICW_EDEVICE;
    }
    c->peak_db.assign(S * 2, ICW_SR_ZERO_SIGNAL_DB);
    c->lr_known.assign(S, 1);
    c->nf_host.assign(S, 0ull);
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, c->device) == hipSuccess) c->n_cu = prop.multiProcessorCount;
        c->k1_mode = -1;
        const char *m = getenv("ICW_K1_MODE");
        if (m && !strcmp(m, "plain")) c->k1_mode = 0;
        if (m && !strcmp(m, "row")) c->k1_mode = 3;
        const char *rr = getenv("ICW_RENDER");
        if (rr && !strcmp(rr, "serial")) c->render_row = 0;
        if (rr && !strcmp(rr, "row")) c->render_row = 1;
        const char *d = getenv("ICW_DITHER");
        c->dither_lane = d && !strcmp(d, "lane");
        c->dither_coop = d && !strcmp(d, "coop");
        const char *kc = getenv("ICW_K3R_COMP");
        if (kc && !strcmp(kc, "0")) c->k3r_comp = false;

        const char *z = getenv("ICW_SERIALIZE");
        c->serialize = z && !strcmp(z, "1");
        const char *cs = getenv("ICW_CU_SPLIT");
        if (cs && !strcmp(cs, "0")) c->cu_split = false;
        const char *wpc = getenv("ICW_K1_WPC");
        if (wpc && atoi(wpc) >= 1 && atoi(wpc) <= 8) c->k1_wpc = atoi(wpc);
        const char *fr = getenv("ICW_FIR_RAMP");
        if (fr && atof(fr) > 1.0 && atof(fr) <= 16.0) c->fir_ramp = atof(fr);
        const char *rc = getenv("ICW_REST_CUS");
        if (rc && (atoi(rc) == 0 || atoi(rc) >= 8)) c->rest_cus = atoi(rc);
        const char *bl = getenv("ICW_BLOCK");
        if (bl && atoi(bl) >= 256 && atoi(bl) <= kMaxBlockFrames) { c->max_block = atoi(bl); c->block_env = true; }
        const char *ns = getenv("ICW_SETS");
        if (ns && atoi(ns) >= 2 && atoi(ns) <= kSets) c->max_sets = atoi(ns);
        const char *zc = getenv("ICW_ZEROCOPY");
        if (zc && !strcmp(zc, "0")) c->zero_copy = false;
        const char *sw = getenv("ICW_SPIN");
        if (sw && !strcmp(sw, "0")) c->spin_wait = false;
        const char *fb = getenv("ICW_FIRST_BLOCK");
        if (fb && atoi(fb) >= 0) { c->first_block = atoi(fb); c->first_block_env = true; }
        const char *tp = getenv("ICW_TAPER");
        if (tp && atof(tp) >= 0.0 && atof(tp) < 1.0) c->taper = atof(tp);
        const char *tm = getenv("ICW_TAPER_MIN");
        if (tm && atoi(tm) >= 64) c->taper_min = atoi(tm);
        const char *dd = getenv("ICW_DEDUP");
        if (dd && !strcmp(dd, "0")) c->dedup_ok = false;
        const char *fd = getenv("ICW_FILL_DRAIN");
        if (fd && !strcmp(fd, "0")) c->fill_drain = false;
        const char *ff = getenv("ICW_FIR_FUSED");
        if (ff && !strcmp(ff, "0")) c->fir_fuse = false;
        const char *che = getenv("ICW_CHAIN");
        if (che && !strcmp(che, "0")) {
            c->chain_ok = false;
            c->prog.chain = c->prog.sig = 0;
            if (hipMemcpy(c->d_prog, &c->prog, sizeof(IcwProg), hipMemcpyHostToDevice) != hipSuccess) {
                free_all(c);
                delete c;
                return ICW_EDEVICE;
            }
        }
        const char *s1e = getenv("ICW_STREAM1");
        if (s1e && !strcmp(s1e, "0")) c->stream1 = false;
        const char *s1o = getenv("ICW_S1_OVL");
        if (s1o && !strcmp(s1o, "0")) c->s1_ovl = false;
        const char *s1s = getenv("ICW_S1_STAMPS");
        if (s1s && !strcmp(s1s, "1") && dalloc(&c->s1_stamps, 8) != ICW_OK) c->s1_stamps = nullptr;
        const char *kl = getenv("ICW_K1_LDS");
        c->k1_lds = kl && !strcmp(kl, "1");
        {
            hipDeviceProp_t p2;
            if (hipGetDeviceProperties(&p2, c->device) == hipSuccess) {
                size_t l = p2.sharedMemPerBlock;
                if (p2.maxSharedMemoryPerMultiProcessor && p2.maxSharedMemoryPerMultiProcessor < l)
                    l = p2.maxSharedMemoryPerMultiProcessor;
                c->lds_cu = (uint32_t)l;
            }
        }
        const char *wg = getenv("ICW_K1_WG");
        if (wg && atoi(wg) >= 1 && atoi(wg) <= 4) { c->k1_wg = atoi(wg); c->k1_wg_env = true; }
    }
    rc = icw_stream_init(c, 0, n_streams);
    if (rc) { free_all(c); delete c; return rc; }
    split_ref(c->device, +1);
    *out = c;
    return ICW_OK;
}

int icw_destroy(icw_ctx *c)
{
    if (!c) return ICW_EINVAL;
    set_dev(c);
    (void)quiesce(c);
    free_all(c);
    split_ref(c->device, -1);
    delete c;
    return ICW_OK;
}

int icw_stream_init(icw_ctx *c, int first, int count)
{
    if (!c || first < 0 || count < 0 || first + count > c->n_streams) return ICW_EINVAL;
    if (count == 0) return ICW_OK;
    std::lock_guard<std::mutex> lk(c->mu);
    if (set_dev(c)) return ICW_EDEVICE;
    DevState &s = c->st;
    const size_t f = (size_t)first, n = (size_t)count;
    hipStream_t st = c->stream;
    bool ok = true;
    ok &= hipMemsetAsync(s.hist + f * 4 * ICW_HIST_PITCH, 0, n * 4 * ICW_HIST_PITCH * sizeof(double), st) == hipSuccess;
    ok &= hipMemsetAsync(s.sncnt + f * 4, 0, n * 4 * sizeof(unsigned long long), st) == hipSuccess;
    ok &= hipMemsetAsync(s.hq_phase + f * 2, 0, n * 2 * sizeof(uint32_t), st) == hipSuccess;
    ok &= hipMemsetD32Async((hipDeviceptr_t)(s.lr_equal + f * 2), 1, n * 2, st) == hipSuccess;
    for (size_t i = 0; i < n; ++i) c->lr_known[f + i] = 1;
    ok &= hipMemsetAsync(s.pos + f, 0, n * sizeof(long long), st) == hipSuccess;
    ok &= hipMemsetAsync(s.n_frame + f, 0, n * sizeof(unsigned long long), st) == hipSuccess;
    for (size_t i = 0; i < n; ++i) c->nf_host[f + i] = 0;
    ok &= hipMemsetAsync(s.bus + f * ICW_N_INPUTS * 4, 0, n * ICW_N_INPUTS * 4 * sizeof(double), st) == hipSuccess;
    ok &= hipMemsetAsync(s.clips + f * 2, 0, n * 2 * sizeof(uint32_t), st) == hipSuccess;
    ok &= hipMemsetAsync(s.peak_bits + f * 2, 0, n * 2 * sizeof(unsigned long long), st) == hipSuccess;
    if (s.fes) ok &= hipMemsetAsync(s.fes + f * 4 * ICW_FES_PITCH, 0, n * 4 * ICW_FES_PITCH * 4, st) == hipSuccess;
    ok &= fir_clear(c, f, n, st);
    /* no track open: n_samples "infinite", no fades (xwave_unpack_csample never fades) */
    std::vector<long long> fd(n * 3);
    for (size_t i = 0; i < n; ++i) { fd[i * 3] = (long long)1 << 62; fd[i * 3 + 1] = 0; fd[i * 3 + 2] = 0; }
    ok &= hipMemcpyAsync(s.fade + f * 3, fd.data(), fd.size() * sizeof(long long), hipMemcpyHostToDevice, st) == hipSuccess;
    /* renders re-seeded (mod_context_init -> sound_render_init, in_cwave.c:69-70) wherever their
     * state exists (a context whose renders never needed it has none yet, ensure_render_state) */
    if (s.mt) ok &= seed_renders(c, f, n, st);
    ok &= hipStreamSynchronize(st) == hipSuccess;
    for (size_t i = f * 2; i < (f + n) * 2; ++i) c->peak_db[i] = ICW_SR_ZERO_SIGNAL_DB;
    return ok ? ICW_OK : ICW_EDEVICE;
}

int icw_stream_open(icw_ctx *c, int s, int64_t n_samples, uint32_t fade_in, uint32_t fade_out,
                    uint32_t sec_align, int clr_nframe, int clr_hilb)
{
    if (!c || s < 0 || s >= c->n_streams || n_samples < 0) return ICW_EINVAL;
    (void)sec_align;   /* the virtual zero tail is produced by the reader (xwave_read_samples) */
    long long nfi = (long long)(((uint64_t)fade_in * (uint64_t)c->cfg.sample_rate) / 1000ULL);
    long long nfo = (long long)(((uint64_t)fade_out * (uint64_t)c->cfg.sample_rate) / 1000ULL);
    if (nfi + nfo >= n_samples) {
        if (n_samples < 300LL) nfi = nfo = 0;
        else {
            if (nfi) nfi = n_samples / 3;
            if (nfo) nfo = n_samples / 3;
        }
    }
    std::lock_guard<std::mutex> lk(c->mu);
    if (set_dev(c)) return ICW_EDEVICE;
    long long fd[3] = {(long long)n_samples, nfi, nfo};
    c->touched = true;
    bool ok = quiesce(c) == hipSuccess;
    ok &= hipMemcpy(c->st.fade + (size_t)s * 3, fd, sizeof(fd), hipMemcpyHostToDevice) == hipSuccess;
    ok &= hipMemset(c->st.pos + s, 0, sizeof(long long)) == hipSuccess;
    if (clr_nframe) {
        ok &= hipMemset(c->st.n_frame + s, 0, sizeof(unsigned long long)) == hipSuccess;
        c->nf_host[s] = 0;
    }
    if (clr_hilb) {
        ok &= hipMemset(c->st.hist + (size_t)s * 4 * ICW_HIST_PITCH, 0, 4 * ICW_HIST_PITCH * sizeof(double)) == hipSuccess;
        ok &= hipMemset(c->st.sncnt + (size_t)s * 4, 0, 4 * sizeof(unsigned long long)) == hipSuccess;
        ok &= hipMemset(c->st.hq_phase + (size_t)s * 2, 0, 2 * sizeof(uint32_t)) == hipSuccess;
        ok &= hipMemsetD32((hipDeviceptr_t)(c->st.lr_equal + (size_t)s * 2), 1, 2) == hipSuccess;
        c->lr_known[s] = 1;
        ok &= fir_clear(c, (size_t)s, 1, c->stream) && hipStreamSynchronize(c->stream) == hipSuccess;
    }
    /* sound_render_set_outbits -> sound_render_recalc: prev_rnd, shaper buffers and prev_ns_err
     * reset, the RNG is not (sound_render.c:527-580) */
    if (c->st.rs)
        ok &= hipMemset(c->st.rs + (size_t)s * 2 * ICW_RSTATE, 0, 2 * ICW_RSTATE * sizeof(double)) == hipSuccess;
    return ok ? ICW_OK : ICW_EDEVICE;
}

int icw_stream_reset_hilbert(icw_ctx *c, int s)
{
    if (!c || s < 0 || s >= c->n_streams) return ICW_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    if (set_dev(c)) return ICW_EDEVICE;
    c->touched = true;
    bool ok = quiesce(c) == hipSuccess;
    ok &= hipMemset(c->st.hist + (size_t)s * 4 * ICW_HIST_PITCH, 0, 4 * ICW_HIST_PITCH * sizeof(double)) == hipSuccess;
    ok &= hipMemset(c->st.sncnt + (size_t)s * 4, 0, 4 * sizeof(unsigned long long)) == hipSuccess;
    ok &= hipMemset(c->st.hq_phase + (size_t)s * 2, 0, 2 * sizeof(uint32_t)) == hipSuccess;
    ok &= hipMemsetD32((hipDeviceptr_t)(c->st.lr_equal + (size_t)s * 2), 1, 2) == hipSuccess;
    c->lr_known[s] = 1;
    ok &= fir_clear(c, (size_t)s, 1, c->stream) && hipStreamSynchronize(c->stream) == hipSuccess;
    return ok ? ICW_OK : ICW_EDEVICE;
}

int icw_fir_taps(int32_t M, double beta, double *g, int n)
{
    if (M < 2 || M > ICW_FIR_MAX_ORDER || (M & 1) || !(beta >= 0.0 && beta < 1e3) || !g) return ICW_EINVAL;
    const int c = M / 2, nt = (c + 1) / 2;
    if (n < nt) return ICW_EINVAL;
    const double i0b = bessel_i0(beta);
    for (int k = 0; k < nt; ++k) {
        const int m = 2 * k + 1;
        const double r = (double)m / (double)c;
        const double w = bessel_i0(beta * sqrt(1.0 - r * r)) / i0b;
        g[k] = (2.0 / (ICW_PI_H * (double)m)) * w;
    }
    return nt;
}

int icw_set_fir_hilbert(icw_ctx *c, int32_t M, double beta)
{
    static_assert(ICW_FIR_MAX_ORDER == ICW_FIR_MAX_M, "FIR order limit of the header and the kernel");
    if (!c || (M != 0 && (M < 2 || M > ICW_FIR_MAX_ORDER || (M & 1))) || !(beta >= 0.0 && beta < 1e3))
        return ICW_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    if (set_dev(c) || quiesce(c) != hipSuccess) return ICW_EDEVICE;
    for (double *&h : c->fir_hist)
        if (h) { (void)hipFree(h); h = nullptr; }
    if (c->d_fir_g) { (void)hipFree(c->d_fir_g); c->d_fir_g = nullptr; }
    c->fir_M = c->fir_nt = 0;
    c->fir_beta = 0.0;
    c->fir_par = 0;
    if (M == 0) return ICW_OK;
    std::vector<double> g((size_t)(M / 2 + 1) / 2);
    const int nt = icw_fir_taps(M, beta, g.data(), (int)g.size());
    if (nt <= 0) return ICW_EINVAL;
    const size_t hb = (size_t)c->n_streams * 2 * (size_t)M;
    int rc = dalloc(&c->d_fir_g, (size_t)nt);
    rc |= dalloc(&c->fir_hist[0], hb);
    rc |= dalloc(&c->fir_hist[1], hb);
    if (rc != ICW_OK || hipMemcpy(c->d_fir_g, g.data(), (size_t)nt * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) {
        for (double *&h : c->fir_hist)
            if (h) { (void)hipFree(h); h = nullptr; }
        if (c->d_fir_g) { (void)hipFree(c->d_fir_g); c->d_fir_g = nullptr; }
        return rc == ICW_ENOMEM ? ICW_ENOMEM : ICW_EDEVICE;
    }
    c->fir_M = M;
    c->fir_nt = nt;
    c->fir_beta = beta;
    bool ok = fir_clear(c, 0, (size_t)c->n_streams, c->stream);
    ok &= hipStreamSynchronize(c->stream) == hipSuccess;
    return ok ? ICW_OK : ICW_EDEVICE;
}

int icw_stream_reset_framecnt(icw_ctx *c, int s)
{
    if (!c || s < 0 || s >= c->n_streams) return ICW_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    if (set_dev(c)) return ICW_EDEVICE;
    if (quiesce(c) != hipSuccess) return ICW_EDEVICE;
    c->touched = true;
    c->nf_host[s] = 0;
    return hipMemset(c->st.n_frame + s, 0, sizeof(unsigned long long)) == hipSuccess ? ICW_OK : ICW_EDEVICE;
}

int icw_stream_seek(icw_ctx *c, int s, int64_t frame_pos)
{
    if (!c || s < 0 || s >= c->n_streams || frame_pos < 0) return ICW_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    if (set_dev(c)) return ICW_EDEVICE;
    long long v = (long long)frame_pos;
    c->touched = true;
    bool ok = quiesce(c) == hipSuccess;
    ok &= hipMemcpy(c->st.pos + s, &v, sizeof(v), hipMemcpyHostToDevice) == hipSuccess;
    return ok ? ICW_OK : ICW_EDEVICE;
}

int icw_set_input(icw_ctx *c, uint32_t sample_rate, uint32_t fmt, uint32_t channels)
{
    if (!c || sample_rate == 0 || sample_rate > ICW_MAX_FS_SRC || fmt > ICW_FMT_CW_F32 || channels == 0) return ICW_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    if (set_dev(c) || quiesce(c) != hipSuccess) return ICW_EDEVICE;
    c->cfg.sample_rate = sample_rate;
    c->cfg.in_format = fmt;
    c->cfg.in_channels = channels;
    return ICW_OK;
}

/* Live edits: what the reference's GUI thread changes while a decode thread runs
 * applies here from the next call on, to every stream of the context; the running call finishes
 * with the old parameters (quiesce).  Per-stream state carries over as in the reference. */
int icw_set_graph(icw_ctx *c, const icw_node *nodes, int n_nodes, int bypass_list, int *accepted)
{
    if (!c || n_nodes < 0 || (n_nodes > 0 && !nodes)) return ICW_EINVAL;
    std::vector<icw_node> nv(nodes, nodes + n_nodes);
    const bool ok = graph_accept(nv);
    if (accepted) *accepted = ok ? 1 : 0;
    if (!ok) return ICW_EGRAPH;
    std::lock_guard<std::mutex> lk(c->mu);
    if (set_dev(c) || quiesce(c) != hipSuccess) return ICW_EDEVICE;
    /* replace_output_plug (adv_modulator.c:176-209) of the removed / re-plugged nodes, matched by
     * position (include/icw.h): their old output slots read zero from now on */
    std::vector<int> clears;
    for (size_t i = 0; i < c->nodes.size(); ++i) {
        const icw_node &o = c->nodes[i];
        if (o.mode != ICW_MODE_SHIFT && o.mode != ICW_MODE_PM && o.mode != ICW_MODE_MIX) continue;
        if (i >= nv.size() || nv[i].mode != o.mode || nv[i].n_out != o.n_out) clears.push_back(o.n_out);
    }
    return apply_graph(c, nv, bypass_list ? 1 : 0, clears);
}

/* the list primitives (include/icw.h): the reference's own edits, each with replace_output_plug's
 * clear (adv_modulator.c:176-209) and nothing else */
int icw_graph_del_last(icw_ctx *c)
{
    if (!c) return ICW_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    if (set_dev(c) || quiesce(c) != hipSuccess) return ICW_EDEVICE;
    if (c->nodes.size() <= 1) return ICW_OK;                        /* am.tail->prev == NULL */
    std::vector<icw_node> nv(c->nodes.begin(), c->nodes.end() - 1);
    std::vector<int> clears;
    const int r = plug_slot(c->nodes.back());
    if (r >= 0) clears.push_back(r);
    return apply_graph(c, nv, c->cfg.bypass_list, clears);
}

int icw_graph_del_all(icw_ctx *c)
{
    if (!c) return ICW_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    if (set_dev(c) || quiesce(c) != hipSuccess) return ICW_EDEVICE;
    if (c->nodes.size() <= 1) return ICW_OK;
    std::vector<int> clears;
    for (size_t i = c->nodes.size() - 1; i >= 1; --i) {             /* tail first (adv_modulator.c:364-371) */
        const int r = plug_slot(c->nodes[i]);
        if (r >= 0) clears.push_back(r);
    }
    std::vector<icw_node> nv(c->nodes.begin(), c->nodes.begin() + 1);
    return apply_graph(c, nv, c->cfg.bypass_list, clears);
}

int icw_graph_add_last(icw_ctx *c, const icw_node *node)
{
    if (!c || !node) return ICW_EINVAL;
    if (node->mode == ICW_MODE_MASTER) return ICW_EGRAPH;           /* create_node_dsp: NULL */
    std::lock_guard<std::mutex> lk(c->mu);
    std::vector<icw_node> nv(c->nodes);
    nv.push_back(*node);
    if (!graph_accept(nv)) return ICW_EGRAPH;
    if (set_dev(c) || quiesce(c) != hipSuccess) return ICW_EDEVICE;
    return apply_graph(c, nv, c->cfg.bypass_list, std::vector<int>());
}

int icw_graph_set_output_plug(icw_ctx *c, int index, int n)
{
    if (!c || n < -1 || n >= ICW_N_INPUTS || n == 0) return ICW_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    if (index < 0 || index >= (int)c->nodes.size()) return ICW_EINVAL;
    if (set_dev(c) || quiesce(c) != hipSuccess) return ICW_EDEVICE;
    std::vector<icw_node> nv(c->nodes);
    std::vector<int> clears;
    const int r = plug_slot(nv[index]);
    if (r >= 0) {
        clears.push_back(r);
        if (n >= 0) nv[index].n_out = n;
    }
    return apply_graph(c, nv, c->cfg.bypass_list, clears);
}

int icw_clear_bus_slot(icw_ctx *c, int slot)
{
    if (!c || slot < 0 || slot >= ICW_N_INPUTS) return ICW_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    if (set_dev(c) || quiesce(c) != hipSuccess) return ICW_EDEVICE;
    return clear_slot(c, slot);
}

int icw_set_render(icw_ctx *c, const icw_render_cfg *r)
{
    if (!c || !r || !render_cfg_ok(*r)) return ICW_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    if (set_dev(c) || quiesce(c) != hipSuccess) return ICW_EDEVICE;
    IcwRenderK k;
    render_consts(*r, c->cfg.need24bits, k);
    icw_config cfg = c->cfg;
    cfg.render = *r;
    const bool serial = needs_serial(cfg, k, c->prog), rstate = needs_render_state(cfg, k, c->prog);
    int rc;
    if (rstate && (rc = ensure_render_state(c))) return rc;
    if (k.hi != c->rk.hi && !fold_peaks(c)) return ICW_EDEVICE;
    /* sound_render_recalc: prev_rnd, the shaper rings and prev_ns_err start again, the RNG goes on */
    if (c->st.rs && hipMemset(c->st.rs, 0, (size_t)c->n_streams * 2 * ICW_RSTATE * sizeof(double)) != hipSuccess)
        return ICW_EDEVICE;
    c->cfg.render = *r;
    c->rk = k;
    c->serial_render = serial;
    c->render_state = rstate;
    return ICW_OK;
}

/* sound_render_set_outbits (sound_render.c:617-621) on both renders of every stream, as
 * mod_context_fopen applies the.cfg.need24bits at every track open (in_cwave.c:212, 233-234): the
 * new bounds, norm_mul and norm_shift, then sound_render_recalc (prev_rnd, the shaper rings and
 * prev_ns_err restart; the MT19937 generators go on).  Applied even when the depth is unchanged,
 * since recalc runs either way. */
int icw_set_outbits(icw_ctx *c, int need24bits)
{
    if (!c) return ICW_EINVAL;
    const int is24 = need24bits ? 1 : 0;
    std::lock_guard<std::mutex> lk(c->mu);
    if (set_dev(c) || quiesce(c) != hipSuccess) return ICW_EDEVICE;
    IcwRenderK k;
    render_consts(c->cfg.render, is24, k);
    icw_config cfg = c->cfg;
    cfg.need24bits = is24;
    const bool serial = needs_serial(cfg, k, c->prog), rstate = needs_render_state(cfg, k, c->prog);
    int rc;
    if (rstate && (rc = ensure_render_state(c))) return rc;
    /* peaks so far in dB against the old bound (sound_render.c:769-780 converts each sample with the
     * bound of its time) */
    if (k.hi != c->rk.hi && !fold_peaks(c)) return ICW_EDEVICE;
    if (c->st.rs && hipMemset(c->st.rs, 0, (size_t)c->n_streams * 2 * ICW_RSTATE * sizeof(double)) != hipSuccess)
        return ICW_EDEVICE;
    c->cfg.need24bits = is24;
    c->rk = k;
    c->serial_render = serial;
    c->render_state = rstate;
    return ICW_OK;
}

int icw_set_hilbert_filter(icw_ctx *c, uint32_t type)
{
    if (!c || type > 5) return ICW_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    if (type == c->cfg.hilbert_type) return ICW_OK;
    if (set_dev(c) || quiesce(c) != hipSuccess) return ICW_EDEVICE;
    /* hq_rp_create: zero rings, ring index 0, counters 0, phase 0 -- for every stream */
    const size_t S = (size_t)c->n_streams;
    DevState &s = c->st;
    bool ok = hipMemset(s.hist, 0, S * 4 * ICW_HIST_PITCH * sizeof(double)) == hipSuccess;
    ok &= hipMemset(s.sncnt, 0, S * 4 * sizeof(unsigned long long)) == hipSuccess;
    ok &= hipMemset(s.hq_phase, 0, S * 2 * sizeof(uint32_t)) == hipSuccess;
    ok &= hipMemsetD32((hipDeviceptr_t)s.lr_equal, 1, S * 2) == hipSuccess;
    if (!ok) return ICW_EDEVICE;
    c->lr_known.assign(S, 1);
    c->cfg.hilbert_type = type;
    set_filter(c);
    return ICW_OK;
}

int icw_set_hilbert_config(icw_ctx *c, int kahan, int subnorm_reject)
{
    if (!c) return ICW_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    if (set_dev(c) || quiesce(c) != hipSuccess) return ICW_EDEVICE;
    /* iir_rp_setcfg: the rings stay, the de-subnorm counters start again ("new world") */
    if (hipMemset(c->st.sncnt, 0, (size_t)c->n_streams * 4 * sizeof(unsigned long long)) != hipSuccess)
        return ICW_EDEVICE;
    c->cfg.iir_kahan = kahan ? 1 : 0;
    c->cfg.iir_subnorm_reject = subnorm_reject ? 1 : 0;
    return ICW_OK;
}

int icw_render_size(const icw_ctx *c) { return c ? (c->cfg.need24bits ? 3 : 2) : ICW_EINVAL; }

int icw_process_streams(icw_ctx *c, int first, int count, const void *in, size_t in_stride, void *out,
                        size_t out_stride, int n_frames, unsigned flags, void *dbg, void *hip_stream)
{
    if (!c || first < 0 || count <= 0 || first + count > c->n_streams || n_frames < 0 || !in || !out)
        return ICW_EINVAL;
    if (n_frames == 0) return ICW_OK;
    std::lock_guard<std::mutex> lk(c->mu);
    if (set_dev(c)) return ICW_EDEVICE;
    ++c->calls;
    hipStream_t st = hip_stream ? (hipStream_t)hip_stream : c->stream;
    /* A NULL handle with device pointers means the legacy default stream (torch's default stream):
     * the call starts after the work already queued there, and returns when its results are in
     * place, so that stream's later work sees them.  The end is a host wait, not an operation on the
     * null stream: a null-stream wait behind the context's CU-masked streams cost C2 13-25 % (its
     * implicit synchronisation with every blocking stream serialises the block pipeline). */
    const bool legacy = !hip_stream && (flags & ICW_F_DEVICE_PTRS);
    if (legacy && (hipEventRecord(c->join, nullptr) != hipSuccess || hipStreamWaitEvent(st, c->join, 0) != hipSuccess))
        return ICW_EDEVICE;
    const icw_config &cfg = c->cfg;
    const unsigned csz = fmt_size(cfg.in_format);
    const unsigned nch = cfg.in_channels;
    const unsigned fsz = csz * nch;
    const int osz = 2 * (cfg.need24bits ? 3 : 2);
    const bool dev = flags & ICW_F_DEVICE_PTRS;
    const bool timing = flags & 4u;
    /* ICW_F_DEBUG_INPUT: K0's output of every launch block is copied aside (test hook, host dbg) */
    const bool xin = flags & ICW_F_DEBUG_INPUT;
    if (xin && (dev || !dbg || (flags & ICW_F_DEBUG_PRE) || c->cfg.in_format >= ICW_FMT_CW_F64 || c->fir_M > 0 ||
                c->cfg.fp_check))
        return ICW_EINVAL;
    const size_t S = (size_t)count;
    if (!dev && (in_stride < (size_t)n_frames * fsz || out_stride < (size_t)n_frames * osz)) return ICW_EINVAL;

    /* FIR Hilbert converter (icw_set_fir_hilbert): real input becomes complex samples in KF and
     * the block continues as CWAVE input does */
    const bool fir = c->fir_M > 0 && cfg.in_format < ICW_FMT_CW_F64;
    const bool cw = cfg.in_format >= ICW_FMT_CW_F64 || fir;
    const bool bus = c->prog.is_bus;
    /* mono dedup: every stream of the call known to hold identical left / right converters */
    const bool fcm = c->cfg.fp_check != 0;                /* FP_CHECK: FC() kernels, no shortcuts */
    bool dedup = !cw && !fcm && nch == 1 && c->dedup_ok && (c->k1_mode <= 0 || c->k1_mode == 3);   /* plain / row K1 */
    for (int i = 0; dedup && i < count; ++i) dedup = c->lr_known[first + i] != 0;
    /* K1 variant of this call.  Auto: the row-broadcast kernel (4 chains per wave, ~17 % fewer
     * instructions per sample) when its waves fit k1_wpc per CU on at most half the chip, else the
     * lane-per-chain kernel (64 chains per wave).  The row kernel needs Kahan + the reject.  (Round
     * 1 kept it off with a serial render; with the partition working, C5 gains 9 % from it.) */
    const int row_waves = (int)(((dedup ? count : 2L * count) + 3) / 4) * 2;
    const bool row_ok = cfg.iir_kahan && cfg.iir_subnorm_reject;
    int k1_mode = c->k1_mode;
    if (k1_mode < 0) k1_mode = (row_ok && row_waves <= (c->n_cu / 2) * c->k1_wpc) ? 3 : 0;
    if (k1_mode == 3 && !row_ok) k1_mode = 0;
    if (fcm) k1_mode = ICW_K1_FC;
    if (!cw) c->last_k1 = k1_mode;
    /* launch blocks.  The tail taper (plan_blocks) is on by default where it fits: a small batch
     * (the row kernel K1r) with a serial render -- its drain is the render of the last block, and
     * the frame-parallel kernels take well under K1r's time per frame (C5: +2 %).  Large batches
     * keep uniform blocks (K0 + K2 take ~0.9 of K1's time there), ICW_TAPER overrides. */
    /* FIR converter: fused with the graph and render (KF2, one kernel per block) where its LDS fits;
     * else KF on its own stream (the caller's: K1's, idle without the IIR) beside K2.  KF2 needs no
     * block scratch and has no recurrence to pipeline against, so its blocks are as long as the
     * scratch bound allows (fewer launches, fewer partly filled waves of workgroups at their ends) */
    const bool fir_fused = fir && c->fir_fuse &&
                           icw_fir_graph_lds(c->fir_M, c->fir_nt, (int)nch, c->prog.chain ? 0 : c->prog.n_regs) > 0 &&
                           !c->prog.is_bus;
    /* The row kernel without a serial render (C2) has K2 at ~0.16 of K1r's time per frame: 65 536-frame
     * blocks (a quarter of the launches, of their gaps and prologues) ending in a steep tail
     * (65 536 -> 16 384 -> 4 096 -> 1 024: the drain stays one short K2) measured +0.8 % on C2
     * (3 170 -> 3 196 Msamples/s; 32 768 with r = 0.5 +0.5 %, 65 536 with no tail +0.5 %). */
    const bool row_long = !cw && k1_mode == 3 && !c->serial_render && !c->block_env && n_frames >= 4 * kMaxBlockFrames;
    /* a dithered render with the flat shaper, rendered frame-parallel in the output kernel (K2 / KF2 /
     * K5) from K3a's dither rows (needs_serial) */
    const bool dith_par = !c->serial_render && cfg.render.render_type != ICW_RENDER_ROUND;
    /* (with a dither generator, blocks of kMaxBlockFrames let K3a of the next block run beside KF2) */
    const bool fir_long = fir_fused && dev && !c->serial_render && !bus && !dith_par;
    const int Tb = std::min(n_frames, ((fir_fused || row_long) && !c->block_env)
                                          ? (fir_long ? kMaxFirBlockFrames : kMaxBlockFrames) : c->max_block);
    const double taper = c->taper >= 0.0 ? c->taper
                       : (!cw && k1_mode == 3) ? (c->serial_render ? kAutoTaper : (row_long ? kRowTaper : 0.0)) : 0.0;
    /* the fused FIR converter with a serial render (c5fir): the render of block 0 waits for its
     * converter and dither alone, so block 0 is short and the next ones ramp up (kFirRenderRamp:
     * profiles/r04_c5fir_timeline_after.txt had 2.2 ms of fill in a 24.3 ms step) */
    const bool fir_ramp = fir_fused && c->serial_render && !c->block_env && c->first_block > 0;
    const std::vector<std::pair<int, int>> blocks =
        fir_ramp ? plan_blocks(n_frames, Tb, c->first_block_env ? c->first_block : kFirRenderFirst, 0.0, c->taper_min,
                               c->fir_ramp > 0.0 ? c->fir_ramp : kFirRenderRamp)
                 : plan_blocks(n_frames, Tb, fir_fused ? 0 : c->first_block, taper, c->taper_min);
    const int n_blocks = (int)blocks.size();
    /* K5 (icw_stream1): one stream, one block, the row recurrence, register-form graph, ROUND / flat */
    const bool s1 = c->stream1 && count == 1 && n_blocks == 1 && !cw && !fcm && k1_mode == 3 && !c->serial_render &&
                    !bus && n_frames <= ICW_S1_MAX && !xin;

    const unsigned char *d_in;
    unsigned char *d_out;
    size_t dis, dos;
    /* a small host-pointer call stages through pinned memory (asynchronous copies, one wait) */
    const size_t stage_in = (size_t)n_frames * fsz * S, stage_out = (size_t)n_frames * osz * S;
    const bool pinned = !dev && stage_in + stage_out + 16 <= kPinnedStage;
    /* pinned host buffers on a call of several launch blocks: each block's input slice goes in and
     * its output slice comes out on the copy stream, beside the other blocks' kernels */
    const bool pipe_io = !dev && !pinned && n_blocks > 1 && !c->serialize && host_pinned(in, c->device) && host_pinned(out, c->device);
    bool zcopy = false;
    if (pinned) {
        if (c->h_stage_bytes < stage_in + stage_out + 16) {
            if (c->h_stage) (void)hipHostFree(c->h_stage);
            c->h_stage = nullptr;
            c->h_stage_bytes = 0;
            if (hipHostMalloc((void **)&c->h_stage, kPinnedStage, hipHostMallocDefault) != hipSuccess) return ICW_ENOMEM;
            c->h_stage_bytes = kPinnedStage;
            void *dp = nullptr;
            c->h_stage_dev = hipHostGetDevicePointer(&dp, c->h_stage, 0) == hipSuccess ? (unsigned char *)dp : nullptr;
            if (!c->h_stage_dev) (void)hipGetLastError();
        }
        zcopy = c->zero_copy && c->h_stage_dev && !(flags & ICW_F_DEBUG_PRE);
    }
    if (dev) {
        d_in = (const unsigned char *)in;
        d_out = (unsigned char *)out;
        dis = in_stride;
        dos = out_stride;
    } else {
        dis = (size_t)n_frames * fsz;
        dos = (size_t)n_frames * osz;
        if (grow((void **)&c->d_in, &c->d_in_bytes, dis * S)) return ICW_ENOMEM;
        if (grow((void **)&c->d_out, &c->d_out_bytes, dos * S + 16)) return ICW_ENOMEM;
        if (pinned) {
            for (size_t i = 0; i < S; ++i)
                memcpy(c->h_stage + i * dis, (const unsigned char *)in + i * in_stride, dis);
            if (!zcopy && hipMemcpyAsync(c->d_in, c->h_stage, dis * S, hipMemcpyHostToDevice, st) != hipSuccess)
                return ICW_EDEVICE;
        } else if (!pipe_io &&
                   hipMemcpy2DAsync(c->d_in, dis, in, in_stride, dis, S, hipMemcpyHostToDevice, st) != hipSuccess) {
            return ICW_EDEVICE;
        }
        /* zero copy: K0 reads the staged input across PCIe and the last kernel writes the output
         * (and icw_advance the error flag) straight into the staging buffer -- a few KB, where the
         * two DMA transfers each cost a setup latency (the 576-frame drop-in) */
        d_in = zcopy ? c->h_stage_dev : c->d_in;
        d_out = zcopy ? c->h_stage_dev + stage_in : c->d_out;
    }
    /* K5 on the zero-copy buffer: the kernel stores the call's sequence number after its output and
     * the host polls for it -- no completion signal and no waking of a waiting thread.  The word is
     * 4-byte aligned inside the output's 16 spare bytes, after the error flag. */
    const bool s1_poll = s1 && zcopy && c->spin_wait && !timing && !c->s1_stamps;
    const size_t done_off = ((stage_in + dos * S + sizeof(int) + 3) & ~(size_t)3) - stage_in;
    uint32_t s1_seq = 0u;
    if (s1_poll) {
        if (++c->s1_seq == 0u) ++c->s1_seq;           /* 0 is never a call's number */
        s1_seq = c->s1_seq;
        /* the word sits in the reused staging buffer, where an earlier, larger call may have left
         * input or output bytes that happen to equal this call's number: store a value that cannot
         * match before the launch (which orders after this store), so the poll sees only the
         * kernel's own store */
        __atomic_store_n((uint32_t *)(c->h_stage + stage_in + done_off), ~s1_seq, __ATOMIC_RELEASE);
    }
    std::vector<uint32_t> xin_phase;
    if (xin) {
        if (grow((void **)&c->d_xin, &c->d_xin_bytes, S * 2 * (size_t)n_frames * sizeof(double))) return ICW_ENOMEM;
        xin_phase.resize(S * 2);
        if (hipMemcpyAsync(xin_phase.data(), ds_phase_of(c, first), S * 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, st) !=
                hipSuccess || hipStreamSynchronize(st) != hipSuccess)
            return ICW_EDEVICE;
    }
    double *d_pre = nullptr;
    if (flags & ICW_F_DEBUG_PRE) {
        if (!dbg) return ICW_EINVAL;
        if (dev) d_pre = (double *)dbg;
        else {
            if (grow((void **)&c->d_pre, &c->d_pre_bytes, S * (size_t)n_frames * 2 * sizeof(double))) return ICW_ENOMEM;
            d_pre = c->d_pre;
        }
    }

    const int N = c->nord;
    const size_t w_pitch = (size_t)Tb + N + 1;
    const size_t x_pitch = ((size_t)Tb + ICW_MAX_IIR_ORDER + 2) & ~(size_t)1;   /* look-ahead pad */
    const int n_sets = std::min(n_blocks, c->max_sets);
    for (int p = 0; p < n_sets && !fir_fused; ++p) {
        if (!cw && grow((void **)&c->w[p], &c->w_bytes[p], S * 4 * w_pitch * sizeof(double))) return ICW_ENOMEM;
        if (grow((void **)&c->xd[p], &c->xd_bytes[p], S * 4 * x_pitch * sizeof(double))) return ICW_ENOMEM;
    }
    if (c->serial_render && !d_pre)
        for (int p = 0; p < n_sets; ++p)
            if (grow((void **)&c->rpre[p], &c->rpre_bytes[p], S * (size_t)Tb * 2 * sizeof(double))) return ICW_ENOMEM;
    /* the shared rotation table pays from two streams on; one stream computes its factors inline */
    const bool table = c->prog.needs_omega && !bus && c->prog.n_trig > 0 && count > 1;
    bool in_step = table;
    for (int i = 1; in_step && i < count; ++i) in_step = c->nf_host[first + i] == c->nf_host[first];
    if (table && grow((void **)&c->trig, &c->trig_bytes, (size_t)((Tb + 7) & ~7) * 2 * c->prog.n_trig * sizeof(double)))
        return ICW_ENOMEM;
    if (bus)
        for (int p = 0; p < n_sets; ++p)
            if (grow((void **)&c->iq[p], &c->iq_bytes[p], S * (size_t)Tb * 4 * sizeof(double))) return ICW_ENOMEM;
    const bool dither = cfg.render.render_type != ICW_RENDER_ROUND;     /* K3a: serial or frame-parallel render */
    if (dither)
        for (int p = 0; p < n_sets; ++p)
            if (grow((void **)&c->dith[p], &c->dith_bytes[p], S * 2 * (size_t)(Tb + 1) * sizeof(double))) return ICW_ENOMEM;
    if (dither && !c->dither_coop && !c->dither_lane) {
        /* chunk rows of at most 2^26 words in all (256 MB), at least 1 024 frames of the widest draw (GAUSS,
         * 24 words per sample), at most the block's */
        const size_t G = S * 2;
        size_t cap = std::max<size_t>(((size_t)1 << 26) / G, (size_t)24 * 1024);
        cap = std::min(cap, (size_t)24 * (size_t)(Tb + 1));
        cap = (cap + 3) & ~(size_t)3;                      /* rows 16-byte aligned */
        if (grow((void **)&c->dwords, &c->dwords_bytes, G * cap * 4) ||
            grow((void **)&c->dbk, &c->dbk_bytes, G * ICW_DBK * 4) ||
            grow((void **)&c->dflag, &c->dflag_bytes, G * 4))
            return ICW_ENOMEM;
        c->dwcap = cap;
    }

    /* Streams.  sK runs the IIR state kernel K1 (the serial, issue-bound one); sA runs the input
     * prep K0, the output kernel K2 and the serial graph / render; sD the dither generator.  When
     * K1 needs few CUs (4 waves per CU, one per SIMD) sK is confined to those CUs and sA / sD to
     * the rest, so the frame-parallel kernels never share a SIMD with a recurrence. */
    hipStream_t sK = st, sA = c->stream2, sD = c->stream3, sR = c->stream4;
    /* sF: an unmasked stream for the pipeline's fill and drain under the CU partition -- K0 of the
     * first block and K2 of the last run while no recurrence does, so they get the whole chip
     * instead of the partition's share (C3 / C4: the drain was one partitioned K2, ~5 % of a step) */
    hipStream_t sF = nullptr;
    /* One launch block: K0 -> K1 -> K2 run in sequence anyway, so everything goes on the caller's
     * stream -- no cross-stream event waits, which cost the 576-frame drop-in call ~135 us (C1
     * p50 361 -> 226 us per call). */
    if (c->serialize || n_blocks == 1) {
        sA = sD = sR = st;
    } else if (!cw) {
        /* plain K1: 128-lane groups of 32 streams (64 with the dedup); the variants: a lane per chain */
        const int k1_waves = (k1_mode == 0 || k1_mode == ICW_K1_FC) ? ((count + (dedup ? 63 : 31)) / (dedup ? 64 : 32)) * 2
                           : row_waves;
        constexpr int kXcd = 8;                               /* MI355X: 8 XCDs */
        const int k1_cus = ((k1_waves + c->k1_wpc - 1) / c->k1_wpc + kXcd - 1) / kXcd * kXcd;
        if (c->cu_split && !c->k1_lds && k1_cus * 2 <= c->n_cu) {
            const CuSplit *cs = cu_split(c, k1_cus);
            if (!cs) return ICW_EDEVICE;
            sK = cs->k1;
            sA = cs->rest;
            sD = cs->dith;
            sR = cs->render;
            if (c->fill_drain) sF = c->stream2;
        }
    } else {
        /* complex input or the FIR converter: no recurrence kernel, so the dither generator runs after
         * the converter / output kernel on sA, beside the serial render of the previous block on sR.
         * On its own stream it shared a hardware queue with the render (4 queues per process,
         * GPU_MAX_HW_QUEUES, streams dealt round-robin): K3a of block b + 1 waited for K3r of block b,
         * 1.2 of every 6.7 ms per c5fir block (profiles/r04_c5fir_timeline.txt).  With a frame-parallel
         * render (no render stream) it gets a stream of its own, ahead of the converter. */
        sD = dith_par ? c->stream3 : sA;
    }
    hipStream_t sC = pipe_io ? c->stream_io : nullptr;
    if (pipe_io && (int)c->ev_io.size() < n_blocks) {
        while ((int)c->ev_io.size() < n_blocks) {
            hipEvent_t e;
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return ICW_EDEVICE;
            c->ev_io.push_back(e);
        }
    }
    /* every stream starts after everything already queued on st (inputs, previous calls); a call
     * whose kernels all run on st (one launch block: the drop-in) records no event -- the marker
     * packet sat in front of its kernel on the queue */
    bool other = false;
    for (hipStream_t x : {sK, sA, sD, sR, sF, sC}) other = other || (x && x != st);
    if (other && hipEventRecord(c->join, st) != hipSuccess)
        return ICW_EDEVICE;
    for (hipStream_t x : {sK, sA, sD, sR, sF, sC})
        if (x && x != st && hipStreamWaitEvent(x, c->join, 0) != hipSuccess) return ICW_EDEVICE;

    DevState &ds = c->st;
    const size_t f0 = (size_t)first;
    if (timing && (int)c->ev.size() < 4 * n_blocks) {
        while ((int)c->ev.size() < 4 * n_blocks) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return ICW_EDEVICE;
            c->ev.push_back(e);
        }
    }
    const unsigned long long ssr = (unsigned long long)cfg.sample_rate * ICW_HZ_SCALE;

    const bool fir_async = fir && !fir_fused && sK != sA;
    /* KF's arguments for launch block b; it reads the history buffer the previous block wrote
     * (same stream, block order) and writes the other one */
    auto fir_args = [&](int b) {
        IcwFirArgs af;
        memset(&af, 0, sizeof(af));
        af.in = d_in + (size_t)blocks[b].first * fsz;
        af.in_stride = dis;
        af.fmt = cfg.in_format;
        af.csz = csz;
        af.fsz = fsz;
        af.nch = nch;
        af.n_streams = count;
        af.T = blocks[b].second;
        af.t0 = blocks[b].first;
        af.pos = ds.pos + f0;
        af.fade = ds.fade + f0 * 3;
        af.M = c->fir_M;
        af.nt = c->fir_nt;
        af.g = c->d_fir_g;
        const size_t hrow = 2 * (size_t)c->fir_M;
        af.hist_in = c->fir_hist[(c->fir_par + b) & 1] + f0 * hrow;
        af.hist_out = c->fir_hist[(c->fir_par + b + 1) & 1] + f0 * hrow;
        af.xd = c->xd[b % n_sets];
        af.x_pitch = x_pitch;
        af.sig = c->prog.chain ? c->prog.sig : 0;
        {
            /* mono input through a Master-only chain (signature count 1, mode MASTER, chain_in `in`:
             * ICW_SIG_M in icw_kernels.hip) whose gains are bit-identical: L and R are one computation */
            const IcwOp &m = c->prog.ops[0];
            af.lr_same = nch == 1 && c->prog.chain && (c->prog.sig & ~(1 << 30)) == 0x41 &&
                         !memcmp(&m.gain[0], &m.gain[1], sizeof(double)) && m.unit_gain[0] == m.unit_gain[1];
        }
        return af;
    };
    /* pinned host input: block b's input slice of every stream goes in on the copy stream, and the
     * stream of the block's first reader (K0, KF or the fused KF2) waits for it */
    auto io_in = [&](int b, hipStream_t s0) -> int {
        if (!pipe_io) return ICW_OK;
        const int t0 = blocks[b].first, T = blocks[b].second;
        if (hipMemcpy2DAsync(c->d_in + (size_t)t0 * fsz, dis, (const unsigned char *)in + (size_t)t0 * fsz, in_stride,
                             (size_t)T * fsz, S, hipMemcpyHostToDevice, sC) != hipSuccess ||
            hipEventRecord(c->ev_io[b], sC) != hipSuccess || hipStreamWaitEvent(s0, c->ev_io[b], 0) != hipSuccess)
            return ICW_EDEVICE;
        return ICW_OK;
    };
    /* K0 of block b on sA: xd[p] was last read by K1 of block b-2 (and, complex input, by K2 of
     * block b-2, which precedes it on sA) */
    auto k0_args = [&](int b) {
        const int t0 = blocks[b].first, T = blocks[b].second, p = b % n_sets;
        IcwK0Args a0;
        memset(&a0, 0, sizeof(a0));
        a0.lds_guard = c->k1_lds ? 256u : 0u;
        a0.in = d_in + (size_t)t0 * fsz;
        a0.in_stride = dis;
        a0.fmt = cfg.in_format;
        a0.csz = csz;
        a0.fsz = fsz;
        a0.nch = nch;
        a0.n_streams = count;
        a0.T = T;
        a0.t0 = t0;
        a0.pos = ds.pos + f0;
        a0.fade = ds.fade + f0 * 3;
        a0.hq_phase = ds.hq_phase + f0 * 2;
        a0.xd = c->xd[p];
        a0.x_pitch = x_pitch;
        a0.dedup = dedup ? 1 : 0;
        return a0;
    };
    auto launch_k0 = [&](int b) -> int {
        if (fir_fused) return ICW_OK;                   /* KF2 converts inside the block's kernel */
        const int p = b % n_sets;
        const IcwK0Args a0 = k0_args(b);
        if (b >= n_sets && !cw && sK != sA && hipStreamWaitEvent(sA, c->k1done[p], 0) != hipSuccess) return ICW_EDEVICE;
        hipStream_t s0 = (b == 0 && sF) ? sF : sA;         /* the fill: nothing else runs yet */
        /* the FIR converter runs on the caller's stream (K1's, idle without the IIR), so KF of the
         * next block overlaps K2 of this one; it rewrites xd[p] after K2(b - n_sets) has read it */
        if (fir_async) {
            s0 = sK;
            if (b >= n_sets && hipStreamWaitEvent(sK, c->k2done[p], 0) != hipSuccess) return ICW_EDEVICE;
        }
        if (io_in(b, s0) != ICW_OK) return ICW_EDEVICE;
        if (fir) {
            IcwFirArgs af = fir_args(b);
            if (timing && hipEventRecord(c->ev[4 * b], s0) != hipSuccess) return ICW_EDEVICE;
            if (icw_launch_fir(&af, s0) != hipSuccess) return ICW_EDEVICE;
            if (timing && hipEventRecord(c->ev[4 * b + 1], s0) != hipSuccess) return ICW_EDEVICE;
        } else if (icw_launch_unpack(&a0, s0) != hipSuccess) {
            return ICW_EDEVICE;
        }
        /* test hook: this block's rows aside before K1 may start (K1 waits for k0done) */
        if (xin && hipMemcpy2DAsync(c->d_xin + a0.t0, (size_t)n_frames * sizeof(double), a0.xd, x_pitch * sizeof(double),
                                    (size_t)a0.T * sizeof(double), S * 2, hipMemcpyDeviceToDevice, s0) != hipSuccess)
            return ICW_EDEVICE;
        if (hipEventRecord(c->k0done[p], s0) != hipSuccess) return ICW_EDEVICE;
        return ICW_OK;
    };

    auto k1_args = [&](int b) {
        const int p = b % n_sets;
        IcwK1Args a1;
        memset(&a1, 0, sizeof(a1));
        a1.xd = c->xd[p];
        a1.x_pitch = x_pitch;
        a1.nch = nch;
        a1.n_streams = count;
        a1.n_chains = count * 4;
        a1.T = blocks[b].second;
        a1.hist = ds.hist + f0 * 4 * ICW_HIST_PITCH;
        a1.sncnt = ds.sncnt + f0 * 4;
        a1.err = ds.err;
        a1.w = c->w[p];
        a1.w_pitch = w_pitch;
        a1.lr_equal = ds.lr_equal + f0 * 2;
        a1.hq_phase = ds.hq_phase + f0 * 2;
        a1.t0 = blocks[b].first;
        a1.info_dup = c->info_dup[p];
        memcpy(a1.pc, c->pc, sizeof(a1.pc));
        a1.wg_waves = c->k1_lds ? 4 : (c->k1_wg_env || k1_mode != 3) ? c->k1_wg : 2;
        a1.lds_hold = c->k1_lds ? c->lds_cu : 0;
        a1.dedup = dedup ? 1 : 0;
        a1.fes = fcm ? ds.fes + f0 * 4 * ICW_FES_PITCH : nullptr;
        return a1;
    };
    auto k2_args = [&](int b) {
        const int t0 = blocks[b].first, T = blocks[b].second, p = b % n_sets;
        IcwK2Args a2;
        memset(&a2, 0, sizeof(a2));
        a2.w = c->w[p];
        a2.w_pitch = w_pitch;
        a2.n_streams = count;
        a2.T = T;
        a2.n_chains = count * 4;
        a2.nch = nch;
        a2.t0 = t0;
        a2.hq_phase = ds.hq_phase + f0 * 2;
        a2.n_frame = ds.n_frame + f0;
        a2.ssr = ssr;
        a2.scaled = cfg.frmod_scaled;
        a2.sample_rate = cfg.sample_rate;
        a2.prog = c->d_prog;
        a2.bus = ds.bus + f0 * ICW_N_INPUTS * 4;
        a2.out = d_out + (size_t)t0 * osz;
        a2.out_stride = dos;
        if (d_pre) {
            a2.pre = d_pre + (size_t)t0 * 2;
            a2.pre_stride = (size_t)n_frames * 2;
        } else if (c->serial_render) {
            a2.pre = c->rpre[p];
            a2.pre_stride = (size_t)T * 2;
        }
        a2.do_render = c->serial_render ? 0 : 1;
        a2.n_regs = c->prog.chain ? 0 : c->prog.n_regs;    /* a chain program keeps its values in VGPRs */
        a2.clips = ds.clips + f0 * 2;
        a2.peak_bits = ds.peak_bits + f0 * 2;
        a2.rk = c->rk;
        memcpy(a2.pc, c->pc, sizeof(a2.pc));
        memcpy(a2.pd, c->pd, sizeof(a2.pd));
        a2.d0 = c->d0;
        a2.cw = cw ? 1 : 0;
        a2.info_dup = cw ? nullptr : c->info_dup[p];
        a2.xin = c->xd[p];
        a2.x_pitch = x_pitch;
        if (bus) a2.iq_out = c->iq[p];
        a2.trig = c->prog.needs_omega;
        a2.sncnt = (!cw && cfg.iir_subnorm_reject) ? ds.sncnt + f0 * 4 : nullptr;
        a2.fes = fcm ? ds.fes + f0 * 4 * ICW_FES_PITCH : nullptr;
        return a2;
    };
    /* the dither generator's / serial render's arguments for block b */
    auto k3_args = [&](int b, const IcwK2Args &a2) {
        const int T = blocks[b].second, p = b % n_sets;
        IcwK3Args a3;
        memset(&a3, 0, sizeof(a3));
        a3.pre = a2.pre;
        a3.pre_stride = a2.pre_stride;
        a3.n_streams = count;
        a3.T = T;
        a3.out = a2.out;
        a3.out_stride = dos;
        a3.mt = ds.mt + f0 * 2;          /* column offset: [624][G] layout, pitch G */
        a3.mt_idx = ds.mt_idx + f0 * 2;
        a3.rs = ds.rs + f0 * 2 * ICW_RSTATE;
        a3.clips = ds.clips + f0 * 2;
        a3.peak_bits = ds.peak_bits + f0 * 2;
        a3.n_gen = count * 2;
        a3.mt_pitch = c->n_streams * 2;
        a3.rk = c->rk;
        a3.fes = fcm ? ds.fes + f0 * 4 * ICW_FES_PITCH : nullptr;
        /* the row-broadcast render (16 lanes per channel) while its waves stay few; FP_CHECK
         * keeps the compact lane-per-channel form */
        a3.row = c->serial_render && !fcm && (c->render_row == 1 || (c->render_row < 0 && a3.n_gen <= kRowRenderMax)) ? 1 : 0;
        a3.comp = a3.row && c->k3r_comp;
        a3.err = ds.err;
        if (dither) {
            a3.dith = c->dith[p];
            /* the row render and the frame-parallel one read runs of one channel: generator-major
             * [count*2][T rounded up to even] (16-byte pairs); the lane-per-channel renders time-major
             * [T][count*2] */
            a3.dith_gm = (a3.row || !c->serial_render) ? 1 : 0;
            a3.dith_pitch = a3.dith_gm ? (size_t)(T + (T & 1)) : (size_t)count * 2;
            if (!c->dither_coop && !c->dither_lane) {
                a3.wbuf = c->dwords;
                a3.wpitch = a3.wcap = c->dwcap;
                a3.dflag = c->dflag;
                a3.dbk = c->dbk;
            }
        }
        return a3;
    };
    auto adv_args = [&]() {
        IcwAdvArgs av;
        memset(&av, 0, sizeof(av));
        av.lds_guard = c->k1_lds ? 256u : 0u;
        av.n_streams = count;
        av.cw = cw ? 1 : 0;
        av.n = n_frames;
        av.hq_phase = ds.hq_phase + f0 * 2;
        av.pos = ds.pos + f0;
        av.n_frame = ds.n_frame + f0;
        av.ssr = ssr;
        av.scaled = cfg.frmod_scaled;
        if (pinned) {
            av.err = ds.err;
            av.err_copy = (int *)(d_out + dos * S);        /* the output buffer has 16 spare bytes */
        }
        if (s1_poll) {
            av.done = (uint32_t *)(d_out + done_off);
            av.seq = s1_seq;
        }
        return av;
    };
    /* K5: a one-stream call of one block (the drop-in's 576-frame calls, playback.c:619) runs its four
     * kernels as phases of one workgroup (icw_stream1): no launch gaps, one launch per call */
    if (s1) {
        IcwS1Args a5;
        memset(&a5, 0, sizeof(a5));
        a5.k0 = k0_args(0);
        a5.k1 = k1_args(0);
        a5.k2 = k2_args(0);
        a5.adv = adv_args();
        a5.stamps = c->s1_stamps;
        a5.ovl = c->s1_ovl ? 1 : 0;
        if (c->prog.needs_omega && c->prog.n_trig > 0 && !bus) {
            /* the one stream's rotation factors, computed by the kernel's idle waves beside the
             * recurrence: the output phase reads them instead of evaluating sin / cos per frame */
            if (grow((void **)&c->trig, &c->trig_bytes, (size_t)n_frames * 2 * c->prog.n_trig * sizeof(double)))
                return ICW_ENOMEM;
            IcwTrigArgs &at = a5.trig;
            at.prog = c->d_prog;
            at.n_frame = ds.n_frame + f0;
            at.t0 = 0;
            at.T = n_frames;
            at.scaled = cfg.frmod_scaled;
            at.trig_pitch = 2 * c->prog.n_trig;
            at.ssr = ssr;
            at.sample_rate = cfg.sample_rate;
            at.tab = c->trig;
            a5.has_trig = 1;
            a5.k2.trig_tab = c->trig;
            a5.k2.trig_pitch = at.trig_pitch;
        }
        if (dith_par) {
            /* the dithered flat render: K3a of the call's block first, on the same stream */
            const IcwK3Args a3 = k3_args(0, a5.k2);
            if ((c->dither_lane ? icw_launch_dither_lane(&a3, st) : icw_launch_dither(&a3, st)) != hipSuccess)
                return ICW_EDEVICE;
            a5.k2.dith = a3.dith;
            a5.k2.dith_pitch = a3.dith_pitch;
        }
        if (timing && hipEventRecord(c->ev[0], st) != hipSuccess) return ICW_EDEVICE;
        if (icw_launch_stream1(&a5, N, st) != hipSuccess) return ICW_EDEVICE;
        if (timing && (hipEventRecord(c->ev[1], st) != hipSuccess || hipEventRecord(c->ev[2], st) != hipSuccess ||
                       hipEventRecord(c->ev[3], st) != hipSuccess))
            return ICW_EDEVICE;
        if (!cw && nch > 1) c->lr_known[first] = 0;
    } else {
    /* n_sets scratch sets (2 by default, ICW_SETS=3): K0 of the first n_sets blocks is queued up
     * front, K0(b + n_sets) as soon as its xd set is free (below); K1(b + n_sets) reuses the w /
     * info_dup set that K2(b) read and waits for it.  Three sets measured slower for large
     * batches (C3: K1 3.96 vs 3.16 ms per launch), so two is the default. */
    int rc0 = ICW_OK;
    for (int b = 0; b < n_sets; ++b)
        if ((rc0 = launch_k0(b)) != ICW_OK) return rc0;
    for (int b = 0; b < n_blocks; ++b) {
        const int t0 = blocks[b].first;
        const int T = blocks[b].second;
        const int p = b % n_sets;

        if (!cw) {
            const IcwK1Args a1 = k1_args(b);
            /* K0(b) done, and K2(b-2), the last reader of w[p] / info_dup[p] */
            if (sK != sA && hipStreamWaitEvent(sK, c->k0done[p], 0) != hipSuccess) return ICW_EDEVICE;
            if (b >= n_sets && sK != sA && hipStreamWaitEvent(sK, c->k2done[p], 0) != hipSuccess) return ICW_EDEVICE;
            if (timing && hipEventRecord(c->ev[4 * b], sK) != hipSuccess) return ICW_EDEVICE;
            const hipError_t e1 = k1_mode == ICW_K1_FC ? icw_launch_iir_fc(&a1, N, cfg.iir_kahan, cfg.iir_subnorm_reject, sK)
                                : k1_mode == 3 ? icw_launch_iir_row(&a1, N, cfg.iir_kahan, cfg.iir_subnorm_reject, sK)
                                               : icw_launch_iir_state(&a1, N, cfg.iir_kahan, cfg.iir_subnorm_reject, sK);
            if (e1 != hipSuccess) return ICW_EDEVICE;
            if (timing && hipEventRecord(c->ev[4 * b + 1], sK) != hipSuccess) return ICW_EDEVICE;
            if (hipEventRecord(c->k1done[p], sK) != hipSuccess) return ICW_EDEVICE;
            if (sK != sA && hipStreamWaitEvent(sA, c->k1done[p], 0) != hipSuccess) return ICW_EDEVICE;
            /* real input: K0(b + n_sets) reuses xd[p], which K1(b) read; queued before K2(b) it
             * runs beside K1(b+1) instead of between two recurrences */
            if (b + n_sets < n_blocks && (rc0 = launch_k0(b + n_sets)) != ICW_OK) return rc0;
        } else if (timing && !fir) {
            if (hipEventRecord(c->ev[4 * b], sA) != hipSuccess || hipEventRecord(c->ev[4 * b + 1], sA) != hipSuccess)
                return ICW_EDEVICE;
        }

        /* the drain: K2 of the last block on the unmasked stream, after K1 of the block and K2 of
         * the one before it (the rotation table and the block order of the meters' owners) */
        const bool drain = sF && b == n_blocks - 1;
        hipStream_t s2 = drain ? sF : sA;
        if (drain && (hipStreamWaitEvent(sF, c->k1done[p], 0) != hipSuccess ||
                      (b >= 1 && hipStreamWaitEvent(sF, c->k2done[(b - 1) % n_sets], 0) != hipSuccess)))
            return ICW_EDEVICE;
        IcwK2Args a2 = k2_args(b);
        if (table) {
            IcwTrigArgs at;
            memset(&at, 0, sizeof(at));
            at.lds_guard = c->k1_lds ? 256u : 0u;
            at.prog = c->d_prog;
            at.n_frame = a2.n_frame;
            at.t0 = t0;
            at.T = T;
            at.scaled = cfg.frmod_scaled;
            at.trig_pitch = 2 * c->prog.n_trig;
            at.ssr = ssr;
            at.sample_rate = cfg.sample_rate;
            at.tab = c->trig;
            /* the fused FIR kernel's lanes hold 4 / 8 consecutive frames: rows 8 frames apart */
            at.perm_q = fir_fused ? (T + 7) / 8 : 0;
            /* same stream as K2: the previous block's K2 has read the table before it is rewritten */
            if (icw_launch_trig_table(&at, s2) != hipSuccess) return ICW_EDEVICE;
            a2.trig_tab = c->trig;
            a2.trig_pitch = at.trig_pitch;
            a2.trig_perm_q = at.perm_q;
        }
        /* rpre[p] / iq[p] were last read by the serial render of block b - n_sets (on sR) */
        if (c->serial_render && b >= n_sets && sR != s2 && hipStreamWaitEvent(s2, c->k3done[p], 0) != hipSuccess)
            return ICW_EDEVICE;
        if (dith_par) {
            /* K3a of this block on its own stream (it depends only on the generators' state, so it runs
             * ahead, beside the converter / output kernel of the block before); dith[p] was last read
             * by the output kernel of block b - n_sets */
            const IcwK3Args a3 = k3_args(b, a2);
            if (b >= n_sets && sD != s2 && hipStreamWaitEvent(sD, c->k2done[p], 0) != hipSuccess) return ICW_EDEVICE;
            const hipError_t ed = c->dither_lane ? icw_launch_dither_lane(&a3, sD) : icw_launch_dither(&a3, sD);
            if (ed != hipSuccess || hipEventRecord(c->ditdone[p], sD) != hipSuccess ||
                (sD != s2 && hipStreamWaitEvent(s2, c->ditdone[p], 0) != hipSuccess))
                return ICW_EDEVICE;
            a2.dith = a3.dith;
            a2.dith_pitch = a3.dith_pitch;
        }
        if (timing && hipEventRecord(c->ev[4 * b + 2], s2) != hipSuccess) return ICW_EDEVICE;
        if (fir_fused) {
            const IcwFirArgs af = fir_args(b);
            if (io_in(b, s2) != ICW_OK) return ICW_EDEVICE;
            if (timing && hipEventRecord(c->ev[4 * b], s2) != hipSuccess) return ICW_EDEVICE;
            if (icw_launch_fir_graph(&af, &a2, in_step, s2) != hipSuccess) return ICW_EDEVICE;
            if (timing && hipEventRecord(c->ev[4 * b + 1], s2) != hipSuccess) return ICW_EDEVICE;
        } else {
            if (fir_async && hipStreamWaitEvent(s2, c->k0done[p], 0) != hipSuccess) return ICW_EDEVICE;
            if (icw_launch_output(&a2, N, cfg.iir_kahan, s2) != hipSuccess) return ICW_EDEVICE;
        }
        if (hipEventRecord(c->k2done[p], s2) != hipSuccess) return ICW_EDEVICE;
        /* the serial part (K4, K3b) on sR after K2(b): it then overlaps K2(b+1) instead of
         * delaying it on sA */
        if (c->serial_render && sR != s2 && hipStreamWaitEvent(sR, c->k2done[p], 0) != hipSuccess) return ICW_EDEVICE;
        if (bus) {
            IcwK4Args a4;
            memset(&a4, 0, sizeof(a4));
            a4.lds_guard = c->k1_lds ? 256u : 0u;
            a4.iq = c->iq[p];
            a4.n_streams = count;
            a4.T = T;
            a4.t0 = t0;
            a4.n_frame = a2.n_frame;
            a4.ssr = a2.ssr;
            a4.scaled = a2.scaled;
            a4.sample_rate = a2.sample_rate;
            a4.prog = c->d_prog;
            a4.bus = a2.bus;
            a4.pre = a2.pre;
            a4.pre_stride = a2.pre_stride;
            if (icw_launch_graph_serial(&a4, sR) != hipSuccess) return ICW_EDEVICE;
        }
        if (c->serial_render) {
            IcwK3Args a3 = k3_args(b, a2);
            if (dither) {
                /* K3a for this block on its own stream: dith[p] was last read by K3b of block b-2 */
                if (b >= n_sets && sD != sR && hipStreamWaitEvent(sD, c->k3done[p], 0) != hipSuccess) return ICW_EDEVICE;
                const hipError_t ed = c->dither_lane ? icw_launch_dither_lane(&a3, sD) : icw_launch_dither(&a3, sD);
                if (ed != hipSuccess || hipEventRecord(c->ditdone[p], sD) != hipSuccess ||
                    (sD != sR && hipStreamWaitEvent(sR, c->ditdone[p], 0) != hipSuccess))
                    return ICW_EDEVICE;
            }
            if (icw_launch_render(&a3, sR) != hipSuccess) return ICW_EDEVICE;
            if (hipEventRecord(c->k3done[p], sR) != hipSuccess) return ICW_EDEVICE;
        }
        if (timing && hipEventRecord(c->ev[4 * b + 3], c->serial_render ? sR : s2) != hipSuccess) return ICW_EDEVICE;
        if (pipe_io) {
            /* this block's output slice, once its last writer (K2, or the serial render) is done */
            if (hipStreamWaitEvent(sC, c->serial_render ? c->k3done[p] : c->k2done[p], 0) != hipSuccess ||
                hipMemcpy2DAsync((unsigned char *)out + (size_t)t0 * osz, out_stride, d_out + (size_t)t0 * osz, dos,
                                 (size_t)T * osz, S, hipMemcpyDeviceToHost, sC) != hipSuccess)
                return ICW_EDEVICE;
        }
        /* complex input: K0(b + n_sets) reuses xd[p], which K2(b) read */
        if (cw && b + n_sets < n_blocks && (rc0 = launch_k0(b + n_sets)) != ICW_OK) return rc0;
    }
    if (!cw && nch > 1)
        for (int i = 0; i < count; ++i) c->lr_known[first + i] = 0;   /* stereo: the halves diverge */
    /* join: the caller's stream continues after every kernel of the call, then the call-start
     * position / phases / frame counters advance (icw_advance) */
    for (hipStream_t x : {sK, sA, sD, sR, sF, sC})
        if (x && x != st && (hipEventRecord(c->join, x) != hipSuccess || hipStreamWaitEvent(st, c->join, 0) != hipSuccess))
            return ICW_EDEVICE;
    /* FIR history: the current rows of every stream stay in fir_hist[fir_par] between calls (a call on
     * a subset of the streams must not move the others' rows); after an odd number of blocks this
     * call's rows are in the other buffer and come back */
    if (fir && (n_blocks & 1)) {
        const size_t hrow = 2 * (size_t)c->fir_M;
        if (hipMemcpyAsync(c->fir_hist[c->fir_par] + f0 * hrow, c->fir_hist[c->fir_par ^ 1] + f0 * hrow,
                           S * hrow * sizeof(double), hipMemcpyDeviceToDevice, st) != hipSuccess)
            return ICW_EDEVICE;
    }
        const IcwAdvArgs av = adv_args();
        if (icw_launch_advance(&av, st) != hipSuccess) return ICW_EDEVICE;
    }   /* !s1 */
    for (int i = 0; i < count; ++i) {   /* icw_advance's arithmetic */
        unsigned long long &v = c->nf_host[first + i];
        v = cfg.frmod_scaled ? (v + (unsigned long long)n_frames) % ssr : v + (unsigned long long)n_frames;
    }
    if (legacy && hipStreamSynchronize(st) != hipSuccess) return ICW_EDEVICE;
    if (!dev) {
        unsigned char *h_out = pinned ? c->h_stage + stage_in : nullptr;
        if (pinned ? (!zcopy && hipMemcpyAsync(h_out, d_out, dos * S + sizeof(int), hipMemcpyDeviceToHost, st) != hipSuccess)
                   : (!pipe_io && hipMemcpy2DAsync(out, out_stride, d_out, dos, dos, S, hipMemcpyDeviceToHost, st) != hipSuccess))
            return ICW_EDEVICE;
        if (d_pre && hipMemcpyAsync(dbg, d_pre, S * (size_t)n_frames * 2 * sizeof(double), hipMemcpyDeviceToHost, st) != hipSuccess)
            return ICW_EDEVICE;
        std::vector<double> rows;
        if (xin) {
            rows.resize(S * 2 * (size_t)n_frames);
            if (hipMemcpyAsync(rows.data(), c->d_xin, rows.size() * sizeof(double), hipMemcpyDeviceToHost, st) != hipSuccess)
                return ICW_EDEVICE;
        }
        int e = 0;
        if (pinned) {
            if (s1_poll ? !poll_done((const uint32_t *)(h_out + done_off), s1_seq, st)
                        : hipStreamSynchronize(st) != hipSuccess)
                return ICW_EDEVICE;
            memcpy(&e, h_out + dos * S, sizeof(int));     /* the flag icw_advance copied */
            for (size_t i = 0; i < S; ++i) memcpy((unsigned char *)out + i * out_stride, h_out + i * dos, dos);
        } else {
            if (hipStreamSynchronize(st) != hipSuccess) return ICW_EDEVICE;
            if (hipMemcpy(&e, ds.err, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return ICW_EDEVICE;
        }
        if (e) return ICW_EDEVICE;
        if (xin) {
            /* the rows hold the channel's signed sample {x, -x, -x, x}[k] at Hilbert phase k (icw_store_frame):
             * the sign undone is x exactly; a mono call (R = L, the dedup writes the left row only) repeats L */
            if (hipStreamSynchronize(st) != hipSuccess) return ICW_EDEVICE;
            double *o = (double *)dbg;
            for (size_t i = 0; i < S; ++i)
                for (int ch = 0; ch < 2; ++ch) {
                    const int rc = nch > 1 ? ch : 0;
                    const double *r = rows.data() + (i * 2 + rc) * (size_t)n_frames;
                    for (int t = 0; t < n_frames; ++t) {
                        const unsigned k = (xin_phase[i * 2 + rc] + (unsigned)t) & 3u;
                        o[(i * (size_t)n_frames + t) * 2 + ch] = (k == 0u || k == 3u) ? r[t] : -r[t];
                    }
                }
        }
    }
    if (s1 && c->s1_stamps) {
        unsigned long long sp[8];
        if (hipStreamSynchronize(st) == hipSuccess && hipMemcpy(sp, c->s1_stamps, sizeof(sp), hipMemcpyDeviceToHost) == hipSuccess)
            fprintf(stderr, "icw_s1 %d %llu %llu %llu %llu %llu %llu\n", n_frames, sp[2] - sp[0], sp[3] - sp[1],
                    sp[4] - sp[2], sp[5] - sp[3], sp[6] - sp[4], sp[7] - sp[5]);
    }
    if (timing) {
        if (hipStreamSynchronize(st) != hipSuccess) return ICW_EDEVICE;
        double m1 = 0, m2 = 0;
        for (int b = 0; b < n_blocks; ++b) {
            float x = 0, y = 0;
            if (hipEventElapsedTime(&x, c->ev[4 * b], c->ev[4 * b + 1]) != hipSuccess ||
                hipEventElapsedTime(&y, c->ev[4 * b + 2], c->ev[4 * b + 3]) != hipSuccess)
                return ICW_EDEVICE;
            m1 += x;
            m2 += y;
        }
        c->last_ms[0] = m1;
        c->last_ms[1] = m2;
        c->last_launches[0] = c->last_launches[1] = n_blocks;
    }
    return hipGetLastError() == hipSuccess ? ICW_OK : ICW_EDEVICE;
}

/* Warm-up of a fresh context (include/icw.h): one call of n_frames frames of digital silence through
 * the path the context's configuration takes, then the fresh state back (icw_stream_init is exactly
 * the state icw_create leaves).  What the first call would otherwise pay happens here: the pinned
 * staging buffer, the device buffers (sized for the widest frame, so a later track's format does
 * not grow them) and the lazy load of the kernels' code objects on the first launch.  The drop-in
 * measured 7 ms for its first 576-frame block (BENCH_r03 C1 block_latency_us.first), against
 * ~113 us for the others. */
int icw_prepare(icw_ctx *c, int n_frames)
{
    if (!c || n_frames < 0) return ICW_EINVAL;
    if (n_frames == 0) n_frames = ICW_S1_MAX;
    const size_t S = (size_t)c->n_streams;
    {
        std::lock_guard<std::mutex> lk(c->mu);
        if (c->calls || c->touched) return ICW_EINVAL;   /* would have to restore state it cannot know */
        if (set_dev(c)) return ICW_EDEVICE;
        const size_t widest = 2 * fmt_size(ICW_FMT_CW_F64), osz = 2 * 3;
        if (grow((void **)&c->d_in, &c->d_in_bytes, (size_t)n_frames * widest * S) ||
            grow((void **)&c->d_out, &c->d_out_bytes, (size_t)n_frames * osz * S + 16))
            return ICW_ENOMEM;
    }
    const unsigned fsz = fmt_size(c->cfg.in_format) * c->cfg.in_channels;
    const size_t osz = 2 * (size_t)(c->cfg.need24bits ? 3 : 2);
    std::vector<unsigned char> in((size_t)n_frames * fsz * S, 0), out((size_t)n_frames * osz * S);
    if (c->cfg.in_format == ICW_FMT_U8) std::fill(in.begin(), in.end(), (unsigned char)0x80);   /* u8 silence */
    int rc = icw_process_streams(c, 0, (int)S, in.data(), (size_t)n_frames * fsz, out.data(), (size_t)n_frames * osz,
                                 n_frames, 0u, nullptr, nullptr);
    if (rc == ICW_OK) rc = icw_stream_init(c, 0, (int)S);
    std::lock_guard<std::mutex> lk(c->mu);
    c->calls = 0;
    return rc;
}

int icw_process_batch(icw_ctx *c, const void *in, size_t in_stride, void *out, size_t out_stride, int n_frames,
                      unsigned flags, void *dbg, void *hip_stream)
{
    if (!c) return ICW_EINVAL;
    return icw_process_streams(c, 0, c->n_streams, in, in_stride, out, out_stride, n_frames, flags, dbg, hip_stream);
}

int icw_host_alloc(size_t bytes, void **p)
{
    if (!p || !bytes) return ICW_EINVAL;
    *p = nullptr;
    /* portable: pinned for every device, so an icw_group's shards on other devices pipeline their
     * slices of the same buffer too (host_pinned) */
    return hipHostMalloc(p, bytes, hipHostMallocPortable) == hipSuccess ? ICW_OK : ICW_ENOMEM;
}

int icw_host_free(void *p)
{
    return (!p || hipHostFree(p) == hipSuccess) ? ICW_OK : ICW_EINVAL;
}

int icw_host_pinned(const void *p, int device)
{
    return p && host_pinned(p, device) ? 1 : 0;
}

int icw_synchronize(icw_ctx *c)
{
    if (!c) return ICW_EINVAL;
    if (set_dev(c)) return ICW_EDEVICE;
    if (quiesce(c) != hipSuccess) return ICW_EDEVICE;
    int e = 0;
    if (hipMemcpy(&e, c->st.err, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess || e) return ICW_EDEVICE;
    return ICW_OK;
}

/* amod_get_clips_peaks (adv_modulator.c:445-465): with isReset the clip counters and peaks are
 * cleared FIRST and the cleared values (0, SR_ZERO_SIGNAL_DB) are returned; the de-subnorm count
 * (mod_context_get_desubnorm_counter, in_cwave.c:300-310) is not reset by it.  The meters are
 * written by kernels that may still run (ICW_F_DEVICE_PTRS calls return early, on several
 * streams), so the read waits for the context's work first, as get_state does. */
int icw_get_meters(icw_ctx *c, int s, int reset, icw_meters *m)
{
    if (!c || !m || s < 0 || s >= c->n_streams) return ICW_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    if (set_dev(c) || quiesce(c) != hipSuccess) return ICW_EDEVICE;
    uint32_t cl[2];
    unsigned long long pb[2], sn[4];
    bool ok = true;
    if (reset) {
        ok &= hipMemset(c->st.clips + (size_t)s * 2, 0, sizeof(cl)) == hipSuccess;
        ok &= hipMemset(c->st.peak_bits + (size_t)s * 2, 0, sizeof(pb)) == hipSuccess;
        c->peak_db[(size_t)s * 2] = c->peak_db[(size_t)s * 2 + 1] = ICW_SR_ZERO_SIGNAL_DB;
    }
    ok &= hipMemcpy(cl, c->st.clips + (size_t)s * 2, sizeof(cl), hipMemcpyDeviceToHost) == hipSuccess;
    ok &= hipMemcpy(pb, c->st.peak_bits + (size_t)s * 2, sizeof(pb), hipMemcpyDeviceToHost) == hipSuccess;
    ok &= hipMemcpy(sn, c->st.sncnt + (size_t)s * 4, sizeof(sn), hipMemcpyDeviceToHost) == hipSuccess;
    if (!ok) return ICW_EDEVICE;
    for (int ch = 0; ch < 2; ++ch) {
        /* peak meter (sound_render.c:769-780): max over samples of 20*log10(|q|/hi) equals
         * 20*log10(max|q| / hi) because the map is monotone; 0 -> SR_ZERO_SIGNAL_DB */
        double mx;
        memcpy(&mx, &pb[ch], 8);
        double cv = mx / c->rk.hi;
        cv = cv ? 20.0 * log10(cv) : ICW_SR_ZERO_SIGNAL_DB;
        double &pv = c->peak_db[(size_t)s * 2 + ch];
        if (cv > pv) pv = cv;
        m->clips[ch] = cl[ch];
        m->peak_db[ch] = pv;
    }
    m->desubnorm = sn[0] + sn[1] + sn[2] + sn[3];
    return ICW_OK;
}

int icw_n_frame(icw_ctx *c, int s, uint64_t *nf)
{
    if (!c || !nf || s < 0 || s >= c->n_streams) return ICW_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    if (set_dev(c) || quiesce(c) != hipSuccess) return ICW_EDEVICE;
    unsigned long long v = 0;
    if (hipMemcpy(&v, c->st.n_frame + s, sizeof(v), hipMemcpyDeviceToHost) != hipSuccess) return ICW_EDEVICE;
    *nf = v;
    /* the host mirror decides whether the fused FIR kernel may take every Shift / PM factor from the
     * shared table (in_step): a device-side write it did not follow would give the stream another
     * stream's rotation, so a divergence fails this read loudly */
    if (c->nf_host[s] != v) {
        fprintf(stderr, "icw_n_frame: stream %d frame counter %llu, host mirror %llu\n", s, v, c->nf_host[s]);
        return ICW_EDEVICE;
    }
    return ICW_OK;
}

/* canonical state blob: see DESIGN.md "Per-stream state" */
struct IcwBlob {
    uint64_t magic, n_frame;
    int64_t pos, n_samples, n_fade_in, n_fade_out;
    uint32_t hq_phase[2], nord, has_render;
    uint32_t fir_M, reserved;         /* FIR converter order in force (0: the quadrature IIR) */
    double hist[4][ICW_HIST_PITCH];
    uint64_t sncnt[4];
    double bus[ICW_N_INPUTS][4];
    /* serial render state per channel (dithered / noise-shaped renders only, else zero):
     * MT19937 words and next index (624: twist due), prev_rnd, prev_ns_err, shaper history by age */
    uint32_t mt[2][624];
    int32_t mt_idx[2];
    double rs[2][ICW_RSTATE];
};
constexpr uint64_t kBlobMagic = 0x33574349ull;   /* "ICW3" */

/* with the FIR Hilbert converter on, its history (2 x k_M doubles, oldest first) follows the blob */
size_t icw_state_size(const icw_ctx *c) { return c ? sizeof(IcwBlob) + 2 * (size_t)c->fir_M * sizeof(double) : 0; }

int icw_get_state(icw_ctx *c, int s, void *blob, size_t size)
{
    if (!c || !blob || size < icw_state_size(c) || s < 0 || s >= c->n_streams) return ICW_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    if (set_dev(c)) return ICW_EDEVICE;
    IcwBlob b;
    memset(&b, 0, sizeof(b));
    b.magic = kBlobMagic;
    b.nord = (uint32_t)c->nord;
    b.has_render = c->render_state ? 1u : 0u;
    b.fir_M = (uint32_t)c->fir_M;
    long long fd[3];
    bool ok = quiesce(c) == hipSuccess;
    ok &= hipMemcpy(&b.n_frame, c->st.n_frame + s, 8, hipMemcpyDeviceToHost) == hipSuccess;
    ok &= hipMemcpy(&b.pos, c->st.pos + s, 8, hipMemcpyDeviceToHost) == hipSuccess;
    ok &= hipMemcpy(fd, c->st.fade + (size_t)s * 3, sizeof(fd), hipMemcpyDeviceToHost) == hipSuccess;
    ok &= hipMemcpy(b.hq_phase, c->st.hq_phase + (size_t)s * 2, 8, hipMemcpyDeviceToHost) == hipSuccess;
    ok &= hipMemcpy(b.hist, c->st.hist + (size_t)s * 4 * ICW_HIST_PITCH, sizeof(b.hist), hipMemcpyDeviceToHost) == hipSuccess;
    ok &= hipMemcpy(b.sncnt, c->st.sncnt + (size_t)s * 4, sizeof(b.sncnt), hipMemcpyDeviceToHost) == hipSuccess;
    ok &= hipMemcpy(b.bus, c->st.bus + (size_t)s * ICW_N_INPUTS * 4, sizeof(b.bus), hipMemcpyDeviceToHost) == hipSuccess;
    if (c->render_state) {
        const size_t G = (size_t)c->n_streams * 2;
        for (int ch = 0; ch < 2; ++ch)
            ok &= hipMemcpy2D(b.mt[ch], 4, c->st.mt + (size_t)s * 2 + ch, G * 4, 4, 624, hipMemcpyDeviceToHost) == hipSuccess;
        ok &= hipMemcpy(b.mt_idx, c->st.mt_idx + (size_t)s * 2, sizeof(b.mt_idx), hipMemcpyDeviceToHost) == hipSuccess;
        ok &= hipMemcpy(b.rs, c->st.rs + (size_t)s * 2 * ICW_RSTATE, sizeof(b.rs), hipMemcpyDeviceToHost) == hipSuccess;
    }
    b.n_samples = fd[0]; b.n_fade_in = fd[1]; b.n_fade_out = fd[2];
    if (c->fir_M) {
        const size_t hrow = 2 * (size_t)c->fir_M;
        ok &= hipMemcpy((unsigned char *)blob + sizeof(b), c->fir_hist[c->fir_par] + (size_t)s * hrow,
                        hrow * sizeof(double), hipMemcpyDeviceToHost) == hipSuccess;
    }
    if (!ok) return ICW_EDEVICE;
    memcpy(blob, &b, sizeof(b));
    return ICW_OK;
}

int icw_set_state(icw_ctx *c, int s, const void *blob, size_t size)
{
    if (!c || !blob || size < icw_state_size(c) || s < 0 || s >= c->n_streams) return ICW_EINVAL;
    IcwBlob b;
    memcpy(&b, blob, sizeof(b));
    /* a blob holds the state of the render and converter forms in force when it was saved: the
     * serial-render words exist only with a dithered / shaped render, the FIR history only at its order */
    if (b.magic != kBlobMagic || b.nord != (uint32_t)c->nord || b.has_render != (c->render_state ? 1u : 0u) ||
        b.fir_M != (uint32_t)c->fir_M)
        return ICW_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    if (set_dev(c)) return ICW_EDEVICE;
    long long fd[3] = {b.n_samples, b.n_fade_in, b.n_fade_out};
    c->touched = true;
    bool ok = quiesce(c) == hipSuccess;
    ok &= hipMemcpy(c->st.n_frame + s, &b.n_frame, 8, hipMemcpyHostToDevice) == hipSuccess;
    c->nf_host[s] = b.n_frame;
    ok &= hipMemcpy(c->st.pos + s, &b.pos, 8, hipMemcpyHostToDevice) == hipSuccess;
    ok &= hipMemcpy(c->st.fade + (size_t)s * 3, fd, sizeof(fd), hipMemcpyHostToDevice) == hipSuccess;
    ok &= hipMemcpy(c->st.hq_phase + (size_t)s * 2, b.hq_phase, 8, hipMemcpyHostToDevice) == hipSuccess;
    ok &= hipMemcpy(c->st.hist + (size_t)s * 4 * ICW_HIST_PITCH, b.hist, sizeof(b.hist), hipMemcpyHostToDevice) == hipSuccess;
    ok &= hipMemcpy(c->st.sncnt + (size_t)s * 4, b.sncnt, sizeof(b.sncnt), hipMemcpyHostToDevice) == hipSuccess;
    ok &= hipMemcpy(c->st.bus + (size_t)s * ICW_N_INPUTS * 4, b.bus, sizeof(b.bus), hipMemcpyHostToDevice) == hipSuccess;
    const uint32_t eq = (b.hq_phase[0] == b.hq_phase[1] && !memcmp(b.hist[0], b.hist[2], sizeof(b.hist[0]) * 2)) ? 1u : 0u;
    const uint32_t eq2[2] = {eq, eq};
    ok &= hipMemcpy(c->st.lr_equal + (size_t)s * 2, eq2, sizeof(eq2), hipMemcpyHostToDevice) == hipSuccess;
    c->lr_known[s] = eq ? 1 : 0;
    if (c->render_state) {
        const size_t G = (size_t)c->n_streams * 2;
        for (int ch = 0; ch < 2; ++ch)
            ok &= hipMemcpy2D(c->st.mt + (size_t)s * 2 + ch, G * 4, b.mt[ch], 4, 4, 624, hipMemcpyHostToDevice) == hipSuccess;
        ok &= hipMemcpy(c->st.mt_idx + (size_t)s * 2, b.mt_idx, sizeof(b.mt_idx), hipMemcpyHostToDevice) == hipSuccess;
        ok &= hipMemcpy(c->st.rs + (size_t)s * 2 * ICW_RSTATE, b.rs, sizeof(b.rs), hipMemcpyHostToDevice) == hipSuccess;
    }
    if (c->fir_M) {
        const size_t hrow = 2 * (size_t)c->fir_M;
        ok &= hipMemcpy(c->fir_hist[c->fir_par] + (size_t)s * hrow, (const unsigned char *)blob + sizeof(b),
                        hrow * sizeof(double), hipMemcpyHostToDevice) == hipSuccess;
    }
    return ok ? ICW_OK : ICW_EDEVICE;
}

int icw_get_fp_census(icw_ctx *c, int s, int reset, uint32_t counts[4][ICW_FES_N])
{
    if (!c || !counts || s < 0 || s >= c->n_streams) return ICW_EINVAL;
    if (!c->st.fes) {
        memset(counts, 0, sizeof(uint32_t) * 4 * ICW_FES_N);
        return ICW_OK;
    }
    std::lock_guard<std::mutex> lk(c->mu);
    if (set_dev(c) || quiesce(c) != hipSuccess) return ICW_EDEVICE;
    uint32_t buf[4 * ICW_FES_PITCH];
    uint32_t *src = c->st.fes + (size_t)s * 4 * ICW_FES_PITCH;
    if (hipMemcpy(buf, src, sizeof(buf), hipMemcpyDeviceToHost) != hipSuccess) return ICW_EDEVICE;
    for (int i = 0; i < 4; ++i)
        for (int k = 0; k < ICW_FES_N; ++k) counts[i][k] = buf[i * ICW_FES_PITCH + k];
    if (reset && hipMemset(src, 0, sizeof(buf)) != hipSuccess) return ICW_EDEVICE;
    return ICW_OK;
}

int icw_last_k1_kernel(const icw_ctx *c)
{
    if (!c) return ICW_EINVAL;
    return c->last_k1;
}

int icw_last_timing(icw_ctx *c, double ms[2], int launches[2])
{
    if (!c || !ms || !launches) return ICW_EINVAL;
    ms[0] = c->last_ms[0];
    ms[1] = c->last_ms[1];
    launches[0] = c->last_launches[0];
    launches[1] = c->last_launches[1];
    return ICW_OK;
}

}  /* extern "C" */
