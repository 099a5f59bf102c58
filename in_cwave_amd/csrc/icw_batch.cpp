/*
 * icw_batch.cpp -- WAV / CWAVE file headers and the batched many-file transcoder
 * (include/icw_reader.h).  Host C++ over the C ABI of icw.h; the samples are processed only by the
 * gfx950 kernels (icw_process_streams with device pointers).
 *
 * Mirrors: check_file_ext (xwave_reader.c:123-131), rwave_reader_create (xwave_reader.c:362-585),
 * cwave_reader_create (via icw_cwave_parse), xwave_reader_create's MAX_FS_SRC check and virtual
 * zero tail (xwave_reader.c:672-697), xwave_read_samples (xwave_reader.c:838-904: data, then the
 * format's zero sample for the tail), transcode.c:39-120 (2-channel output of out_size bytes).
 */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <string.h>
#include <strings.h>

#include <algorithm>
#include <chrono>
#include <map>
#include <memory>
#include <tuple>
#include <vector>

#include "../../include/icw_cwave.h"
#include "../../include/icw_reader.h"

namespace {

uint32_t le16(const unsigned char *p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }
uint32_t le32(const unsigned char *p)
{
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

struct File {
    FILE *f = nullptr;
    ~File() { if (f) fclose(f); }
};

int64_t file_size(FILE *f)
{
    if (fseeko(f, 0, SEEK_END)) return -1;
    const int64_t n = ftello(f);
    if (fseeko(f, 0, SEEK_SET)) return -1;
    return n;
}

bool rd(FILE *f, void *b, size_t n) { return fread(b, 1, n, f) == n; }

/* pcmBpsToFormat (xwave_reader.c:342-358) */
int bps_format(unsigned bps)
{
    switch (bps) {
    case 8: return ICW_FMT_U8;
    case 16: return ICW_FMT_I16;
    case 24: return ICW_FMT_I24;
    case 32: return ICW_FMT_I32;
    }
    return -1;
}

/* rwave_reader_create (xwave_reader.c:362-585) */
int parse_rwave(FILE *f, int64_t fsize, icw_wav_info *w)
{
    static const unsigned char guid_tail[14] = {0x00, 0x00, 0x00, 0x00, 0x10, 0x00, 0x80, 0x00,
                                                0x00, 0xaa, 0x00, 0x38, 0x9b, 0x71};
    const size_t sz_wf = 14, sz_pcmwf = 16, sz_ext = 40;   /* WAVEFORMAT, PCMWAVEFORMAT, ..EXTENSIBLE */
    unsigned char h[12], ch[8], fmt[40];
    int64_t fpos = 0;
    uint32_t fmt_len = 0, data_len = 0;
    if (!rd(f, h, 12) || memcmp(h, "RIFF", 4) || memcmp(h + 8, "WAVE", 4)) return ICW_EINVAL;
    fpos = 12;
    for (;;) {                                             /* "fmt " before any "data" */
        if (!rd(f, ch, 8)) return ICW_EINVAL;
        fmt_len = le32(ch + 4);
        fpos += 8;
        if (fpos + fmt_len > fsize) return ICW_EINVAL;
        if (!memcmp(ch, "fmt ", 4)) break;
        if (!memcmp(ch, "data", 4)) return ICW_EINVAL;
        if (fseeko(f, fmt_len, SEEK_CUR)) return ICW_EINVAL;
        fpos += fmt_len;
    }
    if (fmt_len < sz_wf) return ICW_EINVAL;
    const size_t toread = fmt_len < sz_ext ? fmt_len : sz_ext;
    memset(fmt, 0, sizeof(fmt));
    if (!rd(f, fmt, toread)) return ICW_EINVAL;
    if (toread < fmt_len && fseeko(f, (off_t)(fmt_len - toread), SEEK_CUR)) return ICW_EINVAL;
    fpos += fmt_len;
    const uint32_t tag = le16(fmt), nch = le16(fmt + 2), rate = le32(fmt + 4), align = le16(fmt + 12);
    uint32_t bps = (le16(fmt + 14) + 7) & ~7u;            /* rounded up to whole bytes */
    if (!nch || nch > 2 || !rate) return ICW_EINVAL;
    int format = -1;
    switch (tag) {
    case 1:                                                /* WAVE_FORMAT_PCM */
        if (fmt_len < sz_pcmwf) {
            if (align % nch) return ICW_EINVAL;
            bps = (align / nch) << 3;
            w->htype = ICW_HTYPE_WFONLY;
        } else {
            w->htype = ICW_HTYPE_PCMW;
        }
        format = bps_format(bps);
        break;
    case 3:                                                /* WAVE_FORMAT_IEEE_FLOAT */
        if (fmt_len < sz_pcmwf || bps != 32) return ICW_EINVAL;
        w->htype = ICW_HTYPE_PCMW;
        format = ICW_FMT_F32;
        break;
    case 0xFFFE:                                           /* WAVE_FORMAT_EXTENSIBLE */
        if (fmt_len < sz_ext || le16(fmt + 16) < 2 + 4 + 16) return ICW_EINVAL;
        w->htype = ICW_HTYPE_EXT;
        if (!memcmp(fmt + 26, guid_tail, 14) && (le16(fmt + 24) == 1 || le16(fmt + 24) == 3)) {
            if (le16(fmt + 24) == 1) format = bps_format(bps);
            else format = bps == 32 ? ICW_FMT_F32 : -1;
        }
        break;
    default:
        return ICW_EINVAL;
    }
    if (format < 0) return ICW_EINVAL;
    for (;;) {                                             /* then the "data" chunk */
        if (!rd(f, ch, 8)) return ICW_EINVAL;
        fpos += 8;
        data_len = le32(ch + 4);
        if (fpos + data_len > fsize) return ICW_EINVAL;
        if (!memcmp(ch, "data", 4)) break;
        if (fseeko(f, data_len, SEEK_CUR)) return ICW_EINVAL;
        fpos += data_len;
    }
    const uint32_t csz = bps >> 3, frame = csz * nch;
    w->n_samples = data_len / frame;
    if (w->n_samples < 2 || align != frame) return ICW_EINVAL;   /* MIN_FILE_SAMPLES, nBlockAlign */
    w->fmt = (uint32_t)format;
    w->channels = nch;
    w->sample_rate = rate;
    w->frame_bytes = frame;
    w->data_offset = fpos;
    return ICW_OK;
}

/* the format's zero sample (zero_u8 = 0x80 for unsigned 8 bit, zero bytes otherwise) */
unsigned char zero_byte(uint32_t fmt) { return fmt == ICW_FMT_U8 ? 0x80 : 0x00; }

struct Job {
    int idx;
    icw_wav_info info;
    FILE *in = nullptr, *out = nullptr;
    int64_t total = 0;        /* n_samples + tail */
    int64_t read = 0;         /* data frames read so far */
    int64_t written = 0;      /* output frames written so far */
};

void wav_header(unsigned char *h, uint32_t rate, int bytes_per_sample, uint64_t frames)
{
    const uint32_t block = 2u * (uint32_t)bytes_per_sample;
    const uint64_t data = frames * block;
    const uint32_t d32 = data > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)data;
    auto p32 = [](unsigned char *q, uint32_t v) { q[0] = v; q[1] = v >> 8; q[2] = v >> 16; q[3] = v >> 24; };
    auto p16 = [](unsigned char *q, uint32_t v) { q[0] = v; q[1] = v >> 8; };
    memcpy(h, "RIFF", 4); p32(h + 4, 36 + d32); memcpy(h + 8, "WAVE", 4);
    memcpy(h + 12, "fmt ", 4); p32(h + 16, 16); p16(h + 20, 1); p16(h + 22, 2); p32(h + 24, rate);
    p32(h + 28, rate * block); p16(h + 32, block); p16(h + 34, 8 * bytes_per_sample);
    memcpy(h + 36, "data", 4); p32(h + 40, d32);
}

double now_s()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

/* One group of files sharing (rate, format, channels): one context, one stream per file. */
int run_group(const icw_config &cfg0, const icw_node *nodes, int n_nodes, std::vector<Job *> &jobs,
              const icw_batch_opts &o, icw_batch_stats &st, int *status)
{
    const int S = (int)jobs.size();
    const icw_wav_info &wi = jobs[0]->info;
    icw_config cfg = cfg0;
    cfg.sample_rate = wi.sample_rate;
    cfg.in_format = wi.fmt;
    cfg.in_channels = wi.channels;
    icw_ctx *ctx = nullptr;
    int accepted = 0;
    int rc = icw_create(&cfg, nodes, n_nodes, S, o.device, &ctx, &accepted);
    if (rc != ICW_OK) return rc;
    std::unique_ptr<icw_ctx, int (*)(icw_ctx *)> guard(ctx, icw_destroy);
    const int rs = icw_render_size(ctx), osz = 2 * rs;
    const size_t fsz = wi.frame_bytes;
    const int B = o.block_frames > 0 ? o.block_frames : 65536;
    int64_t T = 0;
    for (int s = 0; s < S; ++s) {
        Job &j = *jobs[s];
        /* xwave_reader_create's virtual zero tail (xwave_reader.c:688-697) */
        int64_t tail = 0;
        if (o.sec_align) {
            const int64_t mt = (int64_t)wi.sample_rate * (int64_t)o.sec_align, fr = j.info.n_samples % mt;
            tail = fr ? mt - fr : 0;
        }
        j.total = j.info.n_samples + tail;
        T = std::max(T, j.total);
        if ((rc = icw_stream_open(ctx, s, j.info.n_samples, o.fade_in_ms, o.fade_out_ms, o.sec_align, 0, 0)) != ICW_OK)
            return rc;
        unsigned char hdr[44];
        wav_header(hdr, wi.sample_rate, rs, (uint64_t)j.total);
        if (fwrite(hdr, 1, 44, j.out) != 44) status[j.idx] = ICW_EINVAL;
        if (fseeko(j.in, j.info.data_offset, SEEK_SET)) status[j.idx] = ICW_EINVAL;
    }
    /* pinned double buffers, device double buffers, a copy stream */
    const size_t in_b = (size_t)S * B * fsz, out_b = (size_t)S * B * osz;
    unsigned char *hin[2] = {nullptr, nullptr}, *hout[2] = {nullptr, nullptr}, *din[2] = {nullptr, nullptr},
                  *dout[2] = {nullptr, nullptr};
    hipStream_t cs = nullptr, ks = nullptr;
    hipEvent_t h2d[2] = {nullptr, nullptr}, comp[2] = {nullptr, nullptr}, d2h[2] = {nullptr, nullptr};
    auto cleanup = [&]() {
        if (cs) (void)hipStreamSynchronize(cs);
        if (ks) (void)hipStreamSynchronize(ks);
        for (int p = 0; p < 2; ++p) {
            if (hin[p]) (void)hipHostFree(hin[p]);
            if (hout[p]) (void)hipHostFree(hout[p]);
            if (din[p]) (void)hipFree(din[p]);
            if (dout[p]) (void)hipFree(dout[p]);
            for (hipEvent_t e : {h2d[p], comp[p], d2h[p]}) if (e) (void)hipEventDestroy(e);
        }
        if (cs) (void)hipStreamDestroy(cs);
        if (ks) (void)hipStreamDestroy(ks);
    };
    bool ok = true;
    for (int p = 0; p < 2 && ok; ++p) {
        ok = hipHostMalloc((void **)&hin[p], in_b, hipHostMallocDefault) == hipSuccess &&
             hipHostMalloc((void **)&hout[p], out_b, hipHostMallocDefault) == hipSuccess &&
             hipMalloc((void **)&din[p], in_b) == hipSuccess && hipMalloc((void **)&dout[p], out_b) == hipSuccess &&
             hipEventCreateWithFlags(&h2d[p], hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&comp[p], hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&d2h[p], hipEventDisableTiming) == hipSuccess;
    }
    ok = ok && hipStreamCreateWithFlags(&cs, hipStreamNonBlocking) == hipSuccess &&
         hipStreamCreateWithFlags(&ks, hipStreamNonBlocking) == hipSuccess;
    if (!ok) { cleanup(); return ICW_ENOMEM; }

    const int nb = (int)((T + B - 1) / B);
    /* xwave_read_samples for block k into hin[k&1]: data frames, then zero samples */
    auto read_block = [&](int k) {
        const double t0 = now_s();
        unsigned char *buf = hin[k & 1];
        for (int s = 0; s < S; ++s) {
            Job &j = *jobs[s];
            unsigned char *row = buf + (size_t)s * B * fsz;
            const int64_t want = std::min<int64_t>(B, std::max<int64_t>(0, j.info.n_samples - j.read));
            size_t got = 0;
            if (want > 0 && status[j.idx] == ICW_OK) {
                got = fread(row, fsz, (size_t)want, j.in);
                if ((int64_t)got != want) status[j.idx] = ICW_EINVAL;      /* short read: broken file */
                j.read += (int64_t)got;
                st.frames_in += got;
            }
            memset(row + got * fsz, zero_byte(j.info.fmt), (size_t)(B - (int64_t)got) * fsz);
        }
        st.io_s += now_s() - t0;
    };
    auto write_block = [&](int k) {
        const double t0 = now_s();
        const unsigned char *buf = hout[k & 1];
        for (int s = 0; s < S; ++s) {
            Job &j = *jobs[s];
            const int64_t n = std::min<int64_t>(B, j.total - j.written);
            if (n <= 0 || status[j.idx] != ICW_OK) continue;
            if (fwrite(buf + (size_t)s * B * osz, osz, (size_t)n, j.out) != (size_t)n) status[j.idx] = ICW_EINVAL;
            j.written += n;
            st.frames_out += (uint64_t)n;
        }
        st.io_s += now_s() - t0;
    };

    read_block(0);
    for (int k = 0; k < nb && rc == ICW_OK; ++k) {
        const int p = k & 1;
        /* H2D(k): d_in[p] was last read by compute(k-2) */
        if (k >= 2 && hipStreamWaitEvent(cs, comp[p], 0) != hipSuccess) rc = ICW_EDEVICE;
        if (rc == ICW_OK && (hipMemcpyAsync(din[p], hin[p], in_b, hipMemcpyHostToDevice, cs) != hipSuccess ||
                             hipEventRecord(h2d[p], cs) != hipSuccess || hipStreamWaitEvent(ks, h2d[p], 0) != hipSuccess))
            rc = ICW_EDEVICE;
        if (rc == ICW_OK)
            rc = icw_process_streams(ctx, 0, S, din[p], (size_t)B * fsz, dout[p], (size_t)B * osz, B,
                                     ICW_F_DEVICE_PTRS, nullptr, ks);
        if (rc == ICW_OK && (hipEventRecord(comp[p], ks) != hipSuccess || hipStreamWaitEvent(cs, comp[p], 0) != hipSuccess ||
                             hipMemcpyAsync(hout[p], dout[p], out_b, hipMemcpyDeviceToHost, cs) != hipSuccess ||
                             hipEventRecord(d2h[p], cs) != hipSuccess))
            rc = ICW_EDEVICE;
        if (rc != ICW_OK) break;
        /* host work overlapping the GPU: read block k+1 (after H2D(k-1) released its buffer),
         * write block k-1 (after its D2H) */
        if (k + 1 < nb) {
            if (k >= 1 && hipEventSynchronize(h2d[(k + 1) & 1]) != hipSuccess) { rc = ICW_EDEVICE; break; }
            read_block(k + 1);
        }
        if (k >= 1) {
            if (hipEventSynchronize(d2h[(k - 1) & 1]) != hipSuccess) { rc = ICW_EDEVICE; break; }
            write_block(k - 1);
        }
    }
    if (rc == ICW_OK && nb >= 1) {
        if (hipEventSynchronize(d2h[(nb - 1) & 1]) != hipSuccess) rc = ICW_EDEVICE;
        else write_block(nb - 1);
    }
    if (rc == ICW_OK) rc = icw_synchronize(ctx);
    cleanup();
    return rc;
}

}  // namespace

extern "C" {

int icw_wav_parse_file(const char *path, icw_wav_info *info)
{
    if (!path || !info) return ICW_EINVAL;
    memset(info, 0, sizeof(*info));
    const char *dot = strrchr(path, '.');
    if (!dot) return ICW_EINVAL;
    const bool cw = !strcasecmp(dot + 1, "CWAVE");
    if (!cw && strcasecmp(dot + 1, "WAV") && strcasecmp(dot + 1, "RWAVE")) return ICW_EINVAL;
    File fh;
    if (!(fh.f = fopen(path, "rb"))) return ICW_EINVAL;
    const int64_t fsize = file_size(fh.f);
    if (fsize < 0) return ICW_EINVAL;
    int rc;
    if (cw) {
        unsigned char hdr[ICW_CWAVE_HEADER_BYTES];
        if (!rd(fh.f, hdr, sizeof(hdr))) return ICW_EINVAL;
        icw_cwave_header h;
        uint32_t fmt = 0, fb = 0;
        if ((rc = icw_cwave_parse(hdr, sizeof(hdr), fsize, &h, &fmt, &fb)) != ICW_OK) return rc;
        info->fmt = fmt;
        info->channels = h.n_channels;
        info->sample_rate = h.sample_rate;
        info->frame_bytes = fb;
        info->n_samples = h.n_samples;
        info->data_offset = h.hsize;
        info->htype = ICW_HTYPE_CWAVE;
    } else if ((rc = parse_rwave(fh.f, fsize, info)) != ICW_OK) {
        return rc;
    }
    if (info->sample_rate > ICW_MAX_FS_SRC) return ICW_EINVAL;         /* xwave_reader.c:672-674 */
    return ICW_OK;
}

int icw_transcode_files(const icw_config *cfg, const icw_node *nodes, int n_nodes, const char *const *in_paths,
                        const char *const *out_paths, int n, const icw_batch_opts *opts, icw_batch_stats *stats,
                        int *status)
{
    if (!cfg || n < 0 || (n > 0 && (!in_paths || !out_paths))) return ICW_EINVAL;
    const double t0 = now_s();
    icw_batch_opts o;
    memset(&o, 0, sizeof(o));
    o.device = -1;
    if (opts) o = *opts;
    icw_batch_stats st;
    memset(&st, 0, sizeof(st));
    std::vector<int> stat_local(n > 0 ? n : 1, ICW_OK);
    int *sts = status ? status : stat_local.data();
    std::vector<Job> jobs(n);
    std::map<std::tuple<uint32_t, uint32_t, uint32_t>, std::vector<Job *>> groups;
    for (int i = 0; i < n; ++i) {
        sts[i] = ICW_OK;
        Job &j = jobs[i];
        j.idx = i;
        if (!in_paths[i] || !out_paths[i] || (sts[i] = icw_wav_parse_file(in_paths[i], &j.info)) != ICW_OK) {
            if (sts[i] == ICW_OK) sts[i] = ICW_EINVAL;
            continue;
        }
        if (!(j.in = fopen(in_paths[i], "rb")) || !(j.out = fopen(out_paths[i], "wb"))) {
            sts[i] = ICW_EINVAL;
            continue;
        }
        setvbuf(j.in, nullptr, _IOFBF, 1 << 20);
        setvbuf(j.out, nullptr, _IOFBF, 1 << 20);
        groups[std::make_tuple(j.info.sample_rate, j.info.fmt, j.info.channels)].push_back(&j);
    }
    int rc = ICW_OK;
    for (auto &g : groups) {
        const int r = run_group(*cfg, nodes, n_nodes, g.second, o, st, sts);
        if (r != ICW_OK) {
            rc = r;
            for (Job *j : g.second) if (sts[j->idx] == ICW_OK) sts[j->idx] = r;
        }
        ++st.n_groups;
    }
    for (Job &j : jobs) {
        if (j.in) fclose(j.in);
        if (j.out && fclose(j.out) != 0 && sts[j.idx] == ICW_OK) sts[j.idx] = ICW_EINVAL;
        if (sts[j.idx] == ICW_OK) ++st.n_files;
        else if (rc == ICW_OK) rc = sts[j.idx];
    }
    st.wall_s = now_s() - t0;
    if (stats) *stats = st;
    return rc;
}

}  /* extern "C" */
