/*
 * icw_group.cpp -- several GPUs from one host process (include/icw_group.h): contiguous stream
 * shards, one icw_ctx per device, one host thread per device per call.  No data moves between the
 * devices: the streams are independent.
 */
#include <chrono>
#include <cstring>
#include <memory>
#include <new>
#include <thread>
#include <vector>

#include "../../include/icw_group.h"

struct icw_group {
    struct Shard {
        int first = 0, count = 0, device = -1;
        icw_ctx *ctx = nullptr;
    };
    std::vector<Shard> shards;
    int n_streams = 0;
};

namespace {

/* the rank split of in_cwave_amd/shard.py: contiguous, the first n % k shards one larger */
void split(int n, int k, int d, int &first, int &count)
{
    const int base = n / k, extra = n % k;
    first = d * base + (d < extra ? d : extra);
    count = base + (d < extra ? 1 : 0);
}

const icw_group::Shard *owner(const icw_group *g, int s)
{
    for (const auto &sh : g->shards)
        if (s >= sh.first && s < sh.first + sh.count) return &sh;
    return nullptr;
}

/* run f(d) for every shard on its own thread; the first nonzero status wins */
template <class F>
int each_shard(size_t n, F f)
{
    std::vector<int> rc(n, ICW_OK);
    std::vector<std::thread> th;
    th.reserve(n);
    for (size_t d = 0; d < n; ++d) th.emplace_back([&, d] { rc[d] = f(d); });
    for (auto &t : th) t.join();
    for (int r : rc)
        if (r != ICW_OK) return r;
    return ICW_OK;
}

double now_s()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

extern "C" {

int icw_group_create(const icw_config *cfg, const icw_node *nodes, int n_nodes, int n_streams,
                     const int *devices, int n_devices, icw_group **out, int *accepted)
{
    if (!cfg || !out || !devices || n_devices <= 0 || n_streams < n_devices) return ICW_EINVAL;
    *out = nullptr;
    std::unique_ptr<icw_group> g(new (std::nothrow) icw_group);
    if (!g) return ICW_ENOMEM;
    g->n_streams = n_streams;
    g->shards.resize((size_t)n_devices);
    int acc_all = 1;
    for (int d = 0; d < n_devices; ++d) {
        auto &sh = g->shards[(size_t)d];
        split(n_streams, n_devices, d, sh.first, sh.count);
        sh.device = devices[d];
        int acc = 0;
        const int rc = icw_create(cfg, nodes, n_nodes, sh.count, sh.device, &sh.ctx, &acc);
        if (rc != ICW_OK) {
            icw_group_destroy(g.release());
            return rc;
        }
        acc_all &= acc;
    }
    if (accepted) *accepted = acc_all;
    *out = g.release();
    return ICW_OK;
}

int icw_group_destroy(icw_group *g)
{
    if (!g) return ICW_EINVAL;
    int rc = ICW_OK;
    for (auto &sh : g->shards)
        if (sh.ctx) {
            const int r = icw_destroy(sh.ctx);
            if (rc == ICW_OK) rc = r;
        }
    delete g;
    return rc;
}

int icw_group_shard(const icw_group *g, int d, int *first, int *count, int *device, icw_ctx **ctx)
{
    if (!g || d < 0 || d >= (int)g->shards.size()) return ICW_EINVAL;
    const auto &sh = g->shards[(size_t)d];
    if (first) *first = sh.first;
    if (count) *count = sh.count;
    if (device) *device = sh.device;
    if (ctx) *ctx = sh.ctx;
    return ICW_OK;
}

int icw_group_process(icw_group *g, const void *in, size_t in_stride, void *out, size_t out_stride,
                      int n_frames, unsigned flags, void *dbg)
{
    if (!g || !in || !out || n_frames < 0) return ICW_EINVAL;
    if (flags & ICW_F_DEVICE_PTRS) return ICW_EINVAL;     /* host pointers: each shard stages its rows */
    if ((flags & ICW_F_DEBUG_PRE) && !dbg) return ICW_EINVAL;
    return each_shard(g->shards.size(), [&](size_t d) {
        const auto &sh = g->shards[d];
        const char *i = (const char *)in + (size_t)sh.first * in_stride;
        char *o = (char *)out + (size_t)sh.first * out_stride;
        double *p = (flags & ICW_F_DEBUG_PRE) ? (double *)dbg + (size_t)sh.first * (size_t)n_frames * 2 : nullptr;
        return icw_process_streams(sh.ctx, 0, sh.count, i, in_stride, o, out_stride, n_frames, flags, p, nullptr);
    });
}

int icw_group_get_meters(icw_group *g, int s, int reset, icw_meters *m)
{
    const icw_group::Shard *sh = g ? owner(g, s) : nullptr;
    if (!sh) return ICW_EINVAL;
    return icw_get_meters(sh->ctx, s - sh->first, reset, m);
}

int icw_group_n_frame(icw_group *g, int s, uint64_t *n_frame)
{
    const icw_group::Shard *sh = g ? owner(g, s) : nullptr;
    if (!sh) return ICW_EINVAL;
    return icw_n_frame(sh->ctx, s - sh->first, n_frame);
}

int icw_transcode_files_devices(const icw_config *cfg, const icw_node *nodes, int n_nodes,
                                const char *const *in_paths, const char *const *out_paths, int n,
                                const icw_batch_opts *opts, const int *devices, int n_devices,
                                icw_batch_stats *stats, int *status)
{
    if (!cfg || n < 0 || !devices || n_devices <= 0 || (n > 0 && (!in_paths || !out_paths))) return ICW_EINVAL;
    const double t0 = now_s();
    const int k = n < n_devices ? (n > 0 ? n : 1) : n_devices;
    std::vector<icw_batch_stats> st((size_t)k);
    std::vector<int> stat_local(n > 0 ? (size_t)n : 1, ICW_OK);
    int *sts = status ? status : stat_local.data();
    const int rc = each_shard((size_t)k, [&](size_t d) {
        int first, count;
        split(n, k, (int)d, first, count);
        memset(&st[d], 0, sizeof(st[d]));
        if (count == 0) return ICW_OK;
        icw_batch_opts o;
        memset(&o, 0, sizeof(o));
        if (opts) o = *opts;
        o.device = devices[d];
        return icw_transcode_files(cfg, nodes, n_nodes, in_paths + first, out_paths + first, count, &o, &st[d],
                                   sts + first);
    });
    if (stats) {
        icw_batch_stats s;
        memset(&s, 0, sizeof(s));
        for (const auto &x : st) {
            s.n_files += x.n_files;
            s.n_groups += x.n_groups;
            s.frames_in += x.frames_in;
            s.frames_out += x.frames_out;
            s.io_s += x.io_s;
        }
        s.wall_s = now_s() - t0;
        *stats = s;
    }
    return rc;
}

}  /* extern "C" */
