/*
 * icw_group.h -- one host process driving several GPUs: a batch of streams sharded into contiguous
 * ranges, one icw_ctx per device, one host thread per device per call.  Streams are
 * independent, so there is no exchange between the devices; results are byte-identical to a
 * single context over all streams.
 *
 * Reference interfaces this serves: the reference drives one MOD_CONTEXT per decode thread
 * (playback.c:567-671, transcode.c:39-120) and has no multi-device form; a group is many
 * amod_process_samples (adv_modulator.c:587-763) decode loops at once, spread over the GPUs of a
 * node.  icw_transcode_files_devices is icw_transcode_files (icw_reader.h) over a device list.
 */
#ifndef ICW_GROUP_H_
#define ICW_GROUP_H_

#include "icw.h"
#include "icw_reader.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct icw_group icw_group;

/* n_streams streams over n_devices devices (entries may repeat: several shards on one GPU).
 * Shard d holds streams [first_d, first_d + count_d): contiguous, the first n_streams % n_devices
 * shards one stream larger (the rank split of in_cwave_amd/shard.py).  The DSP list is
 * normalised per icw_create; *accepted as there. */
int icw_group_create(const icw_config *cfg, const icw_node *nodes, int n_nodes, int n_streams,
                     const int *devices, int n_devices, icw_group **out, int *accepted);
int icw_group_destroy(icw_group *g);

/* shard d: its first stream, stream count, device and context (for per-stream calls such as
 * icw_stream_open / icw_set_state, with stream index s - first) */
int icw_group_shard(const icw_group *g, int d, int *first, int *count, int *device, icw_ctx **ctx);
/* Live edits (icw_set_graph / icw_set_render / icw_set_hilbert_filter / _config, icw.h) apply per
 * context: call them on every shard's ctx to change the whole group. */

/* icw_process_batch over the whole group with HOST pointers: stream s at in + s*in_stride, out +
 * s*out_stride (dbg: double[n_streams][n_frames][2] with ICW_F_DEBUG_PRE).  Every device's thread
 * stages and processes its shard concurrently; returns when all are done, with the first error. */
int icw_group_process(icw_group *g, const void *in, size_t in_stride, void *out, size_t out_stride,
                      int n_frames, unsigned flags, void *dbg);

/* meters / frame counter of global stream s */
int icw_group_get_meters(icw_group *g, int s, int reset, icw_meters *m);
int icw_group_n_frame(icw_group *g, int s, uint64_t *n_frame);

/* icw_transcode_files with the files split into n_devices contiguous shards, one host thread and
 * one device each (opts->device is ignored).  stats are summed over the shards (wall_s: the whole
 * call); status per file as icw_transcode_files. */
int icw_transcode_files_devices(const icw_config *cfg, const icw_node *nodes, int n_nodes,
                                const char *const *in_paths, const char *const *out_paths, int n,
                                const icw_batch_opts *opts, const int *devices, int n_devices,
                                icw_batch_stats *stats, int *status);

#ifdef __cplusplus
}
#endif
#endif /* ICW_GROUP_H_ */
