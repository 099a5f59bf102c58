/*
 * icw_reader.h -- file-side ingestion: the reference's WAV / CWAVE header acceptance rules and a
 * batched transcoder that streams many files through the GPU path with pinned, double-buffered
 * host staging (the many-file form of the reference's transcode.c loop).
 *
 * Reference interfaces replaced (file:line into the reference tree):
 *   icw_wav_parse_file   <- xwave_reader_create (xwave_reader.c:593-700): extension check
 *                           (check_file_ext, xwave_reader.c:118-131), rwave_reader_create
 *                           (xwave_reader.c:362-585) / cwave_reader_create (xwave_reader.c:243-339),
 *                           the MAX_FS_SRC check (xwave_reader.c:672-674)
 *   icw_transcode_files  <- winampGetExtendedRead_open / _getData / _close (transcode.c:39-120)
 *                           driving amod_process_samples per block, for n files at once: each file
 *                           is one stream of a context; the output is the 2-channel 16/24-bit PCM
 *                           the transcoder returns, written as a WAV file
 */
#ifndef ICW_READER_H_
#define ICW_READER_H_

#include "icw.h"

#ifdef __cplusplus
extern "C" {
#endif

/* header type of a RIFF/WAVE file (HRW_HTYPE_*, in_cwave.h) */
#define ICW_HTYPE_WFONLY 0      /* WAVEFORMAT only: bits per sample derived from nBlockAlign */
#define ICW_HTYPE_PCMW   1      /* PCMWAVEFORMAT / WAVE_FORMAT_IEEE_FLOAT */
#define ICW_HTYPE_EXT    2      /* WAVEFORMATEXTENSIBLE */
#define ICW_HTYPE_CWAVE  3      /* a CWAVE file */

typedef struct icw_wav_info {
    uint32_t fmt;               /* ICW_FMT_* (ICW_FMT_CW_* for CWAVE) */
    uint32_t channels;          /* 1 or 2 */
    uint32_t sample_rate;
    uint32_t frame_bytes;       /* bytes per frame in the file */
    int64_t  n_samples;         /* frames in the data part */
    int64_t  data_offset;       /* byte offset of the data part */
    uint32_t htype;             /* ICW_HTYPE_* */
    uint32_t reserved_;
} icw_wav_info;

/* Open `path` the way xwave_reader_create does: the extension selects the reader (".wav" and
 * ".rwave" -> RIFF/WAVE, ".cwave" -> CWAVE; case-insensitive), then the header must pass the
 * reference's checks.  Returns ICW_OK and fills *info, or ICW_EINVAL for a file the reference
 * would refuse (ICW_ENOMEM / ICW_EDEVICE never; I/O errors read as refusals). */
int icw_wav_parse_file(const char *path, icw_wav_info *info);

typedef struct icw_batch_opts {
    uint32_t fade_in_ms, fade_out_ms;   /* FADE_IN / FADE_OUT */
    uint32_t sec_align;                 /* SEC_ALIGN: virtual zero tail to a multiple of it, s */
    int32_t  block_frames;              /* frames per stream per GPU block (0: 65536) */
    int32_t  device;                    /* HIP device, -1: current */
    int32_t  reserved_;
} icw_batch_opts;

typedef struct icw_batch_stats {
    int32_t  n_files, n_groups;         /* files transcoded; contexts used (one per input format) */
    uint64_t frames_in, frames_out;     /* data frames read; frames written (tails included) */
    double   wall_s;                    /* whole call */
    double   io_s;                      /* host time spent reading and writing files */
} icw_batch_stats;

/* Transcode n files: in_paths[i] -> out_paths[i] (a 2-channel PCM WAV, 16 or 24 bit per
 * cfg->need24bits), every file a fresh stream (mod_context_init state) with its own fades and
 * tail.  Files are grouped by (sample rate, format, channels); each group is one context whose
 * streams advance together block by block while the host reads the next block and writes the
 * previous one (pinned buffers, a copy stream, HIP events).  status (nullable, n entries) gets
 * ICW_OK or the file's error.  Returns ICW_OK if every file was transcoded. */
int icw_transcode_files(const icw_config *cfg, const icw_node *nodes, int n_nodes, const char *const *in_paths,
                        const char *const *out_paths, int n, const icw_batch_opts *opts, icw_batch_stats *stats,
                        int *status);

#ifdef __cplusplus
}
#endif
#endif /* ICW_READER_H_ */
