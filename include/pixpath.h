/*
 * pixpath.h -- C ABI of libpixpath.so, the MI355X (gfx950) raw-frame pixel path
 * behind pnats2avhd/processing-chain's command builders (lib/ffmpeg.py) and SRC
 * analysis hooks (util/SRC_analysis.py, util/complexity_classification.py).
 *
 * Plain C types only: device pointers, byte strides, sizes, an opaque context.
 * Every entry point returns PP_OK (0) or a negative PP_ERR_* code; the message
 * of the last failure is available from pp_last_error() (thread-local).
 * Kernels are enqueued on the caller's HIP stream (`stream`, a hipStream_t
 * passed as void*; NULL = the null stream) and never synchronise it.
 * A context is bound to one device and is not thread-safe (one per process,
 * matching the one-process-per-GPU model of SURVEY.md section 8e).
 *
 * Which reference interface each entry point replaces is given per function as
 * reference file:line.  The reference reaches all of these through ffmpeg
 * command strings; the strings are reproduced by the Python host
 * (processing-chain_amd/pixpath/ffmpeg.py), which calls this library.
 */
#ifndef PIXPATH_H
#define PIXPATH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PP_ABI_VERSION 7

/* return codes */
#define PP_OK 0
#define PP_ERR_INVALID -1     /* bad argument / unsupported combination */
#define PP_ERR_HIP -2         /* HIP runtime failure */
#define PP_ERR_NOMEM -3
#define PP_ERR_UNSUPPORTED -4

/* pixel formats (ffmpeg -pix_fmt names in comments) */
enum pp_pix_fmt {
    PP_FMT_YUV420P = 0,      /* yuv420p */
    PP_FMT_YUV422P = 1,      /* yuv422p */
    PP_FMT_YUV444P = 2,      /* yuv444p */
    PP_FMT_YUV420P10LE = 3,  /* yuv420p10le */
    PP_FMT_YUV422P10LE = 4,  /* yuv422p10le */
    PP_FMT_YUV444P10LE = 5,  /* yuv444p10le */
    PP_FMT_UYVY422 = 6,      /* uyvy422 (packed, 1 plane) */
    PP_FMT_V210 = 7          /* -c:v v210 payload (packed, 1 plane) */
};

/* swscale flag values (same bits as FFmpeg's SWS_*) */
#define PP_SWS_BILINEAR 0x2
#define PP_SWS_BICUBIC 0x4
#define PP_SWS_LANCZOS 0x200
#define PP_SWS_PARAM_DEFAULT 123456.0
/* ABI v5: plan flag selecting the general scale_kernel even where the strip
 * kernel applies (both are bit-exact; tests run every plan through both). */
#define PP_PLAN_GENERIC 0x10000000

/*
 * A batch of `nframes` frames.  Plane p of frame f starts at
 * data[p] + f * frame_stride[p]; rows are linesize[p] bytes apart.
 * Packed formats use plane 0 only.  Every row of a plane, the last one
 * included, must be readable for min(linesize, width rounded up to 16 bytes)
 * bytes: with 16-byte aligned pointers and linesizes the kernels read whole
 * 16-byte granules (a plane allocated as height x linesize always qualifies).
 */
typedef struct pp_frames {
    void *data[3];
    int64_t linesize[3];
    int64_t frame_stride[3];
} pp_frames;

typedef struct pp_ctx pp_ctx;
typedef struct pp_scale_plan pp_scale_plan;

/* ---- library / context ------------------------------------------------- */
int pp_abi_version(void);
const char *pp_last_error(void);
/* Select `device` and create a context.  Replaces nothing in the reference
 * (the reference runs CPU processes, lib/cmd_utils.py:93-101). */
int pp_ctx_create(int device, pp_ctx **out);
int pp_ctx_destroy(pp_ctx *ctx);

/* Byte size of one plane of one frame and the v210 line size (v210enc.c:
 * ceil(w/48)*48*8/3). */
int64_t pp_plane_bytes(int fmt, int w, int h, int plane, int64_t linesize);
int64_t pp_v210_linesize(int w);

/* ---- scaling / format conversion (libswscale restatement) --------------
 * Replaces `scale=W:H:flags=bicubic` at lib/ffmpeg.py:992 (create_avpvs_short),
 * :1038 (create_avpvs_segment), :1213 (create_cpvs mobile), `scale=W:-2` at
 * :800 (encode_segment) and the implicit `-pix_fmt` conversions at :994, :1048,
 * :1198.  flags: PP_SWS_BICUBIC | PP_SWS_LANCZOS | PP_SWS_BILINEAR; param0/1 as
 * FFmpeg's sws param[0]/[1] (PP_SWS_PARAM_DEFAULT = FFmpeg default).
 * dst_fmt may be planar YUV or PP_FMT_UYVY422 (packed output path).
 * Coefficient tables are built on the host once per plan and kept in HBM.
 * ctx == NULL builds a host-only plan (filter introspection, no execution). */
int pp_scale_plan_create(pp_ctx *ctx, int src_fmt, int src_w, int src_h,
                         int dst_fmt, int dst_w, int dst_h, int flags,
                         double param0, double param1, pp_scale_plan **out);
int pp_scale_plan_destroy(pp_scale_plan *plan);
/* Introspection for parity tests: which = 0 luma-H, 1 chroma-H, 2 luma-V,
 * 3 chroma-V.  Copies the FFmpeg-layout filter (before device compaction):
 * coef[n * size] int16, pos[n] int32 on the host.  Returns size (>0),
 * 0 when the plan uses an unscaled converter, or <0. */
int pp_scale_plan_filter(const pp_scale_plan *plan, int which, int16_t *coef,
                         int32_t *pos, int capacity);
/* Kernel the plan runs for 16-B aligned sources: > 0 = the strip kernel's
 * horizontal window in dwords (the common case), 0 = the general kernel
 * (narrow strips / long vertical filters / unscaled converters).  The
 * environment variable PIXPATH_SCALE_KERNEL=generic at plan creation forces 0
 * (parity tests run both kernels on the same cases). */
int pp_scale_plan_path(const pp_scale_plan *plan);
/* Launch geometry of the plan for measurement and documentation: fills up to
 * n of {LDS bytes per workgroup, threads per workgroup, workgroups per frame,
 * luma chunk rows, luma segment rows, luma V tap pairs, chroma V tap pairs,
 * luma staged columns, luma window rows, luma max new rows per chunk}.
 * Returns the number of values written. */
int pp_scale_plan_stats(const pp_scale_plan *plan, int64_t *out, int n);
/* The two-stage chain of create_avpvs_segment (lib/ffmpeg.py:1037-1048):
 * `scale=W:H:flags=...` into the overlay's yuv420p, then libavfilter's
 * auto-inserted yuv420p -> dst_fmt conversion at the same size (bicubic).
 * Executed with pp_scale_execute; bit-exact with running the two plans one
 * after the other.  When the first stage is a strip plan
 * (pp_scale_plan_path > 0) both stages run in ONE kernel launch with no
 * intermediate in HBM; otherwise two launches through a plan-owned yuv420p
 * scratch batch (so such a plan serves one stream at a time).
 * dst_fmt: yuv420p (one stage), yuv422p, yuv420p10le, yuv422p10le. */
int pp_scale_chain_plan_create(pp_ctx *ctx, int src_fmt, int src_w, int src_h,
                               int dst_fmt, int dst_w, int dst_h, int flags,
                               double param0, double param1, pp_scale_plan **out);
/* Run the plan on `nframes` device frames. */
int pp_scale_execute(pp_scale_plan *plan, const pp_frames *src,
                     const pp_frames *dst, int nframes, void *stream);

/* ---- padding -----------------------------------------------------------
 * Replaces `pad=width=DW:height=DH:x=(ow-iw)/2:y=(oh-ih)/2` at
 * lib/ffmpeg.py:1183 (create_cpvs PC) and :1209 (tablet).  Black is
 * Y 16 / C 128 scaled to the bit depth; x/y are rounded down to the chroma
 * grid.  Pass x = y = -1 for the reference's centring expression. */
int pp_pad_execute(pp_ctx *ctx, int fmt, int src_w, int src_h,
                   const pp_frames *src, int dst_w, int dst_h, int x, int y,
                   const pp_frames *dst, int nframes, void *stream);

/* ---- CPVS packers ------------------------------------------------------
 * `-c:v v210 -pix_fmt yuv422p10le` (lib/test_config.py:208-215 via
 * lib/ffmpeg.py:1198): pack yuv422p10le into v210 (libavcodec/v210enc.c);
 * dst plane 0 with linesize >= pp_v210_linesize(w). */
int pp_v210_pack(pp_ctx *ctx, int w, int h, const pp_frames *src,
                 const pp_frames *dst, int nframes, void *stream);

/* Fused PC CPVS: `fps,pad=W:H:(ow-iw)/2:(oh-ih)/2` + `-pix_fmt` conversion +
 * packing in one pass (lib/ffmpeg.py:1177-1201).  src: AVPVS frames (w x h,
 * yuv420p/yuv422p for out_fmt PP_FMT_UYVY422, yuv420p10le/yuv422p10le for
 * PP_FMT_V210); canvas W x H with the input at (x, y) (-1 = centred, rounded
 * to the chroma grid); dst plane 0, 16-B aligned.  Bit-identical to pad ->
 * swscale (bicubic) -> packer. */
int pp_cpvs_execute(pp_ctx *ctx, int src_fmt, int w, int h, const pp_frames *src,
                    int W, int H, int x, int y, int out_fmt,
                    const pp_frames *dst, int nframes, void *stream);

/* ---- stall compositing (spec PP-STALL-1) -----------------
 * Replaces the external `bufferer -s spinner.png` call at
 * p03_generateAvPvs.py:236-243.  Uploads one spinner animation (n RGBA8
 * frames of sw x sh, host memory) converted for `fmt`. */
int pp_spinner_upload(pp_ctx *ctx, int fmt, const uint8_t *rgba, int n,
                      int sw, int sh);
/* For each output frame k: dst[k] = src[src_index[k]] (or black when
 * src_index[k] < 0) with spinner frame spinner_index[k] composited centred
 * (no overlay when spinner_index[k] < 0).  Index arrays are host memory. */
int pp_stall_compose(pp_ctx *ctx, int fmt, int w, int h, const pp_frames *src,
                     const int32_t *src_index, const int32_t *spinner_index,
                     const pp_frames *dst, int nframes, void *stream);

/* ---- P.910 SI/TI (spec PP-SITI-1) ------------------------
 * New feature behind util/SRC_analysis.py:120-147 (analyse_src) and
 * util/complexity_classification.py:50-69 (get_difficulty).
 * luma: nframes frames of w x h, 8- or 10-bit (uint16 LE), linesize and
 * frame_stride in bytes.  prev: the frame before luma[0] (1-frame halo) or
 * NULL.  si/ti: DEVICE arrays of nframes doubles; ti[0] is NaN without prev. */
int pp_siti(pp_ctx *ctx, int bitdepth, int w, int h, const void *luma,
            int64_t linesize, int64_t frame_stride, int nframes,
            const void *prev, double *si, double *ti, void *stream);
/* pp_siti with flags: PP_SITI_NORMALIZE divides SI_n and TI_n by
 * 2^(bitdepth-8) (SURVEY.md 8a-13's optional normalisation), so 8- and 10-bit
 * SRCs report on the 8-bit scale; an exact power-of-two scaling of the raw
 * values.  pp_siti(...) == pp_siti_ex(..., 0, stream). */
#define PP_SITI_NORMALIZE 1
int pp_siti_ex(pp_ctx *ctx, int bitdepth, int w, int h, const void *luma,
               int64_t linesize, int64_t frame_stride, int nframes,
               const void *prev, double *si, double *ti, int flags, void *stream);

/* ---- host helpers --------------------------------------------------------
 * vf_fps output->input frame map (lib/ffmpeg.py:832-834, :959-961, :1038,
 * :1179): map[k] = input frame shown at output frame k.  Returns the number of
 * output frames (<= capacity) or <0. */
int pp_fps_map(int n_in, int64_t in_num, int64_t in_den, int64_t out_num,
               int64_t out_den, int32_t *map, int capacity);

/* ---- host transfer: device / pinned host memory, streams, events, copies --
 * SURVEY.md 8(b) "pinned host alloc + async H2D/D2H on caller-supplied
 * streams": everything a host without torch needs between ffmpeg's decode
 * pipe and its encode pipe (the reference hands frames between decoder,
 * filter graph and encoder inside one ffmpeg process, lib/ffmpeg.py:992-998).
 * Streams and events are hipStream_t / hipEvent_t passed as void*.  The
 * caller owns every buffer it allocates here and frees it with the matching
 * call. */
#define PP_COPY_H2D 1
#define PP_COPY_D2H 2
#define PP_COPY_D2D 3
int pp_device_alloc(pp_ctx *ctx, int64_t bytes, void **out);
int pp_device_free(pp_ctx *ctx, void *ptr);
int pp_host_alloc(int64_t bytes, void **out);   /* page-locked (pinned) */
int pp_host_free(void *ptr);
int pp_stream_create(pp_ctx *ctx, void **out);  /* non-blocking stream */
int pp_stream_destroy(pp_ctx *ctx, void *stream);
int pp_stream_synchronize(void *stream);
int pp_event_create(pp_ctx *ctx, void **out);
int pp_event_destroy(void *event);
int pp_event_record(void *event, void *stream);
int pp_stream_wait_event(void *stream, void *event);
int pp_event_synchronize(void *event);
int pp_event_elapsed_ms(void *start, void *end, float *ms);
/* `bytes` contiguous bytes; kind PP_COPY_*. */
int pp_copy_async(void *dst, const void *src, int64_t bytes, int kind, void *stream);
/* `rows` rows of `width_bytes`, pitches in bytes. */
int pp_copy2d_async(void *dst, int64_t dpitch, const void *src, int64_t spitch,
                    int64_t width_bytes, int64_t rows, int kind, void *stream);
/* All planes of `nframes` w x h frames of `fmt` between two pp_frames layouts
 * (e.g. a dense pinned host batch and a pitched device batch). */
int pp_frames_copy_async(int fmt, int w, int h, const pp_frames *dst,
                         const pp_frames *src, int nframes, int kind, void *stream);

/* ---- p02 byte scanners (host only, no device work) -----------------------
 * Per-frame sizes of a bitstream held in host memory, exactly as
 * lib/get_framesize.py computes them, quirks included (see csrc/scan.cpp).
 * Return the number of frames (sizes[] receives the first `cap` of them) or
 * a negative PP_ERR_*.  pp_annexb_frame_sizes replaces the byte loops of
 * get_framesize_h264 (lib/get_framesize.py:144-201, PP_NAL_H264) and
 * get_framesize_h265 (:204-263, PP_NAL_H265) over the *_tmp.h264/.h265 file;
 * an H.264 NAL header on which the reference raises ValueError (hex digit
 * a..f, :180) returns PP_ERR_INVALID.  pp_ivf_frame_sizes replaces
 * get_framesize_vp9's IVF walk (:87-141); *misdetected counts the frames whose
 * header fails the "10" frame-marker test (the reference prints a line each). */
#define PP_NAL_H264 1
#define PP_NAL_H265 2
int64_t pp_annexb_frame_sizes(const uint8_t *buf, int64_t n, int codec, int64_t *sizes, int64_t cap);
int64_t pp_ivf_frame_sizes(const uint8_t *buf, int64_t n, int64_t *sizes, int64_t cap, int64_t *misdetected);

/* ---- FFV1 AVPVS encoder -----------------------
 * Replaces the `-c:v ffv1 -level 3 -coder 1 -context 1 -slicecrc 1` encode of
 * the AVPVS (lib/ffmpeg.py:993, :1047): FFV1 version 3 (RFC 9043), range
 * coder, slice CRCs, every frame a keyframe, one 3-input quantisation set
 * (63 contexts at 10 bits, 172 at 8), slices_h x slices_v slices per
 * frame (<= 256), one GPU lane per slice.  Bitstream choices and the parity
 * status (unpinned: no FFV1 decoder exists here) are in DESIGN.md.
 * pp_ffv1_encoder_create with ctx == NULL builds the configuration record only.
 * pp_ffv1_extradata copies the configuration record (AVI/MKV codec private
 * data) and returns its size (cap 0: size only).
 * pp_ffv1_encode encodes nframes <= max_frames device frames into frame
 * packets laid out back to back in the device buffer dst (frame_sizes[f] on
 * the host); it synchronises `stream` and returns the total bytes or < 0. */
typedef struct pp_ffv1_enc pp_ffv1_enc;
int pp_ffv1_encoder_create(pp_ctx *ctx, int fmt, int w, int h, int slices_h, int slices_v,
                           int max_frames, pp_ffv1_enc **out);
int pp_ffv1_encoder_destroy(pp_ffv1_enc *enc);
int pp_ffv1_extradata(const pp_ffv1_enc *enc, uint8_t *out, int cap);
int64_t pp_ffv1_encode(pp_ffv1_enc *enc, const pp_frames *src, int nframes, uint8_t *dst,
                       int64_t dst_cap, int64_t *frame_sizes, void *stream);
/* ABI v5.  pp_ffv1_encode_packets: the same encode into the encoder's own
 * device packet buffer (grown as needed, kept across calls); *packets points
 * at the packets back to back, valid until the next encode; returns the total
 * bytes.  The encoder sizes its per-slice renorm records for content coding at
 * 2:1 or better and re-codes a batch in halves when a slice needs more, so
 * the packets never depend on that sizing (pp_ffv1_encode_stats: launches of
 * the last encode, 1 unless it was split).  pp_ffv1_encoder_memory: device
 * bytes the encoder holds. */
int64_t pp_ffv1_encode_packets(pp_ffv1_enc *enc, const pp_frames *src, int nframes, int64_t *frame_sizes,
                               const uint8_t **packets, void *stream);
int pp_ffv1_encode_stats(const pp_ffv1_enc *enc, int *launches);
/* Grow the encoder's packet buffer to `packet_bytes` now (a writer process
 * sizes it once, before its first PVS, instead of inside the first encode). */
int pp_ffv1_encoder_reserve(pp_ffv1_enc *enc, int64_t packet_bytes);
int pp_ffv1_encoder_memory(const pp_ffv1_enc *enc, int64_t *bytes);
/* FFV1 decoder (the CPVS stage reads the AVPVS back, lib/ffmpeg.py:1149):
 * version 3 streams with the range coder (default or transmitted state
 * table), up to 8 quantisation table sets of up to 5 inputs, initial context
 * states, intra or inter frames (a GOP's context states carry from frame to
 * frame), with or without slice CRCs, <= 256 slices, 8/10-bit 4:2:0 / 4:2:2 /
 * 4:4:4 YCbCr -- what pp_ffv1_encode writes and what `ffmpeg -c:v ffv1 -level 3
 * -coder 1 -context 1 -slicecrc 1` writes (RFC 9043).  pp_ffv1_decoder_create
 * parses and checks the configuration record (ctx == NULL: record check
 * only); pp_ffv1_decoder_format gives the PP_FMT_* of the decoded frames;
 * pp_ffv1_decode decodes nframes consecutive packets of the stream held back
 * to back in HOST memory (frame_sizes[f] bytes each) into dst (device),
 * checking every slice's CRC, header and end position; synchronises
 * `stream`.  ABI v6: a decode whose first frame is not a keyframe continues
 * the GOP of the previous successful decode's last frame (its context states
 * are kept); pp_ffv1_decoder_reset forgets them (after a seek), and such a
 * decode then fails. */
typedef struct pp_ffv1_dec pp_ffv1_dec;
int pp_ffv1_decoder_create(pp_ctx *ctx, const uint8_t *extradata, int extradata_size, int w, int h,
                           int max_frames, pp_ffv1_dec **out);
int pp_ffv1_decoder_destroy(pp_ffv1_dec *dec);
int pp_ffv1_decoder_format(const pp_ffv1_dec *dec);
/* The slice grid of the stream (configuration record num_h/v_slices). */
int pp_ffv1_decoder_slices(const pp_ffv1_dec *dec, int *slices_h, int *slices_v);
int pp_ffv1_decode(pp_ffv1_dec *dec, const uint8_t *packets, const int64_t *frame_sizes, int nframes,
                   const pp_frames *dst, void *stream);
/* ABI v6.  The record as parsed: up to n of micro_version, coder_type,
 * quantisation table sets, largest context count, intra, ec, bit mask of the
 * sets with transmitted initial states, 1 if the tables are of pixpath's
 * form (one 3-input set: one threshold quantiser at scales 1, L, L^2 -- what
 * pp_ffv1_encode writes: 63 contexts at 10 bits, 172 at 8; round-4 files: 666),
 * decoded by the one-line-row path; returns the count written. */
int pp_ffv1_decoder_info(const pp_ffv1_dec *dec, int *info, int n);
int pp_ffv1_decoder_reset(pp_ffv1_dec *dec);
int pp_ffv1_decoder_geometry(const pp_ffv1_dec *dec, int *slices_per_workgroup, int *row_cap);
/* ABI v7.  One launch over n streams of ONE configuration record (equal
 * extradata, size and context): decs[k] decodes stream k -- nframes[k]
 * packets back to back in host memory at packets[k], sizes frame_sizes[k] --
 * into dst frames [nframes[0] + ... + nframes[k-1], ...) of the one device
 * batch dst, each stream continuing / keeping its own carried GOP states as
 * pp_ffv1_decode does.  The slice chains of an FFmpeg-made AVPVS are few
 * (GOP 12 at 2x2 slices: 200 per 600 frames, one lane each); several
 * streams' chains side by side are what fill the SIMDs -- the reference's
 * ParallelRunner feeds the CPVS stage several PVSes at once
 * (lib/cmd_utils.py:93-101).  decs[0] holds the launch workspace; the
 * decoders' workspaces grow on demand to what a call needs.  Synchronises
 * `stream`; on a slice error the message names the stream. */
int pp_ffv1_decode_group(pp_ffv1_dec *const *decs, int n, const uint8_t *const *packets,
                         const int64_t *const *frame_sizes, const int *nframes, const pp_frames *dst, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* PIXPATH_H */
