/*
 * tomatis_flac.h — C ABI of the native FLAC codec (host library
 * libtomatis_flac.so, source tomatis_audio_processor_amd/csrc/tm_flac.cpp).
 *
 * Replaces the file codec the reference reaches through libsndfile
 * (SURVEY.md §8 row f1):
 *   sf.read / sf.SoundFile(...).read    src/process_tomatis.py:225-233,
 *                                        src/layer2_apply_eq.py:88-93,
 *                                        src/process_tomatis_adaptive.py:186-190
 *        -> tomatis_flac_info + tomatis_flac_decode
 *   sf.SoundFile(out, "w", format="FLAC", subtype="PCM_24") / sf.write
 *                                        src/process_tomatis.py:243-251,
 *                                        src/layer2_apply_eq.py:215-233
 *        -> tomatis_flac_encode
 * Samples cross the ABI as interleaved int32 [frames][ch] integers of the
 * stream's bit depth; float normalisation (libsndfile's 2^(bps-1) rule) is the
 * caller's.  Synchronous, thread-safe, no global state.
 */
#ifndef TOMATIS_FLAC_H
#define TOMATIS_FLAC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TOMATIS_FLAC_OK 0
#define TOMATIS_FLAC_E_ARG (-1)     /* bad argument / sample out of range */
#define TOMATIS_FLAC_E_FORMAT (-2)  /* not FLAC / unsupported or corrupt stream */
#define TOMATIS_FLAC_E_CRC (-3)     /* frame header CRC-8 or frame CRC-16 mismatch */
#define TOMATIS_FLAC_E_NOMEM (-4)

/* Encode interleaved int32 PCM (|v| within bps bits, 4 <= bps <= 32, 1..8
 * channels) to a complete FLAC stream in *out (free with tomatis_flac_free). */
int tomatis_flac_encode(const int32_t* pcm, int64_t frames, int32_t ch, int32_t sr, int32_t bps,
                        uint8_t** out, int64_t* out_len);
void tomatis_flac_free(uint8_t* p);

/* STREAMINFO of an in-memory FLAC stream. */
int tomatis_flac_info(const uint8_t* data, int64_t len, int32_t* sr, int32_t* ch, int32_t* bps,
                      int64_t* frames);

/* Decode up to max_frames frames into pcm [max_frames][ch] (int32, stream bit
 * depth); *frames_out = frames written.  CRCs are verified.  pcm == NULL with
 * max_frames == 0 counts: *frames_out = the stream's decoded length (for
 * streams whose STREAMINFO total is 0, "unknown").  Bytes after the last
 * frame that do not start a verified frame (an ID3v1 tag) end the stream. */
int tomatis_flac_decode(const uint8_t* data, int64_t len, int32_t* pcm, int64_t max_frames,
                        int64_t* frames_out);

/* Streaming encoder (the output side of a file pipeline: segments of PCM are
 * pushed as they arrive from the device and encoded on host threads while the
 * next segment is in flight).  Every push but the last must hold a multiple of
 * 4096 frames; finish returns the complete stream (free with
 * tomatis_flac_free), byte-identical to tomatis_flac_encode of the whole PCM. */
typedef struct tomatis_flac_enc_s* tomatis_flac_enc_t;
int tomatis_flac_enc_open(int32_t ch, int32_t sr, int32_t bps, tomatis_flac_enc_t* out);
int tomatis_flac_enc_push(tomatis_flac_enc_t enc, const int32_t* pcm, int64_t frames);
int tomatis_flac_enc_finish(tomatis_flac_enc_t enc, uint8_t** out, int64_t* out_len);
/* Streaming to a file: take (and drop) the frame bytes encoded so far (free
 * with tomatis_flac_free); at the end write the 42-byte header from
 * tomatis_flac_enc_header over a 42-byte placeholder at offset 0. */
int tomatis_flac_enc_take(tomatis_flac_enc_t enc, uint8_t** out, int64_t* out_len);
int tomatis_flac_enc_header(tomatis_flac_enc_t enc, uint8_t* hdr42);
void tomatis_flac_enc_close(tomatis_flac_enc_t enc);

/* Byte offset of the first audio frame (after the metadata blocks), or -1. */
int64_t tomatis_flac_first_frame(const uint8_t* data, int64_t len);

/* Decode the frames whose first byte lies in [lo, hi) into pcm at their own
 * sample offsets (pcm holds the whole stream, [max_frames][ch]); [*s_lo, *s_hi)
 * = the samples written.  Consecutive byte ranges give consecutive sample
 * ranges: the input side of a file pipeline uploads each range while the next
 * one decodes. */
int tomatis_flac_decode_bytes(const uint8_t* data, int64_t len, int64_t lo, int64_t hi,
                              int32_t* pcm, int64_t max_frames, int64_t* s_lo, int64_t* s_hi);

#ifdef __cplusplus
}
#endif

#endif /* TOMATIS_FLAC_H */
