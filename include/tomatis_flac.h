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

#ifdef __cplusplus
}
#endif

#endif /* TOMATIS_FLAC_H */
